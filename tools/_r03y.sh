# round 3 (y): which plan-stage check costs config 3 its ~7 us (stage A/B in one process)
set -o pipefail
O=gpurun_out/r03_y; mkdir -p $O
timeout -k 10 500 python -u tools/ab_libs.py --rounds 7 head=tools/_build/var_head/libsmx.so new=semantic_merge_amd/libsmx.so nofp=tools/_build/var_nofp/libsmx.so nokh=tools/_build/var_nokh/libsmx.so nocs=tools/_build/var_nocs/libsmx.so none=tools/_build/var_none/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; exit $rc
