# round 3 (q): step-5 scan with one barrier, final order fused into the rank loop
set -o pipefail
O=gpurun_out/r03_q; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py new=tools/_build/var_new/libsmx.so > $O/parity.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_libs.py --rounds 7 rel=semantic_merge_amd/libsmx.so new=tools/_build/var_new/libsmx.so fusefin=tools/_build/var_fusefin/libsmx.so scan1=tools/_build/var_scan1/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
SMX_LIB=tools/_build/var_new/libsmx.so timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
