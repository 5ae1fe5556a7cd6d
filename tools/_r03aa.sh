# round 3 (aa): step 2's merge-path search in fixed predicated steps -- parity + stage A/B
set -o pipefail
O=gpurun_out/r03_aa; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py new=semantic_merge_amd/libsmx.so > $O/parity.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/ab_libs.py --rounds 7 head=tools/_build/var_head/libsmx.so new=semantic_merge_amd/libsmx.so msloop=tools/_build/var_msloop/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; exit $rc
