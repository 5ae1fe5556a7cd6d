# round 3 (o): XCD-ordered generic windows (config 5) -- parity + A/B
set -o pipefail
O=gpurun_out/r03_o; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_libs.py --config c5 --rounds 7 xcd=semantic_merge_amd/libsmx.so xcdoff=tools/_build/var_xcdoff/libsmx.so > $O/ab_c5.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --config c3s --n-ops 20000000 --rounds 3 xcd=semantic_merge_amd/libsmx.so xcdoff=tools/_build/var_xcdoff/libsmx.so > $O/ab_c3s.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab_c3s.txt; [ $rc -eq 0 ] || exit $rc
