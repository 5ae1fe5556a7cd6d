# round 3 (p): XCD order for the table reduce and the presorted windows -- parity + A/B
set -o pipefail
O=gpurun_out/r03_p; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py rel=semantic_merge_amd/libsmx.so xcdwf=tools/_build/var_xcdwf/libsmx.so > $O/parity.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_libs.py --rounds 7 rel=semantic_merge_amd/libsmx.so xcdtboff=tools/_build/var_xcdtboff/libsmx.so xcdwf=tools/_build/var_xcdwf/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
