set -o pipefail
O=gpurun_out/r03_m; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 rel=semantic_merge_amd/libsmx.so out2on=tools/_build/var_out2on/libsmx.so head=tools/_build/var_head/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
SMX_LIB=tools/_build/var_out2on/libsmx.so timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests_out2.log 2>&1; rc=$?; tail -2 $O/tests_out2.log; [ $rc -eq 0 ] || exit $rc
