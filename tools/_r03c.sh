set -o pipefail
O=gpurun_out/r03_c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_rel.log 2>&1; rc=$?; tail -3 $O/tests_rel.log; [ $rc -eq 0 ] || exit $rc
SMX_LIB=tools/_build/var_emitvec/libsmx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread > $O/tests_emitvec.log 2>&1; rc=$?; tail -2 $O/tests_emitvec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 base=tools/_build/var_base/libsmx.so ts32=semantic_merge_amd/libsmx.so emitvec=tools/_build/var_emitvec/libsmx.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_probe.py 8 1 > $O/shard_probe.txt 2>&1; rc=$?; cat $O/shard_probe.txt; [ $rc -eq 0 ] || exit $rc
bash tools/probe_sq.sh $O/probe list ablate sq1 sq2 ta
