set -o pipefail
O=gpurun_out/r03_k; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 new=semantic_merge_amd/libsmx.so out2off=tools/_build/var_out2off/libsmx.so bz4off=tools/_build/var_bz4off/libsmx.so head=tools/_build/var_head/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env SMX_LIB=tools/_build/var_diag/libsmx.so python3 -u tools/window_ablate.py > $O/ablate.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ablate.txt; [ $rc -eq 0 ] || exit $rc
for v in new head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_head/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 python3 tools/bench_rga.py > $O/rga_$v.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }
  echo "rga $v $(cat $O/rga_$v.json)"
done
timeout -k 10 300 python3 -u tools/shard_probe.py 8 > $O/shard_probe.txt 2>&1; rc=$?; grep -v "amdgpu.ids\|socket.cpp" $O/shard_probe.txt | tail -4; [ $rc -eq 0 ] || exit $rc
