set -o pipefail
O=gpurun_out/r03_j; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_rga.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 out2=semantic_merge_amd/libsmx.so out2off=tools/_build/var_out2off/libsmx.so bk2off=tools/_build/var_bk2off/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
for v in new head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_head/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 python3 tools/bench_rga.py > $O/rga_$v.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }
  echo "rga $v $(cat $O/rga_$v.json)"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc --no-e2e > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-1500 $O/bench.json
