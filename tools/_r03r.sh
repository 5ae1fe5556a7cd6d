# round 3 (r): RGA list kernel with one hash slot per event -- parity + A/B
set -o pipefail
O=gpurun_out/r03_r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in new ht1off; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 python3 tools/bench_rga.py > $O/rga_${v}_$r.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }; echo "rga $v $(cat $O/rga_${v}_$r.json)"
done; done
