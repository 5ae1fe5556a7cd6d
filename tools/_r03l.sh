# round 3 (l): OUT2 bisect, full GPU suite on the committed default, bench with PMC, shard probe, RGA
set -o pipefail
O=gpurun_out/r03_l; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py invpass=tools/_build/var_invpass/libsmx.so out2on=tools/_build/var_out2on/libsmx.so rel=semantic_merge_amd/libsmx.so > $O/parity_libs.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity_libs.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-e2e > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-900 $O/bench.json
timeout -k 10 300 python3 -u tools/shard_probe.py 8 > $O/shard_probe.txt 2>&1; rc=$?; grep -v "amdgpu.ids\|socket.cpp" $O/shard_probe.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_rga.py > $O/bench_rga.json 2> $O/bench_rga.err || { tail -5 $O/bench_rga.err; exit 1; }
cut -c1-400 $O/bench_rga.json
for v in h16 h16off; do
  if [ $v = h16 ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_h16off/libsmx.so; fi
  for r in 1 2; do SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 python3 tools/bench_rga.py > $O/rga_${v}_$r.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }; echo "rga $v $(cat $O/rga_${v}_$r.json)"; done
done
