# round 3 (t): host path of the synchronous merge (event pool, pinned meta readback) -- A/B on bench steps
set -o pipefail
O=gpurun_out/r03_t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in new head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/b_${v}_$r.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/b_${v}_$r.json'));print('$v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['async_api']['ms_per_step'], d['stages_ms_per_step'])"
done; done
