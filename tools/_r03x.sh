# round 3 (x): + host waits for k_khist verdict (no tail behind a sure failure), sample-line long-group check, walk scan reverted
# inside the segmented plan, one-block walk candidate scan -- GPU suite + c3/c5 A/B vs HEAD
O=gpurun_out/r03_x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in new head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  for c in c3 c5; do
    SMX_LIB=$L timeout -k 10 200 python -u bench.py --config $c --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/${c}_${v}_$r.json 2> $O/${c}_$v.err || { tail -5 $O/${c}_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$O/${c}_${v}_$r.json'));print('$c $v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['async_api'].get('ms_per_step'), d['stages_ms_per_step'])"
  done
done; done
