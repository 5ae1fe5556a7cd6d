# round 3 (v): segmented plan without the mid-merge host sync, one segsort launch, long groups flagged by k_khist, sorted kinds from the segmented sort (noskind: without) -- GPU suite + c5 A/B
set -o pipefail
O=gpurun_out/r03_v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in new noskind head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c5_${v}_$r.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/c5_${v}_$r.json'));print('$v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['async_api'].get('ms_per_step'), d['stages_ms_per_step'])"
done; done
