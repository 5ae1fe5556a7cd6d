# round 3 (ac): k_khist's long-group flag read before it is raised (first blocks only); c3 stage A/B
# with and without the host-side early verdict; c5 A/B
set -o pipefail
O=gpurun_out/r03_ac; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_compose.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/ab_libs.py --rounds 9 head=tools/_build/var_head/libsmx.so new=semantic_merge_amd/libsmx.so noearly=tools/_build/var_noearly/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in new noearly head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c5_${v}_$r.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['stages_ms_per_step'])"
done; done
