# round 3 (ab): fixed-step merge search, one long-group atomic per k_khist block, no meta read after
# an early verdict -- GPU suite, c3 stage A/B and c5 bench A/B vs HEAD
set -o pipefail
O=gpurun_out/r03_ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/ab_libs.py --rounds 7 head=tools/_build/var_head/libsmx.so new=semantic_merge_amd/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in new head; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c5_${v}_$r.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['stages_ms_per_step'])"
done; done
