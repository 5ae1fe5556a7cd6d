# round 3 (af): timed steps carry events around the roofline stages only; breakdown in an untimed leg
set -o pipefail
O=gpurun_out/r03_af; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -k bench -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c3_$r.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/c3_$r.json'));print('c3', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['graph_api']['ms_per_step'], d['async_api'].get('ms_per_step'), d['stages_ms_per_step'])"
done
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python3 -c "import json,sys;d=json.load(open('$O/c5.json'));print('c5', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['graph_api']['ms_per_step'], d['stages_ms_per_step'])"
