# round 3 (ah): bench lines (PMC + CPU legs) after the PMC child's merge count fix
set -o pipefail
O=gpurun_out/r03_ah; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --no-e2e > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
cut -c1-400 $O/bench_c5.json
