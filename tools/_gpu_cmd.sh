set -o pipefail
O=gpurun_out/${TAG:-r02s}; mkdir -p $O
timeout -k 10 300 python -u bench.py --config c5 --no-pmc --no-e2e > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
cut -c1-300 $O/bench_c5.json
timeout -k 10 300 python -u bench.py --config c2 --no-pmc --no-e2e --steps 50 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
timeout -k 10 300 python -u tools/bench_rga.py > $O/bench_rga.json 2>&1 || { tail -5 $O/bench_rga.json; exit 1; }
tail -1 $O/bench_rga.json | cut -c1-300
