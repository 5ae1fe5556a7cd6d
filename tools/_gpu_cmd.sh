set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; tail -2 $O/tests.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; tail -3 $O/bench.err; cat $O/bench.json
