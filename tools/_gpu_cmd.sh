set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -2 $O/tests.log
