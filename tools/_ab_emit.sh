set -o pipefail
O=gpurun_out/t15; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -4 $O/tests.log
