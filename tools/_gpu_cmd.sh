set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_async.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -25 $O/tests.log
