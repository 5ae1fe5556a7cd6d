set -o pipefail
O=gpurun_out/r1s34; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
