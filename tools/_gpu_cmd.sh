set -o pipefail
O=gpurun_out/r1s16; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
timeout -k 10 200 python tools/stage_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
