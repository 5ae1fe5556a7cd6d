set -o pipefail
O=gpurun_out/t11; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/stage_ab.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | grep -v amdgpu.ids
