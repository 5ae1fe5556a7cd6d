set -o pipefail
O=gpurun_out/r02zg; mkdir -p $O
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/stage_ab.py 2>/dev/null | tail -1
