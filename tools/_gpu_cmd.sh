set -o pipefail
O=gpurun_out/${TAG:-r02s}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo -n "c3: "; timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done
