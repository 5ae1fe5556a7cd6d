set -o pipefail
TAG=${TAG:-r02k_ab13}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 200 --timeout-method thread -k c3 > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in 0 192 128 224; do
    echo -n "cus $k: "; SMX_SIDE_CUS=$k timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  done
done
