set -o pipefail
TAG=${TAG:-r02k_final}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_compose.py -x -q --timeout 200 --timeout-method thread -k "segmented or c5 or seg3000 or groups10k" > $O/tests_seg.log 2>&1; rc=$?; tail -3 $O/tests_seg.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo -n "c5 bucket: "; timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/seg_ab.txt || exit 1
  echo -n "c5 bitonic: "; SMX_LIB=tools/_build/var_segbit/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/seg_ab.txt || exit 1
done
for r in 1 2; do
  echo -n "prio0: "; timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/prio_ab.txt || exit 1
  echo -n "prio1: "; SMX_SIDE_PRIO=1 timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/prio_ab.txt || exit 1
done
