set -o pipefail
TAG=${TAG:-r02k_ab10}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo -n "c5 fields: "; timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  echo -n "c5 prev: "; SMX_LIB=tools/_build/var_prev/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done
