set -o pipefail
TAG=${TAG:-r02k_ab11}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo -n "khr4: "; timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  echo -n "khr1: "; SMX_LIB=tools/_build/var_khr1/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done
