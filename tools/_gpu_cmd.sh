set -o pipefail
O=gpurun_out/r02zn; mkdir -p $O
V=$PWD/tools/_build
SMX_LIB=$V/var_w1024/libsmx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -x -q --timeout 200 --timeout-method thread > $O/tests_w1024.log 2>&1; rc=$?; tail -2 $O/tests_w1024.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in base w1024 w1024b; do
  if [ $v = base ]; then L=$PWD/semantic_merge_amd/libsmx.so; else L=$V/var_$v/libsmx.so; fi
  echo -n "$v: "; SMX_LIB=$L timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done; done
