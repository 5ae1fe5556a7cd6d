set -o pipefail
O=gpurun_out/r1s32; mkdir -p $O
SMX_LIB=$PWD/tools/_build/var_cur/libsmx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in head cur head cur; do
  echo "== $v"; SMX_LIB=$PWD/tools/_build/var_$v/libsmx.so timeout -k 10 200 python tools/window_phases.py 2>&1 | grep "window plain" || exit 1
done
