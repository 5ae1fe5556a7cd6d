set -o pipefail
O=gpurun_out/r1s30; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in cur; do
echo "== $v"
SMX_LIB=$PWD/tools/_build/var_$v/libsmx.so timeout -k 10 300 python -u tools/bench_rga.py 2> $O/rga.err | cut -c1-150 || { tail -20 $O/rga.err; exit 1; }
SMX_LIB=$PWD/tools/_build/var_$v/libsmx.so timeout -k 10 300 python tools/stage_ab.py 20000000 c5 2>&1 | grep -v amdgpu.ids || exit 1
done
