set -o pipefail
O=gpurun_out/t9; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in f48 f64 f48 f64; do
echo "== $v"; SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 120 python -u tools/stage_ab.py 2>&1 | grep -v amdgpu.ids
done
