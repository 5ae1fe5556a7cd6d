set -o pipefail
O=gpurun_out/r1s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests64.log 2>&1 || { tail -30 $O/tests64.log; exit 1; }
tail -2 $O/tests64.log
for v in head cur head cur; do
  echo "== $v"; SMX_LIB=$PWD/tools/_build/var_$v/libsmx.so timeout -k 10 200 python tools/window_phases.py > $O/phases_$v.txt 2>&1 || exit 1
  cat $O/phases_$v.txt | grep -v amdgpu.ids | grep -v "woff\|check\|span"
done
