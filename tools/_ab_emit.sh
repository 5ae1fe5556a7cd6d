set -o pipefail
O=gpurun_out/ab7; mkdir -p $O
for v in r1024x3 r512x3 r256x4 r1024x2 r512x2 r1024x3; do
  echo "== $v" >> $O/ab.txt
  SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 120 python -u tools/bench_rga.py 2>&1 | grep -v amdgpu.ids | cut -c1-200 >> $O/ab.txt || exit 1
done
cat $O/ab.txt
