set -o pipefail
O=gpurun_out/ab12; mkdir -p $O
for v in tl0 tl_512x16 tl_1024x8 tl_512x8 tk4 tk16 tl0; do
  echo "== $v" >> $O/ab.txt
  SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 120 python -u tools/stage_ab.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
done
cat $O/ab.txt
