set -o pipefail
O=gpurun_out/${TAG:-abwin}; mkdir -p $O
for r in 1 2; do
  for v in ${VARS:-base minb4}; do
    echo -n "$v: "; SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab_$v.txt || exit 1
  done
done
