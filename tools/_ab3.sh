set -o pipefail
TAG=${TAG:-r02k_ab3}; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2 3; do
  echo -n "c5 new: "; timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  echo -n "c5 prev: "; SMX_LIB=tools/_build/var_prev/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 20000000 c5 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done
