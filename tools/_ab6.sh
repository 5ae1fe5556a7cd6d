set -o pipefail
TAG=${TAG:-r02k_ab7}; O=gpurun_out/$TAG; mkdir -p $O
for v in w768b6 w1152b6; do
  SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_compose.py -x -q --timeout 200 --timeout-method thread -k "c2_1M or c5_2M or dense160 or value_widths" > $O/tests_$v.log 2>&1; rc=$?; tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for v in base w768b6 w1152b6 w512b8; do
    L=semantic_merge_amd/libsmx.so; [ $v = base ] || L=tools/_build/var_$v/libsmx.so
    echo -n "$v: "; SMX_LIB=$L timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  done
done
