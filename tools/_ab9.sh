set -o pipefail
TAG=${TAG:-r02k_ab9}; O=gpurun_out/$TAG; mkdir -p $O
for v in big4k big3k; do
  SMX_LIB=tools/_build/var_$v/libsmx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -x -q --timeout 200 --timeout-method thread -k "c2_1M or dense160 or hot64 or onesym or full" > $O/tests_$v.log 2>&1; rc=$?; tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for v in base big4k big3k; do
    L=semantic_merge_amd/libsmx.so; [ $v = base ] || L=tools/_build/var_$v/libsmx.so
    echo -n "$v: "; SMX_LIB=$L timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  done
done
