set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in base; do
  if [ $v = base ]; then L=$R/semantic_merge_amd/libsmx.so; else L=$R/tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 RGA_STEPS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/p_$v -o r -- python3 $R/tools/bench_rga.py > $R/$O/$v.log 2>&1 || exit 1
  (cd $R && python3 tools/prof_export.py $O/p_$v $O/$v.csv && python3 -c "
import csv
r=[x for x in csv.reader(open('$O/$v.csv'))][1:5]
print('$v', [(x[0][:22], x[3]) for x in r])
")
done
cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_compose.py -x -q --timeout 200 --timeout-method thread > $O/tests2.log 2>&1; rc=$?; tail -3 $O/tests2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dropin_bench.py --gpu --sizes 1000,10000,1000000 --out $O/dropin.jsonl > $O/dropin.log 2>&1; tail -3 $O/dropin.log
