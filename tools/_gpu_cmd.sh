set -o pipefail
O=gpurun_out/r02zi; mkdir -p $O
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 200 --timeout-method thread > $O/rga_tests.log 2>&1; rc=$?; tail -2 $O/rga_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in base pcu1 t4096; do
  if [ $v = base ]; then L=$R/semantic_merge_amd/libsmx.so; else L=$R/tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 RGA_STEPS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_$v -o r -- python3 $R/tools/bench_rga.py > $R/$O/$v.log 2>&1 || exit 1
  (cd $R && python3 tools/prof_export.py $O/p_$v $O/$v.csv && python3 -c "
import csv
r=list(csv.reader(open('$O/$v.csv')))
print('$v', [(x[0][:22], x[3]) for x in r[1:6]])
print('  total', round(sum(float(x[2]) for x in r[1:] if 'rga' in x[0] or 'rrec' in x[0] or 'scan' in x[0])/int(r[1][1]),1))")
done
