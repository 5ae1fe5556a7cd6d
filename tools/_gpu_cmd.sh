set -o pipefail
O=gpurun_out/r02za; mkdir -p $O
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 200 --timeout-method thread > $O/rga_tests.log 2>&1; rc=$?; tail -2 $O/rga_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o r -- python3 $R/tools/bench_rga.py > $R/$O/rga_prof.log 2>&1 || exit 1
cd $R && python3 tools/prof_export.py $O/prof $O/rga_kernel_stats.csv && python3 -c "
import csv
r=list(csv.reader(open('$O/rga_kernel_stats.csv')))
for x in r[1:12]: print(x[0][:40], x[3])
print('total', sum(float(x[2]) for x in r[1:] if 'rga' in x[0] or 'rrec' in x[0] or 'scan' in x[0])/int(r[1][1]))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py -k "full_size or empty_middle" -x -v --timeout 850 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; exit $rc
