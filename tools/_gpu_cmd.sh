set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
R=$PWD
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -3 $O/bench.err; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e > $R/$O/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || { tail -5 $R/$O/prof.log; exit $rc; }
cd $R && python3 tools/prof_export.py $O/prof $O/kernel_stats.csv && head -12 $O/kernel_stats.csv | cut -c1-150
