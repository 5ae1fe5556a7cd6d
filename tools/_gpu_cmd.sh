set -o pipefail
O=gpurun_out/r02zj; mkdir -p $O
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 200 --timeout-method thread > $O/rga_tests.log 2>&1; rc=$?; tail -2 $O/rga_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -2 $O/bench.err; cat $O/bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e > $R/$O/prof.log 2>&1 || exit 1
cd $R && python3 tools/prof_export.py $O/prof $O/kernel_stats.csv
timeout -k 10 200 python -u tools/bench_rga.py > $O/bench_rga.json 2>&1; tail -1 $O/bench_rga.json | cut -c1-300
