set -o pipefail
O=gpurun_out/r1s31; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
R=$PWD; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_export.py $O/prof $O/kernel_stats.csv && head -8 $O/kernel_stats.csv | cut -c1-100
timeout -k 10 300 python -u tools/bench_rga.py > $O/rga.json 2> $O/rga.err || { tail -20 $O/rga.err; exit 1; }
timeout -k 10 300 python tools/stage_ab.py 20000000 c5 > $O/c5.txt 2>&1 || exit 1
