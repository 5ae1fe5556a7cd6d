# Round-end measurement pass: full GPU suite, smoke, default bench (PMC + CPU legs),
# rocprof kernel stats, config 5 / config 2 / RGA bench lines.
set -o pipefail
TAG=${TAG:-r03_end}; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_check.sh $TAG tests bench prof || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --no-e2e > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --steps 50 --no-pmc --no-e2e > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
timeout -k 10 300 python -u tools/bench_rga.py > $O/bench_rga.json 2> $O/bench_rga.err || { tail -5 $O/bench_rga.err; exit 1; }
timeout -k 10 200 python -u tools/small_merge_probe.py --sizes 1000,2000,10000,1000000 > $O/small_probe.json 2> $O/small_probe.err || { tail -5 $O/small_probe.err; exit 1; }
cut -c1-300 $O/bench_c5.json $O/bench_rga.json $O/small_probe.json
(cd /tmp && export TMPDIR=/tmp && RGA_NO_CPU=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_rga" -o r -- python3 "$R/tools/bench_rga.py" > "$O/prof_rga.log" 2>&1) || { tail -5 "$O/prof_rga.log"; exit 1; }
python3 tools/prof_export.py "$O/prof_rga" "$O/rga_kernel_stats.csv" && head -8 "$O/rga_kernel_stats.csv"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-pmc > "$O/prof_c5.log" 2>&1) || { tail -5 "$O/prof_c5.log"; exit 1; }
python3 tools/prof_export.py "$O/prof_c5" "$O/c5_kernel_stats.csv" && python3 tools/prof_timeline.py "$O/prof_c5" 60 > "$O/c5_timeline.txt" && tail -3 "$O/c5_timeline.txt"
