#!/bin/bash
# GPU-box steps for iterating (each under its own time limit; stops at the first failure):
#   gpurun -- bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# steps: rga (RGA GPU tests), compose (compose GPU tests incl. full-size digests),
#        small (small-plan tests + tools/small_merge_probe.py), smallprof (its kernel trace),
#        smallph (phase stamps, tools/_build/var_stamps), gtests (the whole -m gpu suite),
#        ab / ab5 (tools/ab_libs.py, current vs tools/_build/var_old, configs 3 / 5),
#        rgabench (tools/bench_rga.py), rgaprof (its kernel trace and timeline), bench (bench.py,
#        no PMC / CPU legs), benchfull (bench.py default), c5, c2 (bench.py configs), c2prof
#        (config-2 kernel timeline), shard (sharded GPU tests + tools/shard_probe.py), prof
#        (config-3 kernel stats), sq (tools/pmc_sq.sh)
set -o pipefail
TAG=${1:?tag}; shift
R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p "$O"
run() {  # run <seconds> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; tail -30 "$O/$log"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    rga) run 600 rga_tests.log python -u -m pytest tests/test_gpu_rga.py -x -v --timeout 300 --timeout-method thread
         tail -2 "$O/rga_tests.log";;
    compose) run 900 compose_tests.log python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -x -v --timeout 300 --timeout-method thread
         tail -2 "$O/compose_tests.log";;
    small) run 300 small_tests.log python -u -m pytest tests/test_gpu_small.py -x -v --timeout 120 --timeout-method thread
         tail -2 "$O/small_tests.log"
         run 300 small_probe.json python -u tools/small_merge_probe.py --sizes 1000,2000,10000,1000000 --verify
         tail -1 "$O/small_probe.json";;
    smallprof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/sprof" -o p -- python3 "$R/tools/small_merge_probe.py" --sizes 1000,2000 --reps 30 > "$O/sprof.log" 2>&1) || { echo "smallprof failed"; tail -20 "$O/sprof.log"; exit 1; }
          python3 tools/prof_export.py "$O/sprof" "$O/small_kernel_stats.csv" && head -5 "$O/small_kernel_stats.csv";;
    c2prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/c2prof" -o p -- python3 "$R/tools/small_merge_probe.py" --sizes 1000000 --reps 20 > "$O/c2prof.log" 2>&1) || { echo "c2prof failed"; tail -20 "$O/c2prof.log"; exit 1; }
          python3 tools/prof_timeline.py "$O/c2prof" 40 > "$O/c2_timeline.txt" && tail -42 "$O/c2_timeline.txt";;
    smallph) SMX_LIB=$R/tools/_build/var_stamps/libsmx.so run 300 small_phases.json python -u tools/small_phases.py
          tail -1 "$O/small_phases.json";;
    rgaprof) (cd /tmp && export TMPDIR=/tmp && RGA_NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rgaprof" -o p -- python3 "$R/tools/bench_rga.py" > "$O/rgaprof.log" 2>&1) || { echo "rgaprof failed"; tail -20 "$O/rgaprof.log"; exit 1; }
          python3 tools/prof_export.py "$O/rgaprof" "$O/rga_kernel_stats.csv" && head -14 "$O/rga_kernel_stats.csv"
          python3 tools/prof_timeline.py "$O/rgaprof" 200 > "$O/rga_timeline.txt";;
    shard) run 900 shard_tests.log python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 400 --timeout-method thread
         tail -2 "$O/shard_tests.log"
         run 300 shard_probe.txt python -u tools/shard_probe.py 8
         tail -6 "$O/shard_probe.txt";;
    gtests) run 1100 tests.log python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
         tail -2 "$O/tests.log";;
    ab) run 400 ab_c3.txt python -u tools/ab_libs.py --rounds 4 new=semantic_merge_amd/libsmx.so old=tools/_build/var_old/libsmx.so
        tail -12 "$O/ab_c3.txt";;
    ab5) run 400 ab_c5.txt python -u tools/ab_libs.py --config c5 --rounds 4 new=semantic_merge_amd/libsmx.so old=tools/_build/var_old/libsmx.so
        tail -12 "$O/ab_c5.txt";;
    rgabench) run 300 bench_rga.json python -u tools/bench_rga.py
        tail -1 "$O/bench_rga.json";;
    bench) run 300 bench.json python -u bench.py --no-cpu-baseline --no-pmc --no-e2e
        tail -1 "$O/bench.json" | cut -c1-600;;
    benchfull) run 600 bench_full.json python -u bench.py
        tail -1 "$O/bench_full.json" | cut -c1-600;;
    c5) run 300 bench_c5.json python -u bench.py --config c5 --steps 10 --no-cpu-baseline --no-e2e
        tail -1 "$O/bench_c5.json" | cut -c1-600;;
    c2) run 300 bench_c2.json python -u bench.py --config c2 --steps 50 --no-pmc --no-e2e
        tail -1 "$O/bench_c2.json" | cut -c1-400;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o p -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e > "$O/prof.log" 2>&1) || { echo "prof failed"; tail -20 "$O/prof.log"; exit 1; }
          python3 tools/prof_export.py "$O/prof" "$O/kernel_stats.csv" && head -8 "$O/kernel_stats.csv";;
    c3tl) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/c3tl" -o p -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e --no-breakdown --no-async > "$O/c3tl.log" 2>&1) || { echo "c3tl failed"; tail -20 "$O/c3tl.log"; exit 1; }
          python3 tools/prof_timeline.py "$O/c3tl" 60 > "$O/c3_timeline.txt" && tail -62 "$O/c3_timeline.txt";;
    sq) run 600 sq.log bash tools/pmc_sq.sh "$O/sq"
        tail -3 "$O/sq.log";;
    *) echo "unknown step $s"; exit 2;;
  esac
done
