#!/bin/bash
# One GPU-box pass: parity tests, bench (with cpu_baseline), rocprofv3 kernel stats.
#   gpurun -- bash tools/gpu_check.sh <tag> [tests|bench|prof ...]
set -o pipefail
TAG=${1:-check}; shift
STEPS=${*:-tests bench prof}
R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p "$O"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
           tail -3 "$O/tests.log";;
    bench) timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
           cat "$O/bench.json";;
    benchq) timeout -k 10 200 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
           cat "$O/bench.json";;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o p -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e > "$O/prof.log" 2>&1) || { tail -20 "$O/prof.log"; exit 1; }
          python3 tools/prof_export.py "$O/prof" "$O/kernel_stats.csv" && head -12 "$O/kernel_stats.csv";;
    pmc) timeout -k 10 900 bash tools/pmc_passes.sh "$O/pmc" || exit 1;;
  esac
done
