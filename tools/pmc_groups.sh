#!/bin/bash
# Counter passes over one workload, one rocprofv3 run per group (kernel trace only; no
# sys/runtime traces).  Counters the box does not list (rocprofv3 -L) are dropped from
# their group first.  Run on the GPU box from the repo root:
#   bash tools/pmc_groups.sh OUTDIR 'KERNEL_REGEX' 'GROUP1' 'GROUP2' ... -- CMD ARGS
# e.g. bash tools/pmc_groups.sh gpurun_out/x 'k_emit4' 'TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum' -- python3 bench.py --steps 2
# Limits per pass (MI355X_MICROARCH.md): 8 SQ, 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), 4 TCP,
# 2 TA, 2 TD, 2 GRBM.
set -o pipefail
R=$PWD
OUT=$(realpath -m "$1"); shift
RX=$1; shift
GRPS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GRPS+=("$1"); shift; done
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -s "$OUT/../counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$OUT/../counters.txt" 2>&1 || true
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  keep=""
  for c in $grp; do
    if grep -qw "$c" "$OUT/../counters.txt"; then keep="$keep $c"; else echo "pass $i: $c not listed, dropped"; fi
  done
  [ -z "$keep" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $keep --kernel-include-regex "$RX" -d "$OUT/p$i" -o p \
      --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done:$keep"
done
