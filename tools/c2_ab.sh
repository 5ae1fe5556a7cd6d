#!/bin/bash
# config-2 per-merge A/B (library builds alternating, bench.py timers off outside the
# roofline steps):  bash tools/c2_ab.sh OUT rounds name=lib name=lib
set -o pipefail
O=$1; R=$2; shift 2; mkdir -p "$O"
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%=*}; lib=$(realpath "${spec#*=}")
    SMX_LIB=$lib timeout -k 10 120 python -u bench.py --config c2 --steps 100 --no-pmc --no-e2e --no-cpu-baseline > "$O/c2.$n.$r.json" 2>/dev/null || { echo "c2 $n failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/c2.$n.$r.json').read().strip().splitlines()[-1]); print('$n', $r, d['ms_per_step'], d.get('async_api',{}).get('ms_per_step'))"
  done
done
