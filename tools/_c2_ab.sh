#!/bin/bash
# config 2 wall time (bench.py, graph replay) of two builds, alternating: bash tools/_c2_ab.sh OUT name=lib name=lib
set -o pipefail
O=$1; shift; mkdir -p "$O"
for r in 1 2 3; do
  for spec in "$@"; do
    n=${spec%%=*}; lib=$(realpath "${spec#*=}")
    SMX_LIB=$lib timeout -k 10 120 python -u bench.py --config c2 --steps 100 --no-pmc --no-e2e --no-cpu-baseline > "$O/$n.$r.json" 2>/dev/null || { echo "$n failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$n.$r.json').read().strip().splitlines()[-1]); print('$n', $r, d['ms_per_step'])"
  done
done
