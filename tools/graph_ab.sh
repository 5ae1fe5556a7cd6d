#!/bin/bash
# smx_compose with and without the library's graph replay (timers off: bench.py's graph_api
# leg), alternating builds, configs 2 and 3:  bash tools/graph_ab.sh OUT name=lib name=lib
set -o pipefail
O=$1; shift; mkdir -p "$O"
for cfg in c2 c3; do
  for r in 1 2; do
    for spec in "$@"; do
      n=${spec%%=*}; lib=$(realpath "${spec#*=}")
      SMX_LIB=$lib timeout -k 10 150 python -u bench.py --config $cfg --steps 40 --no-pmc --no-e2e --no-cpu-baseline > "$O/$cfg.$n.$r.json" 2>/dev/null || { echo "$n $cfg failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/$cfg.$n.$r.json').read().strip().splitlines()[-1]); print('$cfg', '$n', $r, 'timed', d['ms_per_step'], 'timers-off', d['graph_api']['ms_per_step'])"
    done
  done
done
