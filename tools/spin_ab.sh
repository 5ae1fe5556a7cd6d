#!/bin/bash
# host-wait A/B (library builds alternating): config 2 and config 3 per merge, RGA per
# call, a 1k-op merge:  bash tools/spin_ab.sh OUT name=lib name=lib
set -o pipefail
O=$1; shift; mkdir -p "$O"
for r in 1 2; do
  for spec in "$@"; do
    n=${spec%%=*}; lib=$(realpath "${spec#*=}")
    SMX_LIB=$lib timeout -k 10 120 python -u bench.py --config c2 --steps 100 --no-pmc --no-e2e --no-cpu-baseline > "$O/c2.$n.$r.json" 2>/dev/null || { echo "c2 $n failed"; exit 1; }
    SMX_LIB=$lib timeout -k 10 150 python -u bench.py --steps 10 --no-pmc --no-e2e --no-cpu-baseline > "$O/c3.$n.$r.json" 2>/dev/null || { echo "c3 $n failed"; exit 1; }
    SMX_LIB=$lib RGA_NO_CPU=1 RGA_STEPS=20 timeout -k 10 120 python -u tools/bench_rga.py > "$O/rga.$n.$r.json" 2>/dev/null || { echo "rga $n failed"; exit 1; }
    SMX_LIB=$lib timeout -k 10 120 python -u tools/small_merge_probe.py --sizes 1000 --reps 100 > "$O/small.$n.$r.json" 2>/dev/null || { echo "small $n failed"; exit 1; }
    python3 - "$O" "$n" "$r" <<'PY'
import json, sys
o, n, r = sys.argv[1:]
ld = lambda f: json.loads(open(f"{o}/{f}").read().strip().splitlines()[-1])
c2, c3, rga, sm = ld(f"c2.{n}.{r}.json"), ld(f"c3.{n}.{r}.json"), ld(f"rga.{n}.{r}.json"), ld(f"small.{n}.{r}.json")
print(n, r, "c2", c2["ms_per_step"], "c3", c3["ms_per_step"], "rga", rga["ms_per_step"], "grouped", rga["grouped"]["ms_per_step"],
      "1k", sm["small_merges"]["1000"]["device_ms"], sm["small_merges"]["1000"]["session_ms"])
PY
  done
done
