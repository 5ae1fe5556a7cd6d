#!/bin/bash
# c2 window-size sweep on a diagnostic build (SMX_WIN_TGT): ms per step and stages
set -o pipefail
O=$1; mkdir -p "$O"
for tgt in 1792 1280 1024 768 512; do
  SMX_LIB=$PWD/tools/_build/var_diag/libsmx.so SMX_WIN_TGT=$tgt timeout -k 10 120 python -u bench.py --config c2 --steps 50 --no-pmc --no-e2e --no-cpu-baseline > "$O/c2_tgt$tgt.json" 2>&1 || { echo "tgt $tgt failed"; tail -5 "$O/c2_tgt$tgt.json"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/c2_tgt$tgt.json').read().strip().splitlines()[-1]); print($tgt, d['ms_per_step'], d.get('stages_ms_per_step'))"
done
