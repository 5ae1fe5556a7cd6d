#!/bin/bash
# Run-grouped window phase exits (SMX_ABLATE 16, 0x10000 + step, 109, 0; diagnostic build
# tools/_build/var_diag) on config 5's shape (wide windows first, SMX_FIRST_WIDE) and on
# config 3's, 20M ops each, SQ counters per exit (tools/sq_ablate.sh):
#   gpurun -- bash tools/ablate_runs.sh gpurun_out/<tag>      (profiles/r05_ablate)
set -o pipefail
O=$1; mkdir -p "$O"
V="16 65537 65538 65539 65540 65541 65542 65543 65544 109 65545 65546 0"
COMPOSE_CFG=c5 SMX_FIRST_WIDE=1 bash tools/sq_ablate.sh "$O/c5" tools/_build/var_diag/libsmx.so "$V" > "$O/c5.txt" 2>&1 || { tail -5 "$O/c5.txt"; exit 1; }
bash tools/sq_ablate.sh "$O/c3" tools/_build/var_diag/libsmx.so "109 65545 65546 0" > "$O/c3.txt" 2>&1 || { tail -5 "$O/c3.txt"; exit 1; }
for f in "$O"/c5/a*.txt "$O"/c3/a*.txt; do echo "$f $(awk '/^k_window_f/{p=1} p && /dur_us/{print $2; exit}' $f)"; done
