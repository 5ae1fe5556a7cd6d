#!/bin/bash
# SQ instruction counters of k_window_f per phase exit (diagnostic build, SMX_ABLATE):
#   bash tools/sq_ablate.sh OUTDIR LIB "16 121 122 ... 0"
# one rocprofv3 --pmc pass per value, 2 merges of a 20M-op config-3-shaped log each
set -o pipefail
R=$PWD
OUT=$(realpath -m "${1:?outdir}"); LIB=$(realpath "${2:?lib}"); VALS=${3:-"16 0"}
mkdir -p "$OUT"
for ab in $VALS; do
  (cd /tmp && export TMPDIR=/tmp && SMX_LIB=$LIB SMX_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
      --kernel-include-regex 'k_window_f' --kernel-trace -d "$OUT/a$ab" -o p --output-format csv -- python3 "$R/tools/compose_runs.py" 2 20000000 > "$OUT/a$ab.log" 2>&1) \
    || { echo "ablate $ab failed"; tail -5 "$OUT/a$ab.log"; exit 1; }
  python3 "$R/tools/pmc_table.py" "$OUT/a$ab" > "$OUT/a$ab.txt" && echo "== $ab" && grep -E "INSTS_VALU|INSTS_SALU|INSTS_LDS|BANK|Duration|dur" "$OUT/a$ab.txt"
done
