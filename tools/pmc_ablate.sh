#!/bin/bash
# SQ instruction counters of k_window_f under each SMX_ABLATE variant (phase costs by
# difference).  Run on the GPU box from the repo root: bash tools/pmc_ablate.sh OUTDIR
set -o pipefail
R=$PWD
OUT=$(realpath -m "${1:-$R/gpurun_out/pmc_ablate}")
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ab in 0 16 2 4; do
  SMX_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
      --kernel-include-regex 'k_window_f' -d "$OUT/a$ab" -o p --output-format csv -- python3 "$R/tools/compose_runs.py" 2 > "$OUT/a$ab.log" 2>&1 || { echo "ablate $ab failed"; tail -5 "$OUT/a$ab.log"; exit 1; }
  echo "ablate $ab done"
done
