#!/bin/bash
# SQ/TCC counter passes on the compose kernels (one rocprofv3 run per group; kernel
# trace only).  Run on the GPU box from the repo root: bash tools/pmc_sq.sh OUTDIR
# (SMX_PMC_CFG=c5: config 5's merges instead of config 3's)
set -o pipefail
R=$PWD
OUT=$(realpath -m "${1:-$R/gpurun_out/pmc_sq}")
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX=${SMX_PMC_RX:-'k_window_f|k_emit|k_tb_scatter|k_tb_reduce'}
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" -d "$OUT/p$i" -o p \
      --output-format csv -- python3 "$R/bench.py" --config "${SMX_PMC_CFG:-c3}" --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-async > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done"
done
cd "$R" && python3 tools/pmc_summary.py "$OUT"/p* > "$OUT/summary.json" && echo summary ok
