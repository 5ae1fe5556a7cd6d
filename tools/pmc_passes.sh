#!/bin/bash
# PMC passes for the hot kernels (run on the GPU box from the repo root).
# One counter group per rocprofv3 run, kernel trace only (no sys/runtime traces).
set -o pipefail
R=$PWD
OUT=${1:-$R/gpurun_out/pmc}
mkdir -p "$OUT"
make -s -C tools || exit 1
cd /tmp && export TMPDIR=/tmp
RX='k_window_f|k_emit|k_tb_scatter|k_tb_reduce|k_calib'
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$RX" -d "$OUT/p$i" -o p \
      --output-format csv -- python3 "$R/tools/pmc_run.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done: $grp"
done
cd "$R" && SMX_PMC_NOPS=100000000 SMX_PMC_OUT="$OUT/pmc_window.json" python3 tools/pmc_summary.py "$OUT"/p* > "$OUT/summary.json" && echo summary ok
