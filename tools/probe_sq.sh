#!/bin/bash
# SQ / TA / TCP counter passes over K compose merges (tools/compose_runs.py, kernel trace
# only, one rocprofv3 run per counter group) and the window-phase ablations of a
# diagnostic build.  Run on the GPU box from the repo root:
#   bash tools/probe_sq.sh OUTDIR [groups...]      groups: sq1 sq2 ta list ablate
set -o pipefail
R=$PWD
OUT=$(realpath -m "${1:-$R/gpurun_out/probe}"); shift
mkdir -p "$OUT"
RX=${SMX_PMC_RX:-'k_window_f|k_emit|k_tb_scatter|k_tb_reduce'}
for g in ${*:-sq1 sq2 ta}; do
  case $g in
    sq1) C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES";;
    sq2) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES";;
    ta) C="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE";;
    list) (cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1); echo "list rc=$?"; continue;;
    ablate) timeout -k 10 300 env SMX_LIB=tools/_build/var_diag/libsmx.so python3 -u tools/window_ablate.py > "$OUT/ablate.txt" 2>&1 || { tail -5 "$OUT/ablate.txt"; exit 1; }
            cat "$OUT/ablate.txt"; continue;;
  esac
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d "$OUT/$g" -o p \
      --output-format csv -- python3 "$R/tools/compose_runs.py" 2 > "$OUT/$g.log" 2>&1) || { echo "pass $g failed"; tail -5 "$OUT/$g.log"; exit 1; }
  echo "pass $g done"
done
python3 tools/pmc_summary.py "$OUT"/sq* "$OUT"/ta > "$OUT/summary.json" 2>/dev/null; echo summary rc=$?
