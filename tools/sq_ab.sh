#!/bin/bash
# SQ counters of the window kernel for several libsmx builds (one rocprofv3 --pmc pass per
# counter group and build; 2 merges of a 20M-op config-3-shaped log each):
#   bash tools/sq_ab.sh OUTDIR name=lib.so [name=lib.so ...]
# -> OUTDIR/<name>/p<group>/..., then tools/pmc_table.py per build into OUTDIR/<name>.txt
set -o pipefail
R=$PWD
OUT=$(realpath -m "${1:?outdir}"); shift
mkdir -p "$OUT"
N=${SQ_N:-20000000}
RX=${SQ_RX:-k_window_f}
for spec in "$@"; do
  name=${spec%%=*}; lib=$(realpath "${spec#*=}")
  mkdir -p "$OUT/$name"
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && SMX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
        -d "$OUT/$name/p$i" -o p --output-format csv -- python3 "$R/tools/compose_runs.py" 2 "$N" > "$OUT/$name/p$i.log" 2>&1) \
      || { echo "$name pass $i failed"; tail -5 "$OUT/$name/p$i.log"; exit 1; }
  done
  python3 "$R/tools/pmc_table.py" "$OUT/$name"/p* > "$OUT/$name.txt" && echo "== $name" && cat "$OUT/$name.txt"
done
