# round 3 (u): SQ counters of the current k_window_f; config 5 kernel timeline
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03_u; mkdir -p $O
SMX_PMC_RX='k_window_f' bash tools/pmc_sq.sh $O/pmc_sq || exit 1
python3 -c "import json;d=json.load(open('$O/pmc_sq/summary.json'))['kernels']['k_window_f'];print({k:d[k] for k in ('SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_LDS_BANK_CONFLICT')})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o c5 -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-pmc > "$O/prof_c5.log" 2>&1) || { tail -5 "$O/prof_c5.log"; exit 1; }
python3 tools/prof_export.py "$O/prof_c5" "$O/c5_kernel_stats.csv" && python3 tools/prof_timeline.py "$O/prof_c5" 70 > $O/c5_timeline.txt; rc=$?; tail -75 $O/c5_timeline.txt; exit $rc
