set -o pipefail
TAG=${TAG:-r02k_c5}; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o p -- python3 "$R/bench.py" --config c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_c5.log" 2>&1) || { tail -20 $O/prof_c5.log; exit 1; }
python3 tools/prof_export.py $O/prof_c5 $O/kernel_stats_c5.csv && cut -c1-60,180- $O/kernel_stats_c5.csv | head -14
