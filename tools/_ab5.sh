set -o pipefail
TAG=${TAG:-r02k_ab5}; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo -n "kh512: "; timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
  echo -n "kh256: "; SMX_LIB=tools/_build/var_kh256/libsmx.so timeout -k 10 200 python -u tools/stage_ab.py 2>&1 | tail -1 | tee -a $O/ab.txt || exit 1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o p -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e > "$O/prof.log" 2>&1) || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_export.py $O/prof $O/kernel_stats.csv && cut -c1-50 $O/kernel_stats.csv | head -14
