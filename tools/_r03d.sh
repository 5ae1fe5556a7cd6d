set -o pipefail
O=gpurun_out/r03_d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env SMX_LIB=tools/_build/var_diag/libsmx.so python3 -u tools/window_ablate.py > $O/ablate.txt 2>&1; rc=$?; cat $O/ablate.txt; [ $rc -eq 0 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rga -o p -- python3 $GRAFT_REPO_ROOT/tools/bench_rga.py > $GRAFT_REPO_ROOT/$O/rga_prof.log 2>&1) || { tail -5 $O/rga_prof.log; exit 1; }
python3 tools/prof_export.py $O/rga $O/rga_kernel_stats.csv && head -20 $O/rga_kernel_stats.csv
