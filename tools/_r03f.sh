set -o pipefail
O=gpurun_out/r03_f; mkdir -p $O
echo "== graphs 600k"; timeout -k 10 200 python -u tools/graph_debug.py 2>&1 | tee $O/graph_rel.txt | grep -v amdgpu.ids
echo "== graphs 5M"; timeout -k 10 200 python -u tools/graph_debug.py 5000000 2>&1 | tee $O/graph_rel5M.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_c.log 2>&1; rc=$?; tail -5 $O/tests_c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 wavebk=semantic_merge_amd/libsmx.so nowbk=tools/_build/var_nowbk/libsmx.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
