# round 3 (q): step-5 scan with one barrier, final order fused into the rank loop
set -o pipefail
O=gpurun_out/r03_q; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py new=tools/_build/var_new/libsmx.so > $O/parity.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_libs.py --rounds 7 rel=semantic_merge_amd/libsmx.so new=tools/_build/var_new/libsmx.so fusefin=tools/_build/var_fusefin/libsmx.so scan1=tools/_build/var_scan1/libsmx.so > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
SMX_LIB=tools/_build/var_new/libsmx.so timeout -k 10 700 python -u -m pytest tests/test_gpu_compose.py tests/test_gpu_full.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc

timeout -k 10 600 python -u -m pytest tests/test_gpu_rga.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in new ht1off; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 python3 tools/bench_rga.py > $O/rga_${v}_$r.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }; echo "rga $v $(cat $O/rga_${v}_$r.json)"
done; done
