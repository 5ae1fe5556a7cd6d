set -o pipefail
O=gpurun_out/r03_e; mkdir -p $O
echo "== release"; timeout -k 10 200 python -u tools/graph_debug.py 2>&1 | tee $O/graph_rel.txt | grep -v amdgpu.ids
echo "== no graphs"; SMX_LIB=tools/_build/var_nograph/libsmx.so timeout -k 10 200 python -u tools/graph_debug.py 2>&1 | tee $O/graph_nog.txt | grep -v amdgpu.ids
timeout -k 10 400 env SMX_LIB=tools/_build/var_diag/libsmx.so python3 -u tools/window_ablate.py > $O/ablate.txt 2>&1; rc=$?; cat $O/ablate.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py --rounds 7 rel=semantic_merge_amd/libsmx.so bk16=tools/_build/var_bk16/libsmx.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
