# round 3 (ae): k_wcount with 128 / 64 threads per window (more windows in flight) -- parity + c5 A/B
set -o pipefail
O=gpurun_out/r03_ae; mkdir -p $O
timeout -k 10 300 python3 tools/parity_libs.py new=semantic_merge_amd/libsmx.so wc128=tools/_build/var_wc128/libsmx.so wc64=tools/_build/var_wc64/libsmx.so > $O/parity.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/parity.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in new wc128 wc64; do
  if [ $v = new ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-pmc --no-e2e > $O/c5_${v}_$r.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['ms_per_step'], d['graph_api']['ms_per_step'], d['stages_ms_per_step'])"
done; done
