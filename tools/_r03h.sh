set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_h; mkdir -p $O
for v in rel rw8 rw6 rw4 rw1; do
  if [ $v = rel ]; then L=semantic_merge_amd/libsmx.so; else L=tools/_build/var_$v/libsmx.so; fi
  SMX_LIB=$L RGA_NO_CPU=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 tools/bench_rga.py > $O/rga_$v.json 2> $O/rga_$v.err || { tail -5 $O/rga_$v.err; exit 1; }
  echo "$v $(cat $O/rga_$v.json)"
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1); cp $f $O/ks_$v.csv
  python3 - $O/ks_$v.csv <<'PY'
import csv,sys
for r in list(csv.reader(open(sys.argv[1])))[1:]:
    if 'rga' in r[0] or 'rrec' in r[0] or 'hscan' in r[0]: print('   ', r[0].split('(')[0][:34], r[3])
PY
done
