#!/bin/bash
# kernel-trace stats of tools/ab_child.py (given modes) for each library given
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=$1; shift
for L in "$@"; do
  n=$(basename $L .so)
  RT_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$n -- python3 tools/ab_child.py $MODES > gpurun_out/kp_$n.log 2>&1 || { tail -5 gpurun_out/kp_$n.log; exit 1; }
  f=$(find gpurun_out/kp_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:8.2f} us\")
" | head -14
done
