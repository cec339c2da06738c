#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/order_bound.py 16 3 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_rp -- python3 tools/order_bound.py 8 1 > gpurun_out/kp_rp.log 2>&1 || exit 1
f=$(find gpurun_out/kp_rp -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:8.2f} us\")
" | head -8
