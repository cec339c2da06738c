"""Average PMC counters per dispatch of one kernel from tools/pmc_trace.sh output."""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "k_trace"
acc = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"] and "persist" not in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:<36s} {sum(v)/len(v):16.4g}   (n={len(v)})")
