"""Summarise tools/coop_prof.py's kernel trace: per cap, per rank (frames
2-4), the k_tile_order / k_trace / k_trace_coop durations in launch order.
usage: python tools/coop_prof_parse.py DIR cap [cap...]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
caps = [int(x) for x in sys.argv[2:]]
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tr = [r for r in rows if "k_trace" in r["Kernel_Name"] or "k_tile_order" in r["Kernel_Name"]]
# skip the build's kernels; group: each frame = [k_tile_order] k_trace [k_trace_coop]
frames, cur = [], None
for r in tr:
    n = r["Kernel_Name"]
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    if "k_tile_order" in n or ("k_trace<" in n and (cur is None or "trace" in cur)):
        if cur is not None and ("k_tile_order" in n or "trace" in cur):
            frames.append(cur)
            cur = None
    if cur is None:
        cur = {"start": int(r["Start_Timestamp"])}
    key = "order" if "k_tile_order" in n else ("coop" if "k_trace_coop" in n else "trace")
    cur[key] = us
    cur["end"] = int(r["End_Timestamp"])
if cur:
    frames.append(cur)
P = int(os.environ.get("COOP_P", "8"))
per_cap = P * 4 + 4
print(f"{len(frames)} frames parsed (expect {per_cap * len(caps)})")
for i, c in enumerate(caps):
    fs = frames[i * per_cap:(i + 1) * per_cap]
    print(f"cap {c}:")
    for r in range(P + 1):
        grp = fs[r * 4:(r + 1) * 4][1:]
        if not grp:
            continue
        tag = f"rank {r}" if r < P else "full  "
        span = [(f["end"] - f["start"]) / 1000.0 for f in grp]
        print(f"  {tag}: trace " + " ".join(f"{f.get('trace', 0):7.1f}" for f in grp) +
              " | coop " + " ".join(f"{f.get('coop', 0):6.1f}" for f in grp) +
              " | span " + " ".join(f"{x:7.1f}" for x in span) + " us")
