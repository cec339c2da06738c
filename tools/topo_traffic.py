"""Summarise tools/topo_traffic.sh: k_topo_refit's HBM traffic per launch at
1M and 10M, split by stream.
usage: python tools/topo_traffic.py [gpurun_out] > profiles/topo_traffic_r06.md

Streams and their floors (SURVEY.md §8(d) K4-K7 = 256 B/prim algorithmic):
  writes  = WRITE_SIZE: internal nodes 32 B + K7w records 64 B + leaf triangle
            records (tri_s) 48 B per prim = 144 B/prim, plus the crossing
            tables (prefix/suffix boxes, topology words, list) -- written whole;
  gather  = the random 36-B triangle read through the sorted index: the
            shipped library's fetch minus the variant's (gseq: leaf k reads
            tris[k], coalesced, 36 B/prim) plus those 36 B/prim;
  other   = the variant's fetch minus the coalesced 36 B/prim: the sorted keys
            (each block stages its 256 keys and 512 on either side) and
            values, bucket starts, crossing words.
FETCH_SIZE is doubled (the gfx950 correction, MI355X_MICROARCH.md); the
request-size pass gives the fabric read requests by size (RDREQ counts, of
which 32 B / 64 B / 128 B)."""
import csv
import glob
import os
import sys
from collections import defaultdict

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
K = "k_topo_refit"


def per_launch(tag, counter):
    files = glob.glob(os.path.join(D, f"tt_{tag}_{counter.split('_sum')[0] if counter.startswith('TCC') else counter}",
                                   "**", "*counter_collection.csv"), recursive=True)
    if not files and counter.startswith("TCC_EA0_RDREQ"):
        files = glob.glob(os.path.join(D, f"tt_{tag}_TCC_EA0_RDREQ_sum", "**", "*counter_collection.csv"), recursive=True)
    if not files and counter.startswith("TCC_EA0_WRREQ"):
        files = glob.glob(os.path.join(D, f"tt_{tag}_TCC_EA0_WRREQ_sum", "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(float)
    for f in files:
        for r in csv.DictReader(open(f)):
            if K in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(vals.values())
    return (sum(v[1:]) / max(len(v) - 1, 1)) if len(v) > 1 else (v[0] if v else float("nan"))  # drop the first (probe) build


print("# k_topo_refit HBM traffic by stream (r06, tools/topo_traffic.sh + tools/topo_traffic.py)\n")
print("Per launch, means over the timed builds of `tools/build_times.py n 8` under one `rocprofv3 --pmc` pass each. "
      "`gseq` = `lib/exp/gseq.so` (-DRT_EXP_GATHER_SEQ: leaf k's triangle read coalesced from tris[k]; wrong output, "
      "traffic attribution only).\n")
for n in (1_000_000, 10_000_000):
    base, seq = f"librtamd_{n}", f"gseq_{n}"
    fb = 2 * 1024 * per_launch(base, "FETCH_SIZE")
    fs = 2 * 1024 * per_launch(seq, "FETCH_SIZE")
    wb = 1024 * per_launch(base, "WRITE_SIZE")
    coal = 36.0 * n
    other = fs - coal
    gather = fb - other
    print(f"## n = {n:,}\n")
    print("| stream | bytes per launch | B/prim | floor B/prim | vs floor |")
    print("|---|---|---|---|---|")
    print(f"| writes (nodes 32 + K7w 64 + tri_s 48 + crossing tables) | {wb:.4g} | {wb / n:.1f} | 144 | {wb / n / 144:.3f} |")
    print(f"| triangle gather (random, through the sorted index) | {gather:.4g} | {gather / n:.1f} | 36 (algorithmic); "
          f"163 as 128-B lines (a 36-B record straddles 2 lines with p = 35/128) | {gather / n / 36:.2f} / {gather / n / 163:.3f} |")
    print(f"| keys window + values + bucket starts + crossing words | {other:.4g} | {other / n:.1f} | 8 (keys + values once) "
          f"| {other / n / 8:.2f} |")
    print(f"| total (2 x FETCH_SIZE + WRITE_SIZE) | {fb + wb:.4g} | {(fb + wb) / n:.1f} | 256 (§8(d)) | {(fb + wb) / n / 256:.3f} |")
    rq = {c: per_launch(base, c) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                                            "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")}
    rs = {c: per_launch(seq, c) for c in rq}
    print("\nfabric requests per launch (shipped / gseq):\n")
    print("| counter | shipped | gseq | shipped per prim |")
    print("|---|---|---|---|")
    for c in rq:
        print(f"| {c} | {rq[c]:.4g} | {rs[c]:.4g} | {rq[c] / n:.3f} |")
    print()
