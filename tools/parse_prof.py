"""Summarise a tools/profile.sh run into profiles/ (markdown + traffic JSON).

usage: python tools/parse_prof.py gpurun_out/prof_<tag> <tag> [config_name]
FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (rocprofv3); per
MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reports 1/2 of a wide coalesced
stream's bytes, so HBM read bytes = 2 x FETCH_SIZE x 1024 (upper estimate for
the trace kernel's scattered 16-B node loads -- both raw and corrected are kept).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    """Kernel name without the argument list: 'k_trace<false, false, true, 256>'."""
    import re
    m = re.search(r"(k_\w+<[^>]*>)", name)
    if m:
        return m.group(1)
    m = re.search(r"(k_\w+)", name.split("(")[0])
    return m.group(1) if m else name.split("(")[0][:60]


def main():
    d, tag = sys.argv[1], sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "soup-1M"
    tr = rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    dur = defaultdict(list)
    for r in tr:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"# rocprofv3 kernel summary ({tag})", "",
             f"source: `rocprofv3 --kernel-trace --stats -- python3 bench.py ...` ({d})", "",
             "| kernel | calls | avg us | min us | max us | total us |", "|---|---|---|---|---|---|"]
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {len(v)} | {sum(v)/len(v):.2f} | {min(v):.2f} | {max(v):.2f} | {sum(v):.1f} |")
    pm = {}
    for kind, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        acc = defaultdict(list)
        for r in rows(os.path.join(d, kind, "**", "*counter_collection.csv")):
            if r.get("Counter_Name") == cname:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        pm[cname] = {k: sum(v) / len(v) for k, v in acc.items()}
    lines += ["", "## HBM traffic per dispatch (PMC, separate passes)", "",
              "| kernel | FETCH_SIZE KiB | WRITE_SIZE KiB | read bytes (2x FETCH, gfx950 corr.) | write bytes |",
              "|---|---|---|---|---|"]
    for k in sorted(set(pm["FETCH_SIZE"]) | set(pm["WRITE_SIZE"])):
        f = pm["FETCH_SIZE"].get(k, float("nan"))
        w = pm["WRITE_SIZE"].get(k, float("nan"))
        lines.append(f"| {k} | {f:.1f} | {w:.1f} | {2*f*1024:.3e} | {w*1024:.3e} |")
    os.makedirs("profiles", exist_ok=True)
    open(f"profiles/rocprof_{tag}.md", "w").write("\n".join(lines) + "\n")
    tk = "k_trace<false, false, true, 256, false, true>"  # the timed launch: no counters, full image, wide traversal, buffer loads
    if tk in pm["FETCH_SIZE"] and tk in pm["WRITE_SIZE"]:
        fetch = pm["FETCH_SIZE"][tk] * 1024
        write = pm["WRITE_SIZE"][tk] * 1024
        json.dump({"config": cfg, "n_gpus": 1, "kernel": tk, "tag": tag,
                   "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
                   "hbm_bytes_per_launch": 2 * fetch + write,
                   "avg_us": sum(dur[tk]) / len(dur[tk]) if dur.get(tk) else None,
                   "note": "hbm = 2*FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE"},
                  open("profiles/traffic_trace.json", "w"), indent=2)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
