"""Per-rank kernel table from a rocprofv3 kernel trace of tools/rank_emul.py
(`gpu_run.sh kstats:<tag>:tools/rank_emul.py:config=<k>~ranks=<P>`): the
dispatches are grouped into frames (a frame = its trace kernel, with the
k_tile_order before it and the k_trace_coop / k_coop_resolve after it), the
first `frames` frames are the full frame, then `frames` per rank in rank
order.  Prints a markdown table: per rank the median over the frames after
the first `drop` of the trace kernel, the queue pass and the frame span.
usage: python tools/rank_trace_md.py <kernel_trace.csv> <P> [frames=6] [drop=2]"""
import csv
import sys

import numpy as np


def frames_of(rows):
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    out, pend = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "k_tile_order" in name:
            pend.append(r)
        elif "k_trace_sl<" in name or "k_trace<" in name:
            out.append({"pre": pend, "trace": r, "post": []})
            pend = []
        elif ("k_trace_coop" in name or "k_coop_resolve" in name) and out:
            out[-1]["post"].append(r)
    return out


def us(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def main():
    path, P = sys.argv[1], int(sys.argv[2])
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    drop = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    fr = frames_of(list(csv.DictReader(open(path))))
    assert len(fr) >= nf * (P + 1), (len(fr), nf, P)
    groups = [("full", fr[:nf])] + [(f"rank {r}", fr[nf * (r + 1): nf * (r + 2)]) for r in range(P)]
    print("| frames | trace kernel | trace kernel us | queue pass us | order us | frame span us | grid |")
    print("|---|---|---|---|---|---|---|")
    spans = []
    for name, g in groups:
        g = g[drop:]
        tr = np.median([us(f["trace"]) for f in g])
        q = np.median([sum(us(x) for x in f["post"]) for f in g])
        o = np.median([sum(us(x) for x in f["pre"]) for f in g])
        sp = np.median([(int((f["post"] or [f["trace"]])[-1]["End_Timestamp"])
                         - int((f["pre"] or [f["trace"]])[0]["Start_Timestamp"])) / 1e3 for f in g])
        if name != "full":
            spans.append(sp)
        grid = int(g[0]["trace"]["Grid_Size_X"]) // int(g[0]["trace"]["Workgroup_Size_X"])
        kern = g[0]["trace"]["Kernel_Name"].split("(")[0].replace("void ", "").replace("rt::", "")
        print(f"| {name} | `{kern}` | {tr:.1f} | {q:.1f} | {o:.1f} | {sp:.1f} | {grid} x {g[0]['trace']['Workgroup_Size_X']} |")
    print(f"\nmax rank span {max(spans):.1f} us, mean {np.mean(spans):.1f} us")


if __name__ == "__main__":
    main()
