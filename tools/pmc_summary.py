"""Summarise one tools/gpu_run.sh profile run of `bench.py --only-timed` into
profiles/: a markdown kernel table (rocprof kernel trace + PMC passes) and the
per-launch entry bench.py's roofline reads (profiles/pmc_summary.json).

usage: python tools/pmc_summary.py <prof dir> <tag> <config name> <warmup> [n_gpus]

Only the timed steps count: the first <warmup> frames' dispatches are dropped.
A frame's trace launch = k_tile_order (when present) + k_trace<...> + k_trace_coop
(the heavy-ray pass, when the queue is on); a build = every build kernel between
two trace launches.

PMC corrections (MI355X_MICROARCH.md §HBM): HBM bytes = 2 x FETCH_SIZE (gfx950
tallies a 128-B read request at 64 B) + WRITE_SIZE, both reported in KiB.
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so cycles per launch = it / 8
(checked against the kernel-trace duration x clock in the table).
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys
from collections import defaultdict

BUILD = ("k_bounds", "k_morton", "k_msb_scan", "k_msb_scatter", "k_bucket_sort", "k_tile_hist", "k_scatter",
         "k_scan_tiles", "k_topo_refit", "k_refit_cross", "k_wide_cross", "k_sparse_level", "k_sparse_near", "k_sparse_far", "k_bounds_final",
         "k_msb_chunk_sum", "k_msb_chunk_apply", "k_msb_scatter_big", "k_bucket_sort_big",
         "k_morton_tb", "k_bucket_gather", "k_bucket_dense", "k_digit_hist", "k_group_tables")
# the build's stages for the per-kernel roofline (bench.py roofline_build.kernels), with the
# SURVEY.md §8(d) bytes per prim each stands for: K0 36 + K1 44 + K2 4; K3 64; K4-K7 256 (local
# nodes in k_topo_refit, crossing nodes in the crossing stage, which the model does not split)
STAGE_OF = {"k_bounds": "k0_k1", "k_morton": "k0_k1", "k_morton_tb": "k0_k1", "k_bounds_final": "k0_k1",
            "k_topo_refit": "topo_refit",
            "k_refit_cross": "crossing", "k_wide_cross": "crossing", "k_group_tables": "crossing",
            "k_sparse_near": "crossing", "k_sparse_far": "crossing", "k_sparse_level": "crossing"}
STAGE_ALGO_BPP = {"k0_k1": 84, "sort": 64, "topo_refit": 256, "crossing": 0}
TRACE = ("k_trace", "k_trace_sl")


def short(name):
    m = re.search(r"(k_\w+<[^>]*>)", name)
    if m:
        return m.group(1)
    m = re.search(r"(k_\w+)", name.split("(")[0])
    return m.group(1) if m else name.split("(")[0][:60]


def base(k):
    return k.split("<")[0]


def dispatches(pattern, counter=None):
    """[(dispatch_id, short name, value or duration_us)] in dispatch order."""
    out = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if counter is None:
                v = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                out[int(r["Dispatch_Id"])] = (short(r["Kernel_Name"]), v)
            elif r["Counter_Name"] == counter:
                k = int(r["Dispatch_Id"])
                prev = out.get(k, (None, 0.0))[1]
                out[k] = (short(r["Kernel_Name"]), prev + float(r["Counter_Value"]))
    return [(k,) + out[k] for k in sorted(out)]


def frames(seq, warmup):
    """Split a dispatch sequence into timed frames: per frame the trace launch
    (tile order + trace + the heavy-ray pass and its resolve) and the build
    kernels before it (also summed per build stage, STAGE_OF)."""
    fr, build = [], []
    stages = defaultdict(float)
    pend_order = None
    for _, k, v in seq:
        b = base(k)
        if b in BUILD:
            build.append(v)
            stages[STAGE_OF.get(b, "sort")] += v
        elif b == "k_tile_order":
            pend_order = v
        elif b in TRACE:
            fr.append({"trace": v, "order": pend_order or 0.0, "coop": 0.0, "build": sum(build), "trace_name": k,
                       "stages": dict(stages)})
            build, pend_order = [], None
            stages = defaultdict(float)
        elif b in ("k_trace_coop", "k_coop_resolve") and fr:
            fr[-1]["coop"] += v
    return fr[warmup:]


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    d, tag, cfg, warmup = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    ngpu = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    tr = dispatches(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    ft = frames(tr, warmup)
    trace_us = mean([f["trace"] + f["coop"] for f in ft])
    coop_us = mean([f["coop"] for f in ft])
    order_us = mean([f["order"] for f in ft])
    build_us = mean([f["build"] for f in ft])
    kname = ft[0]["trace_name"] if ft else "?"

    def per_frame(sub, counter):
        seq = dispatches(os.path.join(d, sub, "**", "*counter_collection.csv"), counter)
        f = frames(seq, warmup)
        return (mean([x["trace"] + x["coop"] + x["order"] for x in f]), mean([x["trace"] + x["coop"] for x in f]),
                mean([x["build"] for x in f]))

    def per_stage(fr):
        keys = sorted({k for x in fr for k in x["stages"]})
        return {k: mean([x["stages"].get(k, 0.0) for x in fr]) for k in keys}

    fetch = per_frame("fetch", "FETCH_SIZE")
    write = per_frame("write", "WRITE_SIZE")
    valu = per_frame("sq", "SQ_INSTS_VALU")
    grbm = per_frame("sq", "GRBM_GUI_ACTIVE")
    waves = per_frame("sq", "SQ_WAVES")
    wcyc = per_frame("sq", "SQ_WAVE_CYCLES")
    wait = per_frame("sq", "SQ_WAIT_ANY")
    thr = per_frame("sq", "SQ_THREAD_CYCLES_VALU")
    act = per_frame("sq", "SQ_ACTIVE_INST_VALU")

    st_us = per_stage(ft)
    st_f = per_stage(frames(dispatches(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE"),
                            warmup))
    st_w = per_stage(frames(dispatches(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE"),
                            warmup))
    build_stages = {k: {"us": st_us[k], "hbm_bytes": (2 * st_f[k] + st_w[k]) * 1024
                        if k in st_f and k in st_w else None, "algo_bytes_per_prim": STAGE_ALGO_BPP.get(k)}
                    for k in st_us}
    hbm = 2 * fetch[0] * 1024 + write[0] * 1024 if fetch[0] is not None and write[0] is not None else None
    bhbm = 2 * fetch[2] * 1024 + write[2] * 1024 if fetch[2] is not None and write[2] is not None else None
    cyc = grbm[1] / 8 if grbm[1] else None
    try:
        tree = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).stdout.strip()
    except Exception:
        tree = "?"
    entry = {
        "config": cfg, "n_gpus": ngpu, "tag": tag, "tree": tree, "kernel": kname, "timed_frames": len(ft),
        "trace_kernel_avg_us": trace_us, "coop_kernel_avg_us": coop_us, "tile_order_avg_us": order_us,
        "build_kernel_sum_ms": build_us / 1e3
        if build_us is not None else None,
        "hbm_bytes_per_launch": hbm, "fetch_kib_raw": fetch[0], "write_kib": write[0],
        "build_hbm_bytes": bhbm, "build_stages": build_stages,
        "valu_insts_per_launch": valu[1], "cycles_per_launch": cyc,
        "cycles_vs_duration_at_2p4ghz": cyc / (trace_us * 2400.0) if cyc and trace_us else None,
        "waves": waves[1], "wait_any_frac": wait[1] / wcyc[1] if wait[1] and wcyc[1] else None,
        "valu_lane_util": thr[1] / (64.0 * act[1]) if thr[1] and act[1] else None,
        "note": "per timed trace launch (k_tile_order + k_trace + k_trace_coop; trace_kernel_avg_us and VALU/cycles: "
                "k_trace + k_trace_coop); hbm = 2*FETCH_SIZE + "
                "WRITE_SIZE (KiB x 1024, gfx950 read correction); cycles = GRBM_GUI_ACTIVE / 8 XCDs",
    }
    jp = os.path.join("profiles", "pmc_summary.json")
    try:
        pj = json.load(open(jp))
    except Exception:
        pj = {"entries": []}
    pj["entries"] = [e for e in pj["entries"] if not (e["config"] == cfg and e.get("n_gpus", 1) == ngpu)]
    pj["entries"].append(entry)
    json.dump(pj, open(jp, "w"), indent=1)

    # markdown: every kernel of the kernel-trace pass + per-dispatch PMC
    dur = defaultdict(list)
    for _, k, v in tr:
        dur[k].append(v)
    pm = {}
    for sub, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"), ("sq", "SQ_INSTS_VALU")):
        acc = defaultdict(list)
        for _, k, v in dispatches(os.path.join(d, sub, "**", "*counter_collection.csv"), c):
            acc[k].append(v)
        pm[c] = {k: mean(v) for k, v in acc.items()}
    L = [f"# rocprofv3 summary {tag}: {cfg}, {ngpu} GPU", "",
         f"command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --only-timed ...` (+ one `--pmc` pass "
         f"each for FETCH_SIZE, WRITE_SIZE and the SQ group), tree {tree}; warm-up frames dropped: {warmup}", "",
         "## timed frames (means per frame)", "",
         f"- trace kernels `{kname}` + k_trace_coop: {trace_us:.2f} us (k_trace_coop {coop_us:.2f}); "
         f"k_tile_order {order_us:.2f} us" if trace_us else "- none",
         f"- build kernels (sum): {build_us:.2f} us" if build_us else "",
         ("- build stages (per build: us, PMC HBM bytes): " + "; ".join(
             f"{k} {v['us']:.2f} us {v['hbm_bytes']:.4g} B" for k, v in build_stages.items()
             if v["hbm_bytes"] is not None)) if build_stages else "",
         f"- HBM bytes per trace launch (PMC): {hbm:.4g}; per build: {bhbm:.4g}" if hbm and bhbm else "",
         f"- VALU wave-instructions per trace launch: {valu[1]:.4g}; cycles (GRBM/8): {cyc:.4g}; "
         f"issue fraction {valu[1] / (512 * cyc):.3f}" if valu[1] and cyc else "",
         "", "## all kernels", "",
         "| kernel | calls | avg us | min us | max us | FETCH KiB | WRITE KiB | HBM bytes (2F+W) | VALU insts |",
         "|---|---|---|---|---|---|---|---|---|"]
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        f = pm["FETCH_SIZE"].get(k)
        w = pm["WRITE_SIZE"].get(k)
        va = pm["SQ_INSTS_VALU"].get(k)
        hb = f"{(2 * f + w) * 1024:.4g}" if f is not None and w is not None else "-"
        L.append(f"| {k} | {len(v)} | {mean(v):.2f} | {min(v):.2f} | {max(v):.2f} | "
                 f"{f if f is None else round(f, 1)} | {w if w is None else round(w, 1)} | {hb} | "
                 f"{'-' if va is None else f'{va:.4g}'} |")
    # the LDS/issue pass (gpu_run.sh pmclds), when it ran
    LDSC = ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES",
            "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY")
    if glob.glob(os.path.join(d, "lds", "**", "*counter_collection.csv"), recursive=True):
        lp = {}
        for c in LDSC:
            acc = defaultdict(list)
            for _, k, v in dispatches(os.path.join(d, "lds", "**", "*counter_collection.csv"), c):
                acc[k].append(v)
            lp[c] = {k: mean(v) for k, v in acc.items()}
        L += ["", "## LDS / issue counters per dispatch (gpu_run.sh pmclds; SQ cycle counters in quad-cycles)", "",
              "| kernel | LDS insts | bank-conflict cycles | LDS array cycles | conflict frac | WAIT_INST_LDS | "
              "SALU insts | WAIT_ANY / WAVE_CYCLES |", "|---|---|---|---|---|---|---|---|"]
        for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            g = {c: lp[c].get(k) for c in LDSC}
            if g["SQ_INSTS_LDS"] is None:
                continue
            cf = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_LDS_IDX_ACTIVE"] if g["SQ_LDS_IDX_ACTIVE"] else None
            wf = g["SQ_WAIT_ANY"] / g["SQ_WAVE_CYCLES"] if g["SQ_WAVE_CYCLES"] else None
            fmt = lambda x: "-" if x is None else f"{x:.4g}"
            L.append(f"| {k} | {fmt(g['SQ_INSTS_LDS'])} | {fmt(g['SQ_LDS_BANK_CONFLICT'])} | "
                     f"{fmt(g['SQ_LDS_IDX_ACTIVE'])} | {fmt(cf)} | {fmt(g['SQ_WAIT_INST_LDS'])} | "
                     f"{fmt(g['SQ_INSTS_SALU'])} | {fmt(wf)} |")
    open(os.path.join("profiles", f"rocprof_{tag}.md"), "w").write("\n".join(x for x in L if x is not None) + "\n")
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
