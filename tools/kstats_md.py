"""Summarise tools/gpu_run.sh `kstats` runs (rocprofv3 --kernel-trace --stats,
or one --pmc pass) into a markdown file under profiles/.
usage: python tools/kstats_md.py OUT.md TITLE gpurun_out/ks_<tag> [gpurun_out/ks_<tag2> ...]
Per run: the command it profiled, then either the kernel stats table or the
per-kernel means of every collected counter (with the LDS conflict share
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE and SQ_WAIT_ANY / SQ_WAVE_CYCLES
when present)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"^void ", "", name.split("(")[0])[:56]


def main():
    out, title, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    L = [f"# {title}", ""]
    for d in dirs:
        log = os.path.join(d, "run.log")
        cmd = "?"
        if os.path.exists(log):
            for line in open(log):
                m = re.search(r"'(python3 [^']*)'", line)
                if m:
                    cmd = m.group(1)
                    break
            res = [x.strip() for x in open(log) if "n=" in x and "us:" in x]
        else:
            res = []
        L += [f"## {os.path.basename(d)}", "", f"command: `rocprofv3 ... -- {cmd}`", ""]
        if res:
            L += ["result line: `" + res[-1] + "`", ""]
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if stats:
            L += ["| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
            for r in csv.DictReader(open(stats[0])):
                L.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                         f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} |")
        if cc:
            acc = defaultdict(lambda: defaultdict(list))
            for f in cc:
                per = defaultdict(lambda: defaultdict(float))
                for r in csv.DictReader(open(f)):
                    per[(short(r["Kernel_Name"]), r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                for (k, _), c in per.items():
                    for cn, v in c.items():
                        acc[k][cn].append(v)
            cols = sorted({cn for k in acc for cn in acc[k]})
            extra = []
            if "SQ_LDS_BANK_CONFLICT" in cols and "SQ_LDS_IDX_ACTIVE" in cols:
                extra.append("conflict/LDS cycles")
            if "SQ_WAIT_ANY" in cols and "SQ_WAVE_CYCLES" in cols:
                extra.append("WAIT_ANY/WAVE_CYCLES")
            L += ["per-dispatch means (SQ cycle counters in quad-cycles, summed over the XCDs)", "",
                  "| kernel | " + " | ".join(cols + extra) + " |", "|---" * (len(cols) + len(extra) + 1) + "|"]
            key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in cols else cols[0]
            for k, c in sorted(acc.items(), key=lambda kv: -sum(kv[1].get(key, [0]))):
                m = {cn: sum(v) / len(v) for cn, v in c.items()}
                row = [f"{m.get(cn, 0):.4g}" for cn in cols]
                if "conflict/LDS cycles" in extra:
                    row.append(f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 0), 1):.3f}")
                if "WAIT_ANY/WAVE_CYCLES" in extra:
                    row.append(f"{m.get('SQ_WAIT_ANY', 0) / max(m.get('SQ_WAVE_CYCLES', 0), 1):.3f}")
                L.append(f"| {k} | " + " | ".join(row) + " |")
        L.append("")
    open(out, "w").write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()
