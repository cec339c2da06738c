"""One summary line of a tools/rank_emul.py JSON block on stdin: the full
frame and every P's max-rank time and efficiency.  usage: ... | python tools/emul_line.py TAG"""
import json
import sys

d = json.load(sys.stdin)
tag = sys.argv[1] if len(sys.argv) > 1 else ""
parts = [f"P{k} max {v['max_ms']:.4f} mean {v['mean_ms']:.4f} eff {v['efficiency']:.3f}" for k, v in d["P"].items()]
print(f"{tag}: full {d['full_frame_ms']:.4f}  " + "  ".join(parts), flush=True)
