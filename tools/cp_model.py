"""CPU model of a children-parallel heavy-ray step for one rank's share of an
8-GPU soup-1M 1080p1 frame, from the per-pixel step
counts of tools/step_dump.py (gpurun_out/steps_<k>.npz) and the measured step
split of tools/diag_steps.py (profiles/diag_steps_r06.log).

Per-lane kernel (today): a wave = an 8x8 quadrant (64 rays), a wave's pass 1
lasts its slowest ray's min(steps, cap) steps.  Children-parallel: 4 lanes
per ray, a wave = a 4x4 block (16 rays), the record test split over the
lanes (one child each), the leaf test and the pop unchanged.  Projected pass
1 = max(critical path, issue throughput), where
  critical path = max over the rank's waves of its slowest ray's capped steps
                  x the step latency of a lone wave;
  issue         = sum over waves of capped max steps x VALU per step /
                  (1024 SIMDs x 0.5 wave-instructions per cycle).
usage: python tools/cp_model.py [steps npz ...]"""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GHZ = 2.33            # the rank kernel's clock in profiles/diag_steps_r06.log
STEP = {"pop": 445, "wait": 439, "rest": 1750}   # cycles per heavy step, measured (stamped)
LEAF_VALU, REC_VALU, OTHER_VALU = 117, 136, 30    # the tile kernel's loop blocks (tools/isa_blocks.py)
REC_VALU_CP = 65      # one child + the per-record setup + ballot ranking + one push (estimate)
files = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "steps_*.npz")))
for f in files:
    d = np.load(f)
    st = d["steps"].astype(np.int64)
    w, h = int(d["w"]), int(d["h"])
    nb = ((w + 15) // 16) * ((h + 15) // 16)
    T = st.reshape(nb, 16, 16)
    valu_lane = LEAF_VALU + REC_VALU + OTHER_VALU
    valu_cp = LEAF_VALU + REC_VALU_CP + OTHER_VALU
    rest_cp = STEP["rest"] * (valu_cp / valu_lane)
    step_lane = sum(STEP.values())
    step_cp = STEP["pop"] + STEP["wait"] + rest_cp
    for cap in (72,):
        crit, issue, crit_cp, issue_cp = [], [], [], []
        for r in range(8):
            t = T[r::8]
            q = np.minimum(t.reshape(-1, 2, 8, 2, 8).transpose(0, 1, 3, 2, 4).reshape(-1, 64).max(1), cap)
            b = np.minimum(t.reshape(-1, 4, 4, 4, 4).transpose(0, 1, 3, 2, 4).reshape(-1, 16).max(1), cap)
            crit.append(q.max() * step_lane / GHZ / 1e3)
            crit_cp.append(b.max() * step_cp / GHZ / 1e3)
            issue.append(q.sum() * valu_lane / 512 / GHZ / 1e3)
            issue_cp.append(b.sum() * valu_cp / 512 / GHZ / 1e3)
        print(f"{os.path.basename(f)} cap {cap}: per-lane pass 1 critical {max(crit):.1f} us, issue {max(issue):.1f} us; "
              f"children-parallel: step {step_cp:.0f} vs {step_lane} cycles ({step_cp / step_lane:.2f}), critical "
              f"{max(crit_cp):.1f} us, issue {max(issue_cp):.1f} us (wave-steps x{np.sum(issue_cp) / np.sum(issue) * valu_lane / valu_cp:.2f})")
