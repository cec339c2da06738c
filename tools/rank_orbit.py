"""Per-rank trace times at P = 2/4/8 on the bench's ORBITING camera (0.25 deg
per frame, so every frame differs and the tile/pixel maps are one frame
stale), one GPU standing in for each rank in turn, soup-1M 1080p1: for each
rank, `frames` successive frames of its tiles, median of the frames after
the first two; prints every rank's median and the max / mean over ranks.
usage: python tools/rank_orbit.py [frames] [knob=value ...]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
for _a in [x for x in sys.argv[1:] if x.startswith("lib=")]:  # a librtamd variant (tools/build_exp.sh)
    os.environ["RT_LIB"] = os.path.join(ROOT, _a[4:])
    sys.argv.remove(_a)
    print("lib", os.environ["RT_LIB"], flush=True)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 10
for kv in [x for x in sys.argv[1:] if "=" in x]:
    k, v = kv.split("=")
    R.config_set(k, int(v))
    print(f"{k} = {v}", flush=True)


def orbit(step, deg=0.25):
    a = math.radians(deg * step)
    ex, ey, ez = (e - c for e, c in zip(V.eye, V.at))
    return (V.at[0] + ex * math.cos(a) + ez * math.sin(a), V.at[1] + ey, V.at[2] - ex * math.sin(a) + ez * math.cos(a))


w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
for P in (2, 4, 8):
    t = []
    for r in range(P):
        slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
        ms = []
        for f in range(frames):
            cam = R.camera_look_at(orbit(f), V.at, V.up, V.vfov, w, h)
            ms.append(s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True))
        t.append(float(np.median(ms[2:])))
        if os.environ.get("RO_VERBOSE"):
            print(f"  P={P} rank {r}: " + " ".join(f"{x:.4f}" for x in ms), flush=True)
    print(f"P={P}: " + " ".join(f"{x:.4f}" for x in t) + f" | max {max(t):.4f} mean {np.mean(t):.4f}", flush=True)
