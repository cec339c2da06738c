"""Cooperative heavy rays (trace.coop_cap / trace.coop_cap_tiles): trace time
of the full frame and the max-over-ranks per-rank time at P = 2, 4, 8 (one GPU
standing in for each rank) for a sweep of step caps, interleaved rounds.
usage: python tools/coop_sweep.py [n] [w] [h] [spp] [rounds] [caps...] [knob=value...]
(knob=value pairs are applied with rt_config_set before the sweep)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

a = [x for x in sys.argv[1:] if "=" not in x]
for kv in [x for x in sys.argv[1:] if "=" in x]:
    k, v = kv.split("=")
    R.config_set(k, int(v))
    print(f"{k} = {v}", flush=True)
n = int(a[0]) if len(a) > 0 else 1_000_000
w = int(a[1]) if len(a) > 1 else 1920
h = int(a[2]) if len(a) > 2 else 1080
spp = int(a[3]) if len(a) > 3 else 1
rounds = int(a[4]) if len(a) > 4 else 3
caps = [int(c) for c in a[5:]] or [0, 32, 48, 64, 96, 128]
s = R.Scene.generate_soup(n, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
Ps = (2, 4, 8)
res = {(c, P): [] for c in caps for P in (1,) + Ps}
for _ in range(rounds):
    for c in caps:
        R.config_set("trace.coop_cap", c)
        R.config_set("trace.coop_cap_tiles", c)
        full = np.median([s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True) for _ in range(6)][1:])
        res[(c, 1)].append(full)
        for P in Ps:
            t = []
            for r in range(P):
                slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
                t.append(np.median([s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True)
                                    for _ in range(5)][1:]))
            res[(c, P)].append(max(t))
print(f"n={n} {w}x{h}x{spp}, {rounds} rounds (medians); per-rank = max over ranks", flush=True)
for c in caps:
    f = np.median(res[(c, 1)])
    print(f"cap {c:4d}: full {f:.4f} ms |" + "".join(
        f" P={P}: {np.median(res[(c, P)]):.4f} ms (eff {np.median(res[(0, 1)]) / P / np.median(res[(c, P)]):.2f})"
        for P in Ps), flush=True)
R.config_set("trace.coop_cap", 0)
R.config_set("trace.coop_cap_tiles", 0)
