"""Per-rank trace times at P = 2/4/8 (one GPU standing in for each rank, soup-1M
1080p, static camera, medians of 5 after 1 warm frame): how far the slowest
rank is from the others.  usage: python tools/rank_spread.py [knob=value ...]"""
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

for kv in [x for x in sys.argv[1:] if "=" in x]:
    k, v = kv.split("=")
    R.config_set(k, int(v))
    print(f"{k} = {v}", flush=True)
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
for P in (2, 4, 8):
    t = []
    for r in range(P):
        slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
        t.append(np.median([s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True)
                            for _ in range(6)][1:]))
    print(f"P={P}: " + " ".join(f"{x:.4f}" for x in t) + f" | max {max(t):.4f} mean {np.mean(t):.4f}", flush=True)
