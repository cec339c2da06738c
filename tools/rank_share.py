"""One GPU standing in for each rank of a P-GPU run: the tiled trace of every
rank r < P (tiles t = r mod P), per kernel configuration.  Reports the max
over ranks (what bench.py's value divides by) against the ideal full/P.
usage: python tools/rank_share.py [n] [w] [h] [spp]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 1
s = R.Scene.generate_soup(n, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
configs = [("row-major 256", {"trace.variant": 0, "trace.wg": 256, "trace.wg_tiles": 256, "trace.tile_order": 0}),
           ("row-major 64", {"trace.variant": 0, "trace.wg": 64, "trace.wg_tiles": 64, "trace.tile_order": 0}),
           ("ordered 256", {"trace.variant": 0, "trace.wg": 256, "trace.wg_tiles": 256, "trace.tile_order": 1}),
           ("ordered 64", {"trace.variant": 0, "trace.wg": 64, "trace.wg_tiles": 64, "trace.tile_order": 1})]
for name, cfg in configs:
    for k, v in cfg.items():
        R.config_set(k, v)
    full = np.median([s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True) for _ in range(6)][1:])
    line = f"{name:<14s} full {full:.3f} ms |"
    for P in (2, 4, 8):
        t = []
        for r in range(P):
            tpr = R.tiles_for_rank(w, h, r, P)
            slab = torch.zeros(max(tpr, 1) * 256, dtype=torch.int32, device="cuda")
            t.append(np.median([s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True)
                                for _ in range(5)][1:]))
        line += f" P={P}: max {max(t):.3f} ms (ideal {full / P:.3f}, eff {full / P / max(t):.2f})"
    print(line, flush=True)
R.config_set("trace.variant", 0)
R.config_set("trace.wg", 256)
R.config_set("trace.wg_tiles", 64)
R.config_set("trace.tile_order", 1)
