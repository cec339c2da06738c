"""Per-rank trace time (max over ranks; one GPU stands in for each rank) at
P = 1, 2, 4, 8 for several tile-kernel configurations, interleaved rounds.
usage: python tools/rank_configs.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
configs = {"wg64": {"trace.wg_tiles": 64, "trace.px_sort": 1},
           "wg256": {"trace.wg_tiles": 256, "trace.px_sort": 1},
           "wg256+px": {"trace.wg_tiles": 256, "trace.px_sort": 2}}
res = {(c, P): [] for c in configs for P in (2, 4, 8)}
for _ in range(rounds):
    for name, cfg in configs.items():
        for k, v in cfg.items():
            R.config_set(k, v)
        for P in (2, 4, 8):
            t = []
            for r in range(P):
                slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
                t.append(np.median([s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True)
                                    for _ in range(5)][1:]))
            res[(name, P)].append(max(t))
for name in configs:
    print(f"{name:<10s}", "  ".join(f"P={P}: {np.median(res[(name, P)]):.4f} ms" for P in (2, 4, 8)), flush=True)
R.config_set("trace.wg_tiles", 64)
R.config_set("trace.px_sort", 1)
