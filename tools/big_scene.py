"""Config-5 sizing (BASELINE.json configs[4]): 10M-triangle soup, 3840x2160x4.
Times the replicated build (per-stage), the full-frame trace on one GPU and
one rank's share of the tiled trace for P = 2, 4, 8 -- what decides whether a
distributed build would pay.
usage: python tools/big_scene.py [n] [w] [h] [spp]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
w = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
h = int(sys.argv[3]) if len(sys.argv) > 3 else 2160
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 4
s = R.Scene.generate_soup(n, 1)
builds = [s.build() for _ in range(6)][2:]
R.config_set("build.stage_events", 1)
s.build()
t = s.build_times()
R.config_set("build.stage_events", 0)
print(f"n={n}: build median {np.median(builds):.3f} ms ({n / np.median(builds) / 1e3:.0f} Mprims/s); stages ms: "
      f"bounds {t.bounds:.3f} morton {t.morton:.3f} sort {t.sort:.3f} topo+local refit {t.topology:.3f} "
      f"cross refit {t.refit:.3f}", flush=True)
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
ms = [s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True) for _ in range(5)][1:]
rays = w * h * spp
print(f"full frame {w}x{h}x{spp}: trace {np.median(ms):.3f} ms, {rays / np.median(ms) / 1e3:.0f} Mrays/s", flush=True)
for P in (2, 4, 8):
    tpr = R.tiles_for_rank(w, h, 0, P)
    slab = torch.zeros(max(tpr, 1) * 256, dtype=torch.int32, device="cuda")
    ms = [s.render_tiles_device(cam, w, h, spp, 0, P, slab.data_ptr(), timed=True) for _ in range(5)][1:]
    print(f"P={P}: rank 0 traces {tpr} tiles in {np.median(ms):.3f} ms; replicated build / trace = "
          f"{np.median(builds) / np.median(ms):.2f}", flush=True)
