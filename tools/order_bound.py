"""How much of the moving-camera frame time is the tile/pixel order's
staleness?  The bench's orbiting sequence (soup-1M 1080p) timed three ways:
(a) as the bench runs it (order from the previous, 0.25 deg older frame),
(b) each frame rendered twice and the second timed (tile and pixel order from
the same camera: the order's upper bound), (c) row-major (no order).
usage: python tools/order_bound.py [frames] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
import bench  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 16
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
view = S.VIEWS["soup"]
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cams = [R.camera_look_at(bench.orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames + 2)]
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
res = {"stale": [], "same_cam": [], "same_cam_tiles_only": [], "row_major": []}
for _ in range(rounds):
    R.config_set("trace.tile_order", 1)
    for c in cams[:2]:
        s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True)
    res["stale"].append(np.mean([s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True) for c in cams[2:]]))
    t = []
    for c in cams[2:]:
        s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True)
        t.append(s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True))
    res["same_cam"].append(np.mean(t))
    R.config_set("trace.px_sort", 0)
    t = []
    for c in cams[2:]:
        s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True)
        t.append(s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True))
    res["same_cam_tiles_only"].append(np.mean(t))
    R.config_set("trace.px_sort", 1)
    R.config_set("trace.tile_order", 0)
    res["row_major"].append(np.mean([s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True) for c in cams[2:]]))
    R.config_set("trace.tile_order", 1)
    R.config_set("trace.tile_order", 1)
for k, v in res.items():
    print(f"{k:10s} {np.median(v):.4f} ms  (rounds: {' '.join(f'{x:.4f}' for x in v)})", flush=True)
