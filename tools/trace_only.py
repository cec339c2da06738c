"""Trace-only driver for PMC profiling: build once, render K frames."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 5
if len(sys.argv) > 2:
    R.config_set("trace.variant", int(sys.argv[2]))
w, h = 1920, 1080
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
for _ in range(k):
    print(s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True))
