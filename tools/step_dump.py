"""Dump the per-pixel wide-traversal step counts of one full soup-1M 1080p1
frame on the bench's orbiting camera (queue off, so every ray's full count;
rt_render_step_map, tile-slot-major: slot * 256 + ly * 16 + lx) to
gpurun_out/steps_<orbit>.npz, for the CPU scheduling model of one rank's
share (tools/cp_model.py).  usage: python tools/step_dump.py [orbit step=8]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
from bench import orbit_view  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = S.CONFIGS[3]
v = S.VIEWS[cfg.scene]
w, h, spp = cfg.w, cfg.h, cfg.spp
R.config_set("trace.coop_cap", 0)
s = R.Scene.generate_soup(cfg.n, 1)
s.build()
cam = R.camera_look_at(orbit_view(v, k), v.at, v.up, v.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
for _ in range(2):
    ms = s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True)
st = s.step_map(w, h, spp)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"steps_{k}.npz"), steps=st, w=w, h=h, frame_ms=ms)
print(f"frame {ms:.4f} ms (queue off); rays {int((st > 0).sum())}, max steps {int(st.max())}, total {int(st.sum())}")
s.close()
