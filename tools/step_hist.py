"""Distribution of per-ray wide-traversal steps (rt_render_step_map) for one
config's static frame: percentiles, rays over step caps, remainder work above
each cap, per-tile maxima.  usage: python tools/step_hist.py [config key]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

key = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = S.CONFIGS[key]
v = S.VIEWS[cfg.scene]
s = R.Scene.generate_soup(cfg.n, 1) if cfg.scene == "soup" else R.Scene.from_soup(S.tris_for(cfg.scene))
s.build()
w, h, spp = cfg.w, cfg.h, cfg.spp
cam = R.camera_look_at(v.eye, v.at, v.up, v.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
for _ in range(3):
    ms = s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True)
st = s.step_map(w, h, spp).astype(np.int64)
tiles = st.reshape(-1, 256)
valid = st[st > 0]
print(f"{cfg.name} {w}x{h}x{spp}: frame {ms:.4f} ms, rays(px) {valid.size}, total steps {valid.sum()}")
print("percentiles 50/90/99/99.9/99.99/max:", [int(np.percentile(valid, q)) for q in (50, 90, 99, 99.9, 99.99)], int(valid.max()))
for cap in (16, 24, 32, 48, 64, 96, 128):
    over = valid[valid > cap]
    print(f"cap {cap:4d}: rays over {over.size:8d} ({over.size / valid.size:.4%}), remainder steps {(over - cap).sum():10d}"
          f" ({(over - cap).sum() / valid.sum():.2%} of all), max remainder {int(over.max() - cap) if over.size else 0}")
tm = tiles.max(axis=1)
print("per-tile max steps percentiles 50/90/99/max:", [int(np.percentile(tm, q)) for q in (50, 90, 99)], int(tm.max()))
hist = np.bincount(np.minimum(valid, 400) // 10)
print("histogram (10-step bins, count):", " ".join(f"{i*10}:{c}" for i, c in enumerate(hist) if c))
