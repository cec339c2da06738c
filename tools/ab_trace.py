"""A/B the trace-kernel variants in ONE process, interleaved rounds (guide
§5.4 rule 24).  usage: python tools/ab_trace.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
variants = [("simple", {"trace.variant": 0})]
for rm in (1, 8, 16, 32, 48):
    for blocks in (1024, 2048):
        variants.append((f"persist refill>={rm} blocks={blocks}", {"trace.variant": 1, "trace.refill_min": rm, "trace.blocks": blocks}))
ref = None
times = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, cfg in variants:
        for k, v in cfg.items():
            R.config_set(k, v)
        ms = [s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True) for _ in range(3)]
        times[name].append(min(ms))
        out = img.cpu().numpy()
        if ref is None:
            ref = out.copy()
        assert np.array_equal(out, ref), name
for name, _ in variants:
    t = np.array(times[name])
    print(f"{name:<36s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  -> {w*h*spp/np.median(t)/1e3:8.1f} Mrays/s")
