"""A/B the path-mode kernel configurations in ONE process, interleaved rounds.
usage: python tools/ab_path.py [rounds] [scene: soup|sponza|bunny] [depth]
Prints per configuration the median launch time, rays traced (kernel
counters) and Mrays/s; asserts every configuration renders the same image."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
scene = sys.argv[2] if len(sys.argv) > 2 else "soup"
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
w, h, spp = 1920, 1080, 1
tris = S.tris_for(scene, 1_000_000 if scene == "soup" else 0)
s = R.Scene.generate_soup(1_000_000, 1) if tris is None else R.Scene.from_soup(tris)
s.build()
V, light = S.VIEWS[scene], S.LIGHTS[scene]
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
variants = [("wide, 256-thread tiles", {"trace.variant": 0, "trace.wg": 256}),
            ("wide, 64-thread quadrants", {"trace.variant": 0, "trace.wg": 64}),
            ("binary, 256-thread tiles", {"trace.variant": 2, "trace.wg": 256})]
rays = {}
for name, cfg in variants:
    for k, v in cfg.items():
        R.config_set(k, v)
    rays[name] = [int(c) for c in s.render_path_work(cam, w, h, spp, light, 0.3, depth)]
    print(name, "work (node records, tri records, rays):", rays[name])
ref = None
times = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, cfg in variants:
        for k, v in cfg.items():
            R.config_set(k, v)
        ms = [s.render_path_device(cam, w, h, spp, light, 0.3, depth, d_rgba=img.data_ptr(), timed=True)
              for _ in range(3)]
        times[name].append(min(ms))
        out = img.cpu().numpy().view(np.uint32)
        if ref is None:
            ref = out.copy()
        assert np.array_equal(out, ref), name
for name, _ in variants:
    t = np.array(times[name])
    print(f"{scene} depth {depth} {name:<28s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  "
          f"rays {rays[name][2]}  -> {rays[name][2] / np.median(t) / 1e3:8.1f} Mrays/s")
R.config_set("trace.variant", 0)
R.config_set("trace.wg", 256)
