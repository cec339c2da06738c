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
def cfg(variant=0, wg=256, wave=0, sort=0):
    return {"trace.variant": variant, "path.wg": wg, "path.wavefront": wave, "path.sort": sort}


variants = [("mega wide, 256-thread tiles", cfg()),
            ("mega wide, 64-thread quadrants", cfg(wg=64)),
            ("mega binary, 256-thread tiles", cfg(variant=2)),
            ("wavefront wide, unsorted", cfg(wave=1, sort=0)),
            ("wavefront wide, sort 1 byte", cfg(wave=1, sort=1)),
            ("wavefront wide, sort 2 bytes", cfg(wave=1, sort=2)),
            ("wavefront wide, sort 3 bytes", cfg(wave=1, sort=3)),
            ("wavefront wide, sort 4 bytes", cfg(wave=1, sort=4))]
if len(sys.argv) > 4:
    variants = [variants[int(i)] for i in sys.argv[4].split(",")]
rays = {}
for name, c in variants:
    for k, v in c.items():
        R.config_set(k, v)
    rays[name] = [int(c) for c in s.render_path_work(cam, w, h, spp, light, 0.3, depth)]
    print(name, "work (node records, tri records, rays):", rays[name])
ref = None
times = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, c in variants:
        for k, v in c.items():
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
    print(f"{scene} depth {depth} {name:<32s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  "
          f"rays {rays[name][2]}  -> {rays[name][2] / np.median(t) / 1e3:8.1f} Mrays/s")
for k, v in {"trace.variant": 0, "path.wg": 64, "path.wavefront": 0, "path.sort": 0}.items():
    R.config_set(k, v)
