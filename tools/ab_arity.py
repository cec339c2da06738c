"""A/B of the wide-record arity (build.wide_arity 4 vs 8) on soup-1M 1080p:
build time, the bench's moving-camera full frames (event-timed trace per
frame, mean), and one rank's tiles at P = 2/4/8 (max over ranks, medians),
interleaved rounds; both scenes' images are checked identical.
usage: python tools/ab_arity.py [rounds] [frames] [n] [knob=value ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
import bench  # noqa: E402

a = [x for x in sys.argv[1:] if "=" not in x]
for kv in [x for x in sys.argv[1:] if "=" in x]:
    k, v = kv.split("=")
    R.config_set(k, int(v))
    print(f"{k} = {v}", flush=True)
rounds = int(a[0]) if len(a) > 0 else 3
frames = int(a[1]) if len(a) > 1 else 12
n = int(a[2]) if len(a) > 2 else 1_000_000
view = S.VIEWS["soup"]
w, h, spp = 1920, 1080, 1
scenes = {}
for ar in (4, 8):
    R.config_set("build.wide_arity", ar)
    sc = R.Scene.generate_soup(n, 1)
    sc.build()
    assert sc.wide_arity == ar
    scenes[ar] = sc
R.config_set("build.wide_arity", 4)
cams = [R.camera_look_at(bench.orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames + 2)]
img = {ar: torch.zeros(w * h, dtype=torch.int32, device="cuda") for ar in (4, 8)}
Ps = (2, 4, 8)
res = {(ar, k): [] for ar in (4, 8) for k in ("build", "moving", "static") + Ps}
for _ in range(rounds):
    for ar, sc in scenes.items():
        R.config_set("build.wide_arity", ar)
        res[(ar, "build")].append(np.median([sc.build() for _ in range(5)]))
        sc.render_device(cams[0], w, h, spp, d_rgba=img[ar].data_ptr(), timed=True)
        sc.render_device(cams[1], w, h, spp, d_rgba=img[ar].data_ptr(), timed=True)
        t = [sc.render_device(cams[2 + i], w, h, spp, d_rgba=img[ar].data_ptr(), timed=True) for i in range(frames)]
        res[(ar, "moving")].append(float(np.mean(t)))
        t = [sc.render_device(cams[0], w, h, spp, d_rgba=img[ar].data_ptr(), timed=True) for i in range(6)]
        res[(ar, "static")].append(float(np.median(t[2:])))
        for P in Ps:
            t = []
            for r in range(P):
                slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
                t.append(np.median([sc.render_tiles_device(cams[0], w, h, spp, r, P, slab.data_ptr(), timed=True)
                                    for _ in range(5)][1:]))
            res[(ar, P)].append(max(t))
    assert torch.equal(img[4], img[8]), "arity changed the image"
R.config_set("build.wide_arity", 4)
print(f"n={n} {w}x{h}x{spp}, {rounds} rounds; moving = mean of {frames} orbiting frames; P = max over ranks", flush=True)
for ar in (4, 8):
    print(f"arity {ar}: build {np.median(res[(ar, 'build')]):.4f} ms | moving {np.median(res[(ar, 'moving')]):.4f} ms"
          f" | static {np.median(res[(ar, 'static')]):.4f} ms |"
          + "".join(f" P={P}: {np.median(res[(ar, P)]):.4f} ms" for P in Ps), flush=True)
