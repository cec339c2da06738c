"""Experiment (diagnostic build): does dispatching the costliest tiles first
shorten the frame?  Measures per-tile wave durations of one frame (stamps),
derives the longest-first order, and times the frame with and without it.
usage: python tools/lpt_exp.py [rounds]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_LIB"] = os.path.join(ROOT, "gpu_raytracer_amd", "lib", "librtamd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

L = R.lib()
L.rt_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
L.rt_debug_tile_order.argtypes = [C.c_void_p]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
w, h = 1920, 1080
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
R.config_set("trace.tile_order", 0)
for _ in range(3):
    s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
ref = img.cpu().numpy().copy()
nb = ((w + 15) // 16) * ((h + 15) // 16)
buf = np.zeros(nb * 16, np.uint64)
assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(nb * 4, 4).astype(np.int64)
dur = (st[:, 1] - st[:, 0]).reshape(nb, 4).max(1) / 100.0  # per tile: slowest wave, us
order = np.argsort(-dur, kind="stable").astype(np.int32)
print(f"tile cost us: median {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}; "
      f"tiles > 100 us: {(dur > 100).sum()}")
rng = np.random.default_rng(0)
orders = {
    "row-major": None,
    "measured longest-first": np.argsort(-dur, kind="stable"),
    "heavy>100us first, stable": np.argsort(-(dur > 100).astype(np.int64), kind="stable"),
    "random": rng.permutation(nb),
}
dev = {k: (torch.from_numpy(v.astype(np.int32)).cuda() if v is not None else None) for k, v in orders.items()}
res = {}
for r in range(rounds):
    for k, o in dev.items():
        L.rt_debug_tile_order(C.c_void_p(o.data_ptr()) if o is not None else None)
        ms = [s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True) for _ in range(3)]
        res.setdefault(k, []).append(min(ms))
        assert np.array_equal(img.cpu().numpy(), ref), k
    L.rt_debug_tile_order(None)
    R.config_set("trace.tile_order", 1)
    ms = [s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True) for _ in range(3)]
    res.setdefault("device cost map (previous frame)", []).append(min(ms))
    assert np.array_equal(img.cpu().numpy(), ref)
    R.config_set("trace.tile_order", 0)
L.rt_debug_tile_order(None)
R.config_set("trace.tile_order", 1)
for k, v in res.items():
    print(f"{k:<28s} median {np.median(v):.3f} ms  min {min(v):.3f}")
