"""Per-wave timeline of the pool trace kernel (diag build, -DRT_STAMPS)."""
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
L.rt_debug_stamps.restype = C.c_int
w, h = 1920, 1080
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 0
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
R.config_set("trace.variant", 1)
R.config_set("trace.blocks", blocks)
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
for _ in range(3):
    ms = s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
print("render ms", ms)
nw = 8192 * 4 if not blocks else blocks * 4
buf = np.zeros(nw * 4, np.uint64)
assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(nw, 4).astype(np.int64)
st = st[st[:, 1] > 0]
t0 = st[:, 0].min()
a = (st[:, 0] - t0) / 100.0
b = (st[:, 1] - t0) / 100.0
d = b - a
it = st[:, 3] & 0xFFFF
fbk = st[:, 3] >> 32
print(f"waves {len(d)} span {b.max():.1f} us; start last {a.max():.1f} us; dur median {np.median(d):.1f} p90 {np.percentile(d,90):.1f} max {d.max():.1f}")
print(f"iterations per wave median {np.median(it):.0f} p90 {np.percentile(it,90):.0f} max {it.max()}; us/iter median {np.median(d/np.maximum(it,1)):.3f}")
tgrid = np.linspace(0, b.max(), 31)
print("live:", " ".join(f"{t:.0f}:{int(((a <= t) & (b > t)).sum())}" for t in tgrid))
print("fallback rays total", fbk.sum(), "waves with fallback", (fbk > 0).sum())
o = np.argsort(-d)[:10]
for i in o:
    print(f"  dur {d[i]:.1f} iters {it[i]} fallbacks {fbk[i]} start {a[i]:.1f}")
