"""Per-wave timeline of k_trace (diagnostic build librtamd_diag.so, -DRT_STAMPS).

Renders the headline frame (1M soup, 1920x1080x1) and reads each wave's
{start, end, HW_ID, XCC_ID}; prints the wave-duration distribution, the
number of live waves over time (occupancy) and the per-CU load balance.
"""
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
variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
if variant:
    R.config_set("trace.variant", variant)
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
for _ in range(3):
    ms = s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
print("render ms", ms)
nbq = ((w + 15) // 16) * ((h + 15) // 16)
cbuf = np.zeros(nbq * 16, np.uint64)
if len(sys.argv) > 2 and sys.argv[2] == "wide":
    s.render_work(cam, w, h, 1)  # the running (wide) kernel's own record counts
else:
    s.render_counters(cam, w, h, 1)  # binary traversal node counts
assert L.rt_debug_stamps(2, cbuf.ctypes.data, cbuf.nbytes) == 0
cst = cbuf.reshape(nbq * 4, 4).astype(np.int64)
mx = cst[:, 3] & 0xFFFFFFFF
sm = cst[:, 3] >> 32
for _ in range(3):
    ms = s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
nb = ((w + 15) // 16) * ((h + 15) // 16)
buf = np.zeros(nb * 16, np.uint64)
assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(nb * 4, 4).astype(np.int64)
t0 = st[:, 0].min()
a = (st[:, 0] - t0) / 100.0  # us
b = (st[:, 1] - t0) / 100.0
d = b - a
hw = st[:, 2] & 0xFFFFFFFF
xcc = (st[:, 2] >> 32) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
print(f"waves {len(d)} span {b.max():.1f} us; wave dur median {np.median(d):.1f} p10 {np.percentile(d,10):.1f} p90 {np.percentile(d,90):.1f} max {d.max():.1f}")
print(f"start: last wave starts at {a.max():.1f} us; ends: p50 {np.median(b):.1f} p90 {np.percentile(b,90):.1f}")
tgrid = np.linspace(0, b.max(), 41)
live = [int(((a <= t) & (b > t)).sum()) for t in tgrid]
print("live waves vs time (us:count):", " ".join(f"{t:.0f}:{c}" for t, c in zip(tgrid, live)))
print("mean live waves:", d.sum() / b.max(), " (max possible 8192)")
key = xcc * 1000 + se * 100 + cu
uk, inv = np.unique(key, return_inverse=True)
busy = np.bincount(inv, weights=d)
cnt = np.bincount(inv)
print(f"CUs seen {len(uk)}; waves/CU min {cnt.min()} max {cnt.max()}; wave-us per CU min {busy.min():.0f} median {np.median(busy):.0f} max {busy.max():.0f}")
print("xcc histogram", np.bincount(xcc, minlength=8))
# duration by image row band (tile row)
tilesX = (w + 15) // 16
blk = np.arange(nb * 4) // 4
ty = blk // tilesX
band = np.bincount(ty * 8 // ((h + 15) // 16), weights=d) / np.bincount(ty * 8 // ((h + 15) // 16))
print("mean wave dur by image band (top..bottom):", np.round(band, 1))

print(f"max-lane nodes per wave: median {np.median(mx):.0f} p90 {np.percentile(mx,90):.0f} p99 {np.percentile(mx,99):.0f} max {mx.max()}")
print(f"mean-lane nodes per wave: median {np.median(sm/64):.1f} p90 {np.percentile(sm/64,90):.1f}")
print(f"SIMD efficiency (sum / (64*max)) overall: {sm.sum() / (64 * mx.sum()):.3f}")
sel = mx > 0
us_per_iter = d[sel] / mx[sel]
print(f"wave us per max-lane node: median {np.median(us_per_iter):.3f} p90 {np.percentile(us_per_iter,90):.3f}")
o = np.argsort(-d)[:10]
print("10 longest waves: dur us, maxlane, meanlane, start us:")
for i in o:
    print(f"  {d[i]:.1f} {mx[i]} {sm[i]/64:.1f} {a[i]:.1f}")
print("corr(dur, maxlane)", np.corrcoef(d[sel], mx[sel])[0, 1])
