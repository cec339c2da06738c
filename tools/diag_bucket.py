"""Phase stamps of k_bucket_sort (diagnostic build librtamd_diag.so): per
phase durations over the 1024 bucket blocks of the 1M-soup build, and when
the blocks start and end (s_memrealtime, 100 MHz)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_LIB"] = os.path.join(ROOT, "gpu_raytracer_amd", "lib", "librtamd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402

L = R.lib()
L.rt_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
L.rt_debug_stamps.restype = C.c_int
s = R.Scene.generate_soup(1_000_000, 1)
for _ in range(3):
    s.build()
buf = np.zeros(1024 * 8, np.uint64)
assert L.rt_debug_stamps(1, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(1024, 8).astype(np.int64)[:, :7]
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
print(f"k_bucket_sort: {len(st)} blocks; start first 0 last {(st[:, 0].max() - t0) / 100:.2f} us; "
      f"end first {(st[:, 6].min() - t0) / 100:.2f} last {(st[:, 6].max() - t0) / 100:.2f} us")
for i, ph in enumerate(["loads", "pass 0 rank", "pass 0 scan+scatter+reload", "pass 1 rank",
                        "pass 1 scan+scatter+reload", "global stores"]):
    d = (st[:, i + 1] - st[:, i]) / 100.0
    print(f"  {ph:<28s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f} us")
q = np.sort(st[:, 0] - t0) / 100
print("  block start quantiles (us):", [round(float(np.percentile(q, p)), 2) for p in (10, 25, 50, 75, 90, 100)])
