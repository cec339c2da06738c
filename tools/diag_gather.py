"""Phase stamps of k_bucket_gather (the gather sort's second level) on the
clustered substitute scenes: diagnostic library
lib/exp/diaggather.so from `tools/build_exp.sh diaggather "-DRT_STAMPS
-DRT_GATHER_BIN_FAST=1024 -DRT_GATHER_SKEW=0"` (the scene stays on the gather
sort).  Per bucket block: bucket size m and the phase durations (s_memrealtime,
100 MHz); the slowest blocks first.
usage: python tools/diag_gather.py [bunny|sponza|soup] [n for soup]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RT_LIB", os.path.join(ROOT, "gpu_raytracer_amd", "lib", "exp", "diaggather.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

L = R.lib()
L.rt_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
L.rt_debug_stamps.restype = C.c_int
scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
s = R.Scene.generate_soup(int(sys.argv[2]) if len(sys.argv) > 2 else 70000, 1) if scene == "soup" \
    else R.Scene.from_soup(S.tris_for(scene))
for _ in range(4):
    s.build()
bt = s.build_times()
print(f"{scene}: n {s.num_tris}, sort_kind {bt.sort_kind}, build {bt.total:.4f} ms")
buf = np.zeros(1024 * 8, np.uint64)
assert L.rt_debug_stamps(1, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(1024, 8).astype(np.int64)
m = st[:, 7]
t0 = st[:, 0].min()
full = m > 0
end = np.where(full, st[:, 6], st[:, 1])
print(f"blocks: {int(full.sum())} non-empty; span {(end.max() - t0) / 100:.2f} us; start of the last block "
      f"{(st[:, 0].max() - t0) / 100:.2f} us; bucket sizes max {int(m.max())} mean {m[full].mean():.1f}")
names = ["table + sizes", "run marks + max-scan", "gather + bin atomics", "bin scan + grouping", "rank in bin",
         "write"]
for i, nm in enumerate(names):
    d = (st[full, i + 1] - st[full, i]) / 100.0
    print(f"  {nm:<22s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
order = np.argsort(-(end - st[:, 0]))
print("slowest blocks (m, phases us):")
for b in order[:8]:
    ph = [(st[b, i + 1] - st[b, i]) / 100.0 for i in range(6)] if m[b] else []
    print(f"  block {b:4d} m {int(m[b]):5d} total {(end[b] - st[b, 0]) / 100:6.2f}  " + " ".join(f"{x:5.2f}" for x in ph))
s.close()
