"""Phase-stamp diagnostics (diagnostic build librtamd_diag.so, -DRT_STAMPS).

Runs the 1M-soup build, then (a) the refit_local stamps of the build and
(b) a stand-alone 4-pass sort (last pass' stamps), and prints per-phase
durations over blocks plus the chip-wide timeline (s_memrealtime, 100 MHz).
"""
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


def stamps(nblocks, which=0):
    buf = np.zeros(nblocks * 8, np.uint64)
    assert L.rt_debug_stamps(which, buf.ctypes.data, buf.nbytes) == 0
    return buf.reshape(nblocks, 8).astype(np.int64)


def report(name, st, phases, nslots):
    t0 = st[:, 0].min()
    print(f"== {name}: {len(st)} blocks, span {(st[:, nslots - 1].max() - t0) / 100:.1f} us")
    print(f"   start: first {0:.1f} us, last {(st[:, 0].max() - t0) / 100:.1f} us; "
          f"end: first {(st[:, nslots - 1].min() - t0) / 100:.1f}, last {(st[:, nslots - 1].max() - t0) / 100:.1f} us")
    for i, ph in enumerate(phases):
        d = (st[:, i + 1] - st[:, i]) / 100.0
        print(f"   {ph:<28s} median {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")
    if os.environ.get("SLOW"):  # the slowest blocks: start, phases (us)
        tot = st[:, nslots - 1] - st[:, 0]
        for b in np.argsort(-tot)[:int(os.environ["SLOW"])]:
            ph = " ".join(f"{(st[b, i + 1] - st[b, i]) / 100:6.2f}" for i in range(len(phases)))
            print(f"   block {b:6d} start {(st[b, 0] - t0) / 100:6.2f} total {tot[b] / 100:6.2f}: {ph}")


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
if os.environ.get("BT_SCENE"):  # a substitute scene (bunny / sponza) instead of the soup
    from gpu_raytracer_amd import scenes as S
    s = R.Scene.from_soup(S.tris_for(os.environ["BT_SCENE"]))
    n = s.num_tris
else:
    s = R.Scene.generate_soup(n, 1)
for _ in range(3):
    s.build()
M = (n + 255) // 256  # 256-leaf refit blocks (r05)
if n <= 1_048_576 and s.build_times().fused_k01:  # the fused K0 + K1 (its records from block 65536 on)
    T = (n + 4095) // 4096
    allst = stamps(65536 + T)
    report("k_morton_tb<fused>", allst[65536:65536 + T, :8],
           ["loads+partial box", "barrier (+ last block's reduction)", "box read", "keys+LDS histogram",
            "scan+table", "cursor scatter (LDS)", "word stores"], 8)
st_tr = stamps(M)
report("k_topo_refit", st_tr[:, :6], ["key window+sync", "topology+leaf (thread 0)", "scans+flags+sync",
                                      "sparse-table sweep+sync", "node+K7w stores"], 6)
own, ws = (st_tr[:, 6] - st_tr[:, 1]) / 100.0, (st_tr[:, 2] - st_tr[:, 6]) / 100.0
print(f"   wave 0's own node + leaf     median {np.median(own):7.2f}  p90 {np.percentile(own, 90):7.2f}  max {own.max():7.2f} us")
print(f"   wave 0's wave-wide searches  median {np.median(ws):7.2f}  p90 {np.percentile(ws, 90):7.2f}  max {ws.max():7.2f} us")
if os.environ.get("BT_SCENE") or os.environ.get("NO_SORT"):
    sys.exit(0)
keys = np.random.default_rng(0).integers(0, 2**30, n, dtype=np.uint64).astype(np.uint32)
for _ in range(2):
    R.stage_sort(keys, np.arange(n, dtype=np.uint32))
nt = (n + 4095) // 4096
st = stamps(nt, 1)
report("k_scatter (last pass)", st[:, :6], ["prefix+loads+sync", "rank+sync", "scans+offsets+sync", "LDS scatter+sync", "global scatter"], 6)
