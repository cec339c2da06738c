"""Where a wide step's time goes in one rank's share of a P-GPU frame
(VERDICT r05 item 1): diagnostic library lib/exp/steps.so, built by
`tools/build_exp.sh steps "-DRT_STAMPS -DRT_STEPSTAMPS"`, whose k_trace stamps
every wide step with the shader clock (s_memtime) at three points:
  entry -> after the stack pop and the address math (pop: LDS read + VALU),
        -> the record / triangle loads back (wait: the memory round trip),
        -> the step's end (rest: box tests, Moller-Trumbore, pushes -- the
           dependent VALU chain, and whatever issue contention it meets).
Per wave it keeps the lane with the most fetching steps.  One GPU plays each
rank r of P (rt_render_tiles_device, t = r mod P) on the bench's orbiting
camera (soup-1M 1080p1), `frames` frames per rank; the last frame's stamps.
Co-residency: for each wave, the mean number of OTHER waves of the same
launch resident on its SIMD (and its CU) over its lifetime, from the stamps'
start/end and HW_ID.  A least-squares fit of the rest-per-step against the
SIMD co-residency splits it into a lone-wave chain (intercept) and issue
contention (slope x co-residency).
usage: python tools/diag_steps.py [P=8] [frames=4] [cap=-1]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_LIB"] = os.path.join(ROOT, "gpu_raytracer_amd", "lib", "exp", "steps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

sys.path.insert(0, ROOT)
from bench import orbit_view  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cap = int(sys.argv[3]) if len(sys.argv) > 3 else -1
L = R.lib()
L.rt_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
L.rt_debug_stamps.restype = C.c_int
R.config_set("trace.coop_cap_tiles", cap)
cfg = S.CONFIGS[3]
view = S.VIEWS[cfg.scene]
w, h, spp = cfg.w, cfg.h, cfg.spp
s = R.Scene.generate_soup(cfg.n, 1)
s.build()
cams = [R.camera_look_at(orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames)]
tmax = max(R.tiles_for_rank(w, h, r, P) for r in range(P))
slab = torch.zeros(tmax * 256, dtype=torch.int32, device="cuda")
slab_hits = torch.empty(tmax * 256 * spp * 4, dtype=torch.float32, device="cuda")
rows = []
print(f"P={P}, soup-1M {w}x{h}x{spp}, {frames} orbit frames per rank, stamps of the last; "
      f"trace.coop_cap_tiles {cap}", flush=True)
for r in range(P):
    ms = [s.render_tiles_device(c, w, h, spp, r, P, slab.data_ptr(), slab_hits.data_ptr(), timed=True) for c in cams]
    nw = R.tiles_for_rank(w, h, r, P) * 4
    buf = np.zeros(nw * 8, np.uint64)
    assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(nw, 8).astype(np.int64)
    rows.append((r, ms, st))

allw = []
for r, ms, st in rows:
    t0 = st[:, 0].min()
    a, b = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # us
    hw = st[:, 2] & 0xFFFFFFFF
    xcc = (st[:, 2] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    simd_id = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    cu_id = simd_id // 4
    nst, pop, wait, ex, cyc = st[:, 3], st[:, 4], st[:, 5], st[:, 6], st[:, 7]
    dur = b - a
    ghz = np.median(cyc[dur > 5] / (dur[dur > 5] * 1e3))
    # co-residency: mean number of other waves on the same SIMD / CU over each wave's life
    order = np.argsort(simd_id, kind="stable")
    co_simd = np.zeros(len(a))
    co_cu = np.zeros(len(a))
    for key, co in ((simd_id, co_simd), (cu_id, co_cu)):
        for k in np.unique(key):
            idx = np.nonzero(key == k)[0]
            A, B = a[idx], b[idx]
            for j, i in enumerate(idx):
                ov = np.clip(np.minimum(B, b[i]) - np.maximum(A, a[i]), 0, None)
                co[i] = (ov.sum() - (b[i] - a[i])) / max(b[i] - a[i], 1e-6)
    for i in range(len(a)):
        allw.append((r, dur[i], b[i], nst[i], pop[i], wait[i], ex[i], cyc[i], co_simd[i], co_cu[i], ghz))
    print(f"rank {r}: frames ms {' '.join(f'{x:.4f}' for x in ms)}; last frame: {len(a)} waves, span "
          f"{b.max():.1f} us, clock {ghz:.2f} GHz", flush=True)

W = np.array(allw, dtype=np.float64)
r_, dur, end, nst, pop, wait, ex, cyc, cos, coc, ghz = W.T
heavy = nst >= 60
print(f"\nall ranks: {len(W)} waves; {int(heavy.sum())} with a lane of >= 60 fetching steps (the capped rays' waves)")
for name, sel in (("heavy (>= 60 steps)", heavy), ("medium (20-59)", (nst >= 20) & (nst < 60)), ("light (< 20)", nst < 20)):
    if not sel.any():
        continue
    n = nst[sel]
    tot = (pop + wait + ex)[sel] / n
    print(f"{name:<20s} waves {int(sel.sum()):5d}  steps med {np.median(n):.0f}  per step (cycles, median): "
          f"pop {np.median(pop[sel] / n):6.0f}  wait {np.median(wait[sel] / n):6.0f}  rest {np.median(ex[sel] / n):6.0f}"
          f"  sum {np.median(tot):6.0f} = {np.median(tot / (ghz[sel] * 1e3)):.3f} us;  "
          f"co-resident waves on its SIMD {np.median(cos[sel]):.2f}, CU {np.median(coc[sel]):.2f}; "
          f"stepping share of the wave {np.median((pop + wait + ex)[sel] / cyc[sel]):.2f}")
# rest per step vs SIMD co-residency (heavy waves): intercept = lone-wave chain
if heavy.sum() > 10:
    y = ex[heavy] / nst[heavy]
    x = cos[heavy]
    A = np.vstack([np.ones_like(x), x]).T
    (c0, c1), *_ = np.linalg.lstsq(A, y, rcond=None)
    yw = wait[heavy] / nst[heavy]
    (w0, w1), *_ = np.linalg.lstsq(A, yw, rcond=None)
    print(f"\nheavy waves, per step: rest = {c0:.0f} + {c1:.0f} x (co-resident waves on the SIMD) cycles; "
          f"wait = {w0:.0f} + {w1:.0f} x (co-resident) cycles")
    g = float(np.median(ghz[heavy]))
    cm = float(np.median(x))
    parts = {"pop (LDS stack + address)": float(np.median(pop[heavy] / nst[heavy])),
             "fetch wait (record + triangle)": float(np.median(yw)),
             "dependent VALU chain (lone wave)": c0,
             "issue contention (co-resident waves)": c1 * cm}
    tot = sum(parts.values())
    print(f"split of a heavy wave's step at its median co-residency {cm:.2f} ({tot:.0f} cycles = {tot / g / 1e3:.3f} us "
          f"at {g:.2f} GHz):")
    for k, v in parts.items():
        print(f"  {k:<40s} {v:6.0f} cycles  {v / g / 1e3:.3f} us  {v / tot:5.1%}")
print("\n(stamps: ~40 cycles each, three per step; the forced vmcnt(0) after the loads moves no VALU: "
      "the step's VALU all depends on the loaded words)")
s.close()
