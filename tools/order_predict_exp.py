"""Experiment (diagnostic build): which statistic of the previous frame best
predicts this frame's costly tiles on the bench's orbiting camera?  For each
frame i of the orbit, frame i-1 is rendered (row-major) to get its per-tile
wave durations (stamps) and per-pixel wide-step counts (rt_render_step_map);
frame i is then timed with tile orders sorted longest-first by
  dur      the slowest wave's duration (what the device cost map holds)
  maxstep  the largest pixel step count of the tile
  sum      the tile's total steps
  q8       the tile's 8th-largest pixel step count
  self     frame i's own durations (upper bound)
usage: python tools/order_predict_exp.py [frames] [reps]
(own top-K: how much of the gap the K costliest tiles of the frame itself close)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_LIB"] = os.path.join(ROOT, "gpu_raytracer_amd", "lib", "librtamd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
import bench  # noqa: E402

L = R.lib()
L.rt_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
L.rt_debug_tile_order.argtypes = [C.c_void_p]
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
view = S.VIEWS["soup"]
w, h = 1920, 1080
nb = ((w + 15) // 16) * ((h + 15) // 16)
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cams = [R.camera_look_at(bench.orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames + 1)]
frames_done = 0
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
R.config_set("trace.px_sort", 2)  # the full-frame kernel writes its step map (the order is overridden below)


def measure(cam):
    """row-major render; per-tile slowest-wave duration (us) and the step map"""
    o = torch.arange(nb, dtype=torch.int32, device="cuda")  # row-major via the override: the
    L.rt_debug_tile_order(C.c_void_p(o.data_ptr()))       # cost and step maps are still written
    s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
    torch.cuda.synchronize()
    L.rt_debug_tile_order(None)
    buf = np.zeros(nb * 16, np.uint64)
    assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(nb * 4, 4).astype(np.int64)
    dur = (st[:, 1] - st[:, 0]).reshape(nb, 4).max(1) / 100.0
    steps = s.step_map(w, h, 1).reshape(nb, 256).astype(np.int64)
    return dur, steps


def timed(cam, order):
    o = torch.from_numpy(order.astype(np.int32)).cuda()
    L.rt_debug_tile_order(C.c_void_p(o.data_ptr()))
    t = [s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True) for _ in range(reps)]
    L.rt_debug_tile_order(None)
    return float(np.median(t))


res = {}
prev = None
for i in range(1, frames + 1):
    dur0, st0 = measure(cams[i - 1])
    dur1, _ = measure(cams[i])
    dm = prev if prev is not None else dur0
    keys = {"mean2": dur0 + dm, "self": dur1}
    base = np.argsort(-(dur0 + dm), kind="stable")
    for K in (32, 128, 512):  # the frame's own K costliest tiles first, the rest by mean2
        top = np.argsort(-dur1, kind="stable")[:K]
        rest = base[~np.isin(base, top)]
        res.setdefault(f"own top-{K} + mean2", []).append(timed(cams[i], np.concatenate([top, rest])))
    prev = dur0
    for k, v in keys.items():
        res.setdefault(k, []).append(timed(cams[i], np.argsort(-v, kind="stable")))
    res.setdefault("row-major", []).append(timed(cams[i], np.arange(nb)))
R.config_set("trace.px_sort", 1)
for k, v in res.items():
    print(f"{k:<10s} mean {np.mean(v):.4f} ms", flush=True)
