"""Experiment (diagnostic build): XCD-aware tile orders.  Blocks are dealt
round-robin over the 8 XCDs (block b and b + 8 share one, MI355X_MICROARCH.md),
each with its own 4-MB L2.  Longest-first by measured tile time (the order the
cost map approximates) against orders that give each XCD a spatially compact,
cost-balanced group of tiles (cut along a Morton curve of the tile grid into
G groups of equal total time), longest-first inside each group, dispatch
position i taking the next tile of group i mod G.
usage: python tools/xcd_order_exp.py [rounds]"""
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
tx, ty = (w + 15) // 16, (h + 15) // 16
nb = tx * ty
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
R.config_set("trace.tile_order", 0)
R.config_set("trace.px_sort", 0)
for _ in range(3):
    s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True)
ref = img.cpu().numpy().copy()
buf = np.zeros(nb * 16, np.uint64)
assert L.rt_debug_stamps(2, buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(nb * 4, 4).astype(np.int64)
dur = (st[:, 1] - st[:, 0]).reshape(nb, 4).max(1) / 100.0


def morton2(x, y):
    def spread(v):
        v = v.astype(np.uint64)
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        v = (v | (v << 1)) & 0x55555555
        return v
    return spread(x) | (spread(y) << 1)


t = np.arange(nb)
curve = np.argsort(morton2(t % tx, t // tx), kind="stable")


def grouped(G):
    c = np.cumsum(dur[curve])
    g_of = np.minimum((c - dur[curve] / 2) * G // c[-1], G - 1).astype(np.int64)
    groups = [curve[g_of == g] for g in range(G)]
    groups = [gr[np.argsort(-dur[gr], kind="stable")] for gr in groups]
    out, ptr = [], [0] * G
    while len(out) < nb:
        for g in range(G):
            if ptr[g] < len(groups[g]):
                out.append(groups[g][ptr[g]])
                ptr[g] += 1
    return np.array(out)


orders = {"measured longest-first": np.argsort(-dur, kind="stable")}
for G in (8, 16, 32):
    orders[f"{G} Morton groups, longest-first"] = grouped(G)
dev = {k: torch.from_numpy(v.astype(np.int32)).cuda() for k, v in orders.items()}
res = {}
for r in range(rounds):
    for k, o in dev.items():
        L.rt_debug_tile_order(C.c_void_p(o.data_ptr()))
        ms = [s.render_device(cam, w, h, 1, d_rgba=img.data_ptr(), timed=True) for _ in range(3)]
        res.setdefault(k, []).append(min(ms))
        assert np.array_equal(img.cpu().numpy(), ref), k
L.rt_debug_tile_order(None)
for k, v in res.items():
    print(f"{k:<36s} median {np.median(v):.4f} ms  min {min(v):.4f}", flush=True)
