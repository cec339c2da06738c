"""Design experiment (CPU model, tests/tools/order_sim.c): node fetches per primary
ray of §9.7's fixed preorder against a nearest-first traversal of the same
binary BVH, per ray and per 8x8 wave (its slowest lane), and how often the
nearest-first answer differs from §9.7's.

    python tests/tools/order_sim.py [n] [rows]
"""
import ctypes as C
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    so = "/tmp/libosim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests/tools/order_sim.c"), "-L", os.path.join(ROOT, "oracle/build"), "-loracle",
                    "-lm", "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    b = O.build(tris)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    pre = np.zeros(W * H, np.uint16)
    nfs = np.zeros(W * H, np.uint16)
    fl = np.zeros(W * H, np.uint8)
    ms = np.zeros(W * H, np.uint8)
    P = C.c_void_p

    def band(y0):
        L.osim_trace(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), C.byref(cam), W, H, y0, min(H, y0 + 24),
                     pre.ctypes.data_as(P), nfs.ctypes.data_as(P), fl.ctypes.data_as(P), ms.ctypes.data_as(P))

    with ThreadPoolExecutor(8) as ex:
        list(ex.map(band, range(0, H, 24)))
    for name, s in (("preorder", pre), ("nearest-first", nfs)):
        s = s.astype(np.int64)
        q = s.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
        print(f"{name:14s} fetches {int(s.sum()):,} | per ray mean {s.mean():.1f} p99 {np.percentile(s, 99):.0f} "
              f"max {s.max()} | 8x8 wave max-lane mean {q.mean():.1f} p99 {np.percentile(q, 99):.0f} max {q.max()}")
    print(f"flagged (non-self-consistent candidate at or before the answer): {int((fl & 1).sum())}; "
          f"answers differ: {int(((fl >> 2) & 1).sum())}; differ unflagged: {int(((fl >> 1) & 1).sum())}; "
          f"nearest-first stack depth max {ms.max()} p99.9 {np.percentile(ms, 99.9):.0f}")


if __name__ == "__main__":
    main()
