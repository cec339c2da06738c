"""VERDICT r04 item 6 -- the stop rule for a certified nearest-first pass
(CPU model, tests/tools/order_sim.c osim_hazards).  For every primary ray of the
soup-1M 1080p frame: the subtrees a nearest-first traversal culls only by
its current best t (§9.7, whose tb is larger there, may enter them).  A sound
certificate has to bound Moller-Trumbore's t error for every triangle in each
such subtree; that error is unbounded as the ray approaches a triangle's
plane (1/|d.n|), so it needs each subtree's normal cone, and only a subtree
of very few triangles has a cone that excludes grazing.  Printed: for all
rays and for the heavy rays (the ~1 % whose §9.7 traversal is longest -- the
ones the queue takes), how many have NO such subtree larger than k leaves.
    python tests/tools/order_cert.py [n]"""
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
    _, _, rlo, rhi, _ = O.karras(b["keys"])
    rlo = np.ascontiguousarray(rlo, np.uint32)
    rhi = np.ascontiguousarray(rhi, np.uint32)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    pre = np.zeros(W * H, np.uint16)
    hc = np.zeros(W * H, np.uint32)
    hm = np.zeros(W * H, np.uint32)
    P = C.c_void_p

    def band(y0):
        L.osim_hazards(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), C.byref(cam), W, y0, min(H, y0 + 24),
                       rlo.ctypes.data_as(P), rhi.ctypes.data_as(P), pre.ctypes.data_as(P), hc.ctypes.data_as(P),
                       hm.ctypes.data_as(P))

    with ThreadPoolExecutor(8) as ex:
        list(ex.map(band, range(0, H, 24)))
    heavy = pre >= np.percentile(pre, 99)
    print(f"rays {W * H}, heavy (top 1 % of §9.7 node visits, >= {int(np.percentile(pre, 99))}): {int(heavy.sum())}")
    for name, sel in (("all rays", np.ones_like(heavy)), ("heavy rays", heavy)):
        c, m = hc[sel], hm[sel]
        print(f"{name}: culled-by-t subtrees per ray mean {c.mean():.1f} p50 {np.median(c):.0f} max {c.max()}; "
              f"largest one's leaves p50 {np.median(m):.0f} p90 {np.percentile(m, 90):.0f}")
        for k in (0, 1, 2, 4, 8, 16):
            print(f"   no culled subtree above {k:2d} leaves: {float((m <= k).mean()):.4f}")


if __name__ == "__main__":
    main()
