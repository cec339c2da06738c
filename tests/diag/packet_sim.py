"""Packet-traversal estimate (trace "tried and rejected"): for random
8x8 pixel quadrants of the soup-1M 1080p frame, the per-lane §9.7 binary node
visits (oracle tree, Python floats) against the union a wave packet would walk.
usage: python tools/packet_sim.py [n] [quadrants]"""
import sys, time, math
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from oracle import oracle as O
from gpu_raytracer_amd.scenes import SOUP_VIEW as V
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
t0 = time.time()
tris = O.soup(n, 1).reshape(-1, 9)
exp = O.build(tris)
nodes = exp["nodes"]
print("built", time.time() - t0, nodes.dtype.names, exp.keys())
lo = nodes["lo"].astype(np.float64).tolist(); hi = nodes["hi"].astype(np.float64).tolist()
A = nodes["a"].tolist(); E = nodes["esc"].tolist()
L0 = n - 1
VALS = exp["vals"].tolist()
W, H = 1920, 1080
cam = O.camera_look_at(V.eye, V.at, V.up, V.vfov, W, H)
c = cam.as_array().astype(np.float64).reshape(4, 3)
eye, w00, du, dv = c
T = tris.astype(np.float64).tolist()
SENT = 0xFFFFFFFF
def mt(o, d, tri, tb):
    v0 = tri[0:3]; e1 = [tri[3+i]-v0[i] for i in range(3)]; e2 = [tri[6+i]-v0[i] for i in range(3)]
    p = [d[1]*e2[2]-d[2]*e2[1], d[2]*e2[0]-d[0]*e2[2], d[0]*e2[1]-d[1]*e2[0]]
    det = e1[0]*p[0]+e1[1]*p[1]+e1[2]*p[2]
    if det == 0: return None
    inv = 1.0/det
    s = [o[i]-v0[i] for i in range(3)]
    u = (s[0]*p[0]+s[1]*p[1]+s[2]*p[2])*inv
    if u < 0 or u > 1: return None
    q = [s[1]*e1[2]-s[2]*e1[1], s[2]*e1[0]-s[0]*e1[2], s[0]*e1[1]-s[1]*e1[0]]
    v = (d[0]*q[0]+d[1]*q[1]+d[2]*q[2])*inv
    if v < 0 or u + v > 1: return None
    t = (e2[0]*q[0]+e2[1]*q[1]+e2[2]*q[2])*inv
    if t <= 0 or t >= tb: return None
    return t
def trace(o, d):
    inv = [1.0/x if x != 0 else math.inf for x in d]
    tb = math.inf; X = 0; visited = []
    while X != SENT:
        l = lo[X]; h = hi[X]
        tn = 0.0; tf = tb
        for i in range(3):
            a = (l[i]-o[i])*inv[i]; b = (h[i]-o[i])*inv[i]
            if a > b: a, b = b, a
            tn = max(tn, a); tf = min(tf, b)
        visited.append(X)
        if tn <= tf:
            if X < L0:
                X = A[X]; continue
            k = X - L0
            prim = VALS[k]
            t = mt(o, d, T[prim], tb)
            if t is not None: tb = t
        X = E[X]
    return visited
rng = np.random.default_rng(0)
qs = [(int(rng.integers(0, W // 8)), int(rng.integers(0, H // 8))) for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 60)]
sum_max = sum_union = sum_mean = 0
for qx, qy in qs:
    sets = []
    for ly in range(8):
        for lx in range(8):
            x, y = qx*8+lx, qy*8+ly
            d = [(w00[i] + (x+0.5)*du[i]) + (y+0.5)*dv[i] for i in range(3)]
            sets.append(trace(list(eye), d))
    lens = [len(s) for s in sets]
    u = len(set().union(*map(set, sets)))
    sum_max += max(lens); sum_union += u; sum_mean += np.mean(lens)
print(f"quadrants {len(qs)}: mean-lane {sum_mean/len(qs):.1f}  max-lane {sum_max/len(qs):.1f}  union {sum_union/len(qs):.1f}  union/max {sum_union/sum_max:.3f}  mean/max {sum_mean/sum_max:.3f}")
