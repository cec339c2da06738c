"""Distributed build (rt_dbuild_*) emulated on one GPU: P threads = P ranks,
each with its own scene, exchanging by device copies (dist.ThreadExchange).
Every rank's device phases run under one lock, synchronised and timed alone,
so each is that rank's own GPU time; the exchanges are counted in bytes (on
P GPUs they travel over xGMI, not measurable here).  Prints per phase the max
over ranks, the critical path of the compute, the bytes each rank receives,
and the replicated rt_bvh_build time of the same soup.
usage: python tools/dbuild_emulate.py [n] [P...]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import dist as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
Ps = [int(x) for x in sys.argv[2:]] or [2, 4, 8]
LOCK = threading.Lock()
PHASES = ("bounds", "keys", "sort", "subtrees", "merge")


class Timed(D.LibStages):
    def __init__(self, scene, dev):
        super().__init__(scene, dev)
        self.t = {p: 0.0 for p in PHASES}

    def _run(self, name, f, *a):
        with LOCK:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f(*a)
            torch.cuda.synchronize()
            self.t[name] += (time.perf_counter() - t0) * 1e3
        return r

    def bounds(self, rank, P): return self._run("bounds", super().bounds, rank, P)
    def keys(self, rank, P, b): return self._run("keys", super().keys, rank, P, b)
    def sort(self, c): return self._run("sort", super().sort, c)
    def subtrees(self, rank, P): return self._run("subtrees", super().subtrees, rank, P)
    def merge(self, tot): return self._run("merge", super().merge, tot)


ref = R.Scene.generate_soup(n, 1)
bt = [ref.build() for _ in range(6)][1:]
print(f"n={n}: replicated rt_bvh_build {np.median(bt):.4f} ms (event-timed, median of 5)", flush=True)
for P in Ps:
    scenes = [R.Scene.generate_soup(n, 1) for _ in range(P)]
    res = {}
    for rep in range(3):
        hub = D.ThreadExchange.Hub(P)
        st = [Timed(scenes[r], "cuda:0") for r in range(P)]
        info = [None] * P

        def run(r):
            torch.cuda.set_device(0)
            info[r] = D.distributed_build(st[r], D.ThreadExchange(hub, r))
        th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        res = {p: max(s.t[p] for s in st) for p in PHASES}
        res["bytes_in"] = max(i["bytes_in"] for i in info)
        res["crossing"] = info[0]["crossing"]
    same = all(np.array_equal(a, b) for a, b in zip(
        [ref.read_bvh()["nodes"].view(np.uint32), ref.read_wide()],
        [scenes[P - 1].read_bvh()["nodes"].view(np.uint32), scenes[P - 1].read_wide()]))
    crit = sum(res[p] for p in PHASES)
    print(f"P={P}: " + "  ".join(f"{p} {res[p]:.3f}" for p in PHASES) +
          f" ms | compute critical path {crit:.3f} ms | received per rank {res['bytes_in'] / 1e6:.1f} MB"
          f" ({res['bytes_in'] / n:.0f} B/prim) | crossing nodes {res['crossing']} | bit-identical {same}", flush=True)
    for s in scenes:
        s.close()
