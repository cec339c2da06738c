"""Randomised build stress against the oracle, aimed at the sort paths a
scene's key distribution selects (r06): a uniform soup plus random clusters
(a few to thousands of small triangles in a cube of random size, so bins from
a few keys up to whole buckets, and buckets beyond one block's LDS) and
random runs of duplicated triangles (identical keys).  Each scene is built
three times (the probe build and the builds after its verdict), under a
random build.sort; sorted keys, indices and every node are compared with the
oracle bit for bit, and the sort kinds are counted.
usage: python tests/tools/stress_build.py [iterations] [seed]"""
import os
import sys
import time
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from oracle import oracle as O  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)


def scene(rng):
    parts = [O.soup(int(rng.integers(0, 200000)), int(rng.integers(1, 1000))).reshape(-1, 9)]
    for _ in range(int(rng.integers(0, 5))):  # clusters
        m = int(rng.integers(1, 2500))
        side = float(10.0 ** rng.uniform(-4, -0.5))
        c = rng.random((m, 1, 3)).astype(np.float32) * side + rng.random(3).astype(np.float32)
        parts.append((c + rng.standard_normal((m, 3, 3)).astype(np.float32) * side * 0.01).reshape(-1, 9))
    for _ in range(int(rng.integers(0, 3)) * int(rng.random() < 0.5)):  # duplicated triangles
        base = O.soup(int(rng.integers(1, 50)), int(rng.integers(1, 1000))).reshape(-1, 9)
        parts.append(np.repeat(base, int(rng.integers(2, 100)), axis=0))
    t = np.ascontiguousarray(np.concatenate(parts), np.float32)
    if len(t) < 2:
        t = O.soup(2, 1).reshape(-1, 9)
    return t[rng.permutation(len(t))] if rng.random() < 0.5 else t


bad = 0
kinds = Counter()
t0 = time.time()
for it in range(iters):
    tris = scene(rng)
    sort = int(rng.choice([2, 2, 2, 1, 0]))
    R.config_set("build.sort", sort)
    exp = O.build(tris)
    with R.Scene.from_soup(tris) as s:
        for b in range(3):
            s.build()
            kinds[(sort, s.build_times().sort_kind)] += 1
            got = s.read_bvh()
            ok = (np.array_equal(got["keys"], exp["keys"]) and np.array_equal(got["vals"], exp["vals"])
                  and np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32)))
            if not ok:
                bad += 1
                print(f"MISMATCH it {it} build {b}: n {len(tris)} build.sort {sort} "
                      f"sort_kind {s.build_times().sort_kind}", flush=True)
    if it % 20 == 0:
        print(f"it {it} ({time.time() - t0:.0f} s)", flush=True)
R.config_set("build.sort", 2)
print("sort kinds (build.sort, sort_kind): " + ", ".join(f"{k}: {v}" for k, v in sorted(kinds.items())))
print(f"done: {iters} scenes x 3 builds, {bad} mismatching builds")
sys.exit(1 if bad else 0)
