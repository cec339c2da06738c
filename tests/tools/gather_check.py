"""Gather-sort parity and timing on clustered scenes:
for each scene, 3 builds through the library $RT_LIB (default: in-tree) --
keys, indices and nodes against the oracle, the sort kind of every build --
then the median build time over 20 builds.
usage: python tests/tools/gather_check.py [scene ...]   (bunny sponza soup70k hot dup)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def scene_tris(name):
    if name in ("bunny", "sponza"):
        return np.ascontiguousarray(S.tris_for(name), np.float32).reshape(-1, 9)
    if name.startswith("soup"):  # soup70k, soup1m, ...
        k = name[4:].lower()
        return O.soup(int(float(k[:-1]) * (1000 if k.endswith("k") else 1000000)), 2).reshape(-1, 9)
    rng = np.random.default_rng(7)
    if name == "hot":  # a uniform soup plus 1500 small triangles crowded into a cube of side 0.01
        t = O.soup(60000, 3).reshape(-1, 9)
        c = rng.random((1500, 1, 3)).astype(np.float32) * 0.01 + 0.3
        h = (c + rng.standard_normal((1500, 3, 3)).astype(np.float32) * 1e-4).reshape(-1, 9)
        return np.ascontiguousarray(np.concatenate([t, h]), np.float32)
    if name == "dup":  # 300 copies of each of 200 triangles: identical keys in long runs
        t = O.soup(30000, 4).reshape(-1, 9)
        d = np.repeat(O.soup(200, 5).reshape(-1, 9), 300, axis=0)
        return np.ascontiguousarray(np.concatenate([t, d]), np.float32)
    raise SystemExit(f"unknown scene {name}")


for name in sys.argv[1:] or ["bunny", "sponza", "soup70k", "hot", "dup"]:
    t = scene_tris(name)
    exp = O.build(t)
    kinds, ok = [], True
    with R.Scene.from_soup(t) as s:
        for _ in range(3):
            s.build()
            kinds.append(s.build_times().sort_kind)
            got = s.read_bvh()
            ok &= bool(np.array_equal(got["keys"], exp["keys"]) and np.array_equal(got["vals"], exp["vals"])
                       and np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32)))
        tt = []
        for _ in range(20):
            s.build()
            tt.append(s.build_times().total)
    print(f"{name}: n {len(t)} parity {'OK' if ok else 'MISMATCH'} sort_kind {kinds} "
          f"build median {np.median(tt) * 1e3:.1f} us min {np.min(tt) * 1e3:.1f} us", flush=True)
    if not ok:
        sys.exit(1)
