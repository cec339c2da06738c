"""Digest of the built BVH (sorted keys, vals, nodes, wide records) for a few
soup sizes, plus the median event-timed build: compare two librtamd variants
(RT_LIB) for bit-identical builds and their speed.
usage: RT_LIB=<lib.so> python tools/bvh_digest.py [n ...]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [100003, 1000000, 2097152]
lib = os.path.basename(os.environ.get("RT_LIB", "librtamd.so"))
for n in sizes:
    s = R.Scene.generate_soup(n, 1)
    s.build()
    b = s.read_bvh()
    h = hashlib.sha1()
    for k in sorted(b):
        h.update(np.ascontiguousarray(b[k]).tobytes())
    h.update(np.ascontiguousarray(s.read_wide()).tobytes())
    ms = [s.build() for _ in range(30)]
    print(f"{lib:<14s} n={n:<8d} digest {h.hexdigest()[:16]} build median {np.median(ms) * 1e3:7.1f} us", flush=True)
    s.close()
