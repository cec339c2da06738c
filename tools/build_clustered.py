"""Build time of a clustered soup, whose dense cell overflows one LDS bucket
sort (the global chunked passes of k_bucket_sort / k_bucket_sort_big):
usage: python tools/build_clustered.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rng = np.random.default_rng(5)
t = rng.random((n, 9), dtype=np.float32)
k = n // 4
t[:k] = 0.5 + rng.random((k, 9), dtype=np.float32) * 1e-4  # a quarter of the soup in one tiny cell
with R.Scene.from_soup(rng.random((n, 9), dtype=np.float32)) as w:  # loads every build kernel first
    [w.build() for _ in range(3)]
with R.Scene.from_soup(t) as s:
    ms = [s.build() for _ in range(12)]
print(f"clustered n={n}: first build (MSB, decides the sort) {ms[0]:.4f} ms, then median {np.median(ms[2:]):.4f} ms (min {min(ms[2:]):.4f})",
      flush=True)
