"""Which sort each build of a scene ends up with (rt_build_times.sort_kind:
0 LSB, 1 MSB, 2 gather) and its event-timed total, for the BASELINE
substitute scenes and the soup, under each build.sort setting; plus the
scene's top-10-bit bucket and fine-bin maxima from the built BVH's sorted keys (what the
gather probe's verdicts look at: bucket > its LDS capacity = dense, a bin of
more than 64 keys = clustered).
usage: python tools/sort_verdict.py [builds=5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

builds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
scenes = {"bunny": S.tris_for("bunny"), "sponza": S.tris_for("sponza"),
          "soup-262K": None, "soup-1M": None}
for name, tris in scenes.items():
    for sort in (2, 1, 0):
        R.config_set("build.sort", sort)
        s = (R.Scene.from_soup(np.ascontiguousarray(tris, np.float32).reshape(-1, 9)) if tris is not None
             else R.Scene.generate_soup(262144 if "262K" in name else 1_000_000, 1))
        row = []
        for _ in range(builds):
            ms = s.build()
            row.append((s.build_times().sort_kind, round(ms * 1e3, 1)))
        if sort == 2:
            k = s.read_bvh()["keys"]
            b = np.bincount(k >> 20, minlength=1024)
            f = np.bincount(k >> 10)
            extra = f"top bucket max {b.max()}, fine bin max {f.max()} (bins > 64: {(f > 64).sum()})"
        else:
            extra = ""
        s.close()
        print(f"{name:10s} build.sort={sort}: (kind, us) per build {row} {extra}", flush=True)
R.config_set("build.sort", 2)
