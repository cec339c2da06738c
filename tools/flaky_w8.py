"""Repeat the 8-ary (and 4-ary) Cornell 64x64 render against the oracle and
report every mismatch (looking for a nondeterministic result)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
cases = [(S.cornell_tris(), S.CORNELL_VIEW, (64, 64, 1)), (S.bunny_substitute_tris(), S.BUNNY_VIEW, (160, 90, 1)),
         (S.sponza_substitute_tris(), S.SPONZA_VIEW, (96, 54, 2))]
exp = []
for tris, view, (w, h, spp) in cases:
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    b = O.build(tris)
    ocam = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, _ = O.trace(b["nodes"], tris, ocam, w, h, spp)
    exp.append((tris, view, (w, h, spp), eh, b))
bad = {4: 0, 8: 0}
for it in range(iters):
    for ar in (8, 4):
        R.config_set("build.wide_arity", ar)
        for ci, (tris, view, (w, h, spp), eh, b) in enumerate(exp):
            cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
            with R.Scene.from_soup(tris) as s:
                s.build()
                hits, rgba, _ = s.render(cam, w, h, spp)
                got = s.read_bvh()
            d = np.nonzero(hits["prim"] != eh["prim"])[0]
            nb = not np.array_equal(got["nodes"].view(np.uint32), b["nodes"].view(np.uint32))
            if len(d) or nb:
                bad[ar] += 1
                print(f"iter {it} arity {ar} case {ci}: {len(d)} prims differ (first {d[:5]}: got "
                      f"{hits['prim'][d[:5]]} exp {eh['prim'][d[:5]]}), bvh differs {nb}", flush=True)
R.config_set("build.wide_arity", 4)
print("mismatching renders:", bad, "of", iters * len(cases), "each", flush=True)
