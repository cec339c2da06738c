"""Randomised render stress against the oracle: scenes of random size, arity,
traversal variant, stack cap, sort and frame shape (1-16 spp), the queue,
order and store knobs, full frames or emulated ranks, rendered fresh and on
successive frames; any hit or pixel that differs from the oracle is
reported.
usage: python tests/tools/stress_render.py [iterations] [seed]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
presets = [(S.cornell_tris(), S.CORNELL_VIEW), (S.bunny_substitute_tris(), S.BUNNY_VIEW)]
V = S.SOUP_VIEW
bad = 0
t0 = time.time()
for it in range(iters):
    kind = rng.integers(0, 3)
    if kind < 2:
        tris, view = presets[kind]
        tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    else:
        n = int(rng.integers(2, 40000))
        tris = O.soup(n, int(rng.integers(1, 1000))).reshape(-1, 9)
        view = V
    ar = int(rng.choice([4, 8]))
    var = int(rng.choice([0, 0, 0, 2]))
    cap = int(rng.choice([0, 0, 1, 3, 14]))
    w, h = int(rng.integers(8, 200)), int(rng.integers(8, 120))
    spp = int(rng.choice([1, 1, 2, 3, 4, 8, 16]))
    P = int(rng.choice([1, 1, 1, 2, 3, 8]))
    knobs = {"build.wide_arity": ar, "trace.variant": var, "trace.stack_cap": cap,
             "build.sort": int(rng.choice([2, 2, 1, 0])),
             "trace.coop_cap": int(rng.choice([-1, -1, 0, 2, 24])),
             "trace.coop_cap_tiles": int(rng.choice([-1, -1, 0, 4])),
             "trace.spp_lanes": int(rng.choice([2, 1, 0])), "trace.px_sort": int(rng.choice([1, 1, 2, 0])),
             "trace.wg": int(rng.choice([256, 64])), "render.emulate": 1 if P > 1 else 0}
    for k, v in knobs.items():
        R.config_set(k, v)
    b = O.build(tris)
    ocam = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, _ = O.trace(b["nodes"], tris, ocam, w, h, spp)
    er = O.shade(eh, w, h, spp)
    cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for f in range(3):  # fresh, then with the previous frames' orders
            hits, rgba, _ = s.render(cam, w, h, spp, ngpus=P)
            d = np.nonzero(hits["prim"] != eh["prim"])[0]
            dp = np.nonzero(np.any(rgba.reshape(-1, 4) != er.reshape(-1, 4), axis=1))[0]
            if len(d) or len(dp):
                bad += 1
                print(f"MISMATCH it {it} frame {f}: n {len(tris)} {w}x{h}x{spp} P {P} {knobs}: "
                      f"{len(d)} hits, {len(dp)} pixels; first hits {d[:5].tolist()} got {hits['prim'][d[:5]].tolist()} "
                      f"exp {eh['prim'][d[:5]].tolist()}", flush=True)
    if it % 20 == 0:
        print(f"it {it} ({time.time() - t0:.0f} s)", flush=True)
for k, v in (("build.wide_arity", 4), ("trace.variant", 0), ("trace.stack_cap", 0), ("build.sort", 2),
             ("trace.coop_cap", -1), ("trace.coop_cap_tiles", -1), ("trace.spp_lanes", 2), ("trace.px_sort", 1),
             ("trace.wg", 256), ("render.emulate", 0)):
    R.config_set(k, v)
print(f"done: {iters} scenes x 3 frames, {bad} mismatching renders", flush=True)
