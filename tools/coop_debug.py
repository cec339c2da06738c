"""Debug: mismatches of a coop frame vs the oracle (lanes, cap from argv)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from oracle import oracle as O  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

lanes, cap = int(sys.argv[1]), int(sys.argv[2])
tris = O.soup(40000, 11).reshape(-1, 9)
w, h, spp = 200, 120, 1
exp = O.build(tris)
ocam = O.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
eh, _ = O.trace(exp["nodes"], tris, ocam, w, h, spp)
R.config_set("trace.coop_lanes", lanes)
R.config_set("trace.coop_cap", cap)
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
with R.Scene.from_soup(tris) as s:
    s.build()
    hits, rgba, _ = s.render(cam, w, h, spp)
bad = np.nonzero((hits["prim"] != eh["prim"]) | (hits["t"].view(np.uint32) != eh["t"].view(np.uint32)))[0]
print("mismatches", len(bad), "of", len(eh))
for i in bad[:20]:
    print(i, i % w, i // w, "got", hits["t"][i], hits["prim"][i], "exp", eh["t"][i], eh["prim"][i])
