"""Per-rank launches for a rocprofv3 kernel trace of the heavy-ray queue:
P = 8 ranks, 4 frames each, for each cap given (trace.coop_cap_tiles), then
the full frame (trace.coop_cap).  Parse with tools/coop_prof_parse.py.
COOP_ORBIT=1: frame f of every rank uses the bench's orbiting camera at step
f (0.25 deg per frame, tools/rank_orbit.py) instead of the static one.
usage: rocprofv3 --kernel-trace -d DIR -- python tools/coop_prof.py cap [cap...]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

w, h, spp, P = 1920, 1080, 1, int(os.environ.get("COOP_P", "8"))
R.config_set("trace.coop_lanes", int(os.environ.get("COOP_LANES", "64")))
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
ORBIT = os.environ.get("COOP_ORBIT", "0") == "1"


def cam_at(f):
    if not ORBIT:
        return R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    a = math.radians(0.25 * f)
    ex, ey, ez = (e - c for e, c in zip(V.eye, V.at))
    eye = (V.at[0] + ex * math.cos(a) + ez * math.sin(a), V.at[1] + ey, V.at[2] - ex * math.sin(a) + ez * math.cos(a))
    return R.camera_look_at(eye, V.at, V.up, V.vfov, w, h)


img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
for c in [int(x) for x in sys.argv[1:]]:
    R.config_set("trace.coop_cap_tiles", c)
    R.config_set("trace.coop_cap", c)
    for r in range(P):
        slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
        for f in range(4):
            s.render_tiles_device(cam_at(f), w, h, spp, r, P, slab.data_ptr(), timed=True)
    for f in range(4):
        s.render_device(cam_at(f), w, h, spp, d_rgba=img.data_ptr(), timed=True)
print("done")
