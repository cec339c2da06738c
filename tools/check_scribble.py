"""Confirms the debug hooks are live: one small build + render with
RT_DEBUG_LDS_SCRIBBLE=1 / RT_DEBUG_POISON=1 set by the caller.  Run under
`rocprofv3 --kernel-trace --stats`: k_lds_scribble must appear once before
every library kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

with R.Scene.generate_soup(5000, 3) as s:
    s.build()
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, 64, 48)
    for _ in range(2):
        s.render(cam, 64, 48, 1)
print("scribble check done")
