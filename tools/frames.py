"""K frames of one BASELINE config on the bench's orbiting camera (a build
before each, hits written, as bench.py's step), with librtamd knobs: a
driver for `rocprofv3 --kernel-trace` (gpu_run.sh kstats) of one kernel
configuration.
usage: python tools/frames.py [config=3] [frames=20] [knob=value ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

args = dict(a.split("=", 1) for a in sys.argv[1:])
key = int(args.pop("config", 3))
frames = int(args.pop("frames", 20))
for k, v in args.items():
    R.config_set(k, int(v))
cfg = S.CONFIGS[key]
view = S.VIEWS[cfg.scene]
w, h, spp = cfg.w, cfg.h, cfg.spp
scene = bench.make_scene(R, S, cfg)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
t = []
for i in range(frames):
    scene.build()
    cam = R.camera_look_at(bench.orbit_view(view, i), view.at, view.up, view.vfov, w, h)
    t.append(scene.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True))
print(f"config {key} knobs {args}: mean trace {np.mean(t[3:]):.4f} ms over frames 3..{frames - 1}", flush=True)
scene.close()
