"""A/B of trace configurations on the bench's moving-camera sequence (the
headline workload: soup-1M 1080p, eye orbiting 0.25 deg per frame), full
frames on one GPU; each configuration renders the whole sequence in turn,
interleaved over rounds; reports the mean event-timed trace per frame.
usage: python tools/ab_moving.py [rounds] [frames] name:knob=v,knob=v ...  (or name@knob=v,...)
AB_CONFIG=<k> runs BASELINE configs[k-1] (its scene and frame shape) instead of 3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402
import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rebuild = os.environ.get("AB_REBUILD", "0") == "1"  # rebuild the BVH before every timed frame, as bench.py does
configs = [("base", {})]
for a in sys.argv[3:]:
    name, kv = a.split(":", 1) if ":" in a else a.split("@", 1)
    configs.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
cfg = S.CONFIGS[int(os.environ.get("AB_CONFIG", "3"))]
view = S.VIEWS[cfg.scene]
w, h, spp = cfg.w, cfg.h, cfg.spp
scene = bench.make_scene(R, S, cfg)
scene.build()
cams = [R.camera_look_at(bench.orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames + 2)]
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
hp = hits.data_ptr() if os.environ.get("AB_HITS", "0") == "1" else None  # the bench writes hit records too
defaults = {}
res = {n: [] for n, _ in configs}
for _ in range(rounds):
    for name, kv in configs:
        for k, v in kv.items():
            R.config_set(k, v)
        scene.render_device(cams[0], w, h, spp, d_rgba=img.data_ptr(), d_hits=hp, timed=True)  # this shape's first frame
        scene.render_device(cams[1], w, h, spp, d_rgba=img.data_ptr(), d_hits=hp, timed=True)
        t = []
        for i in range(frames):
            if rebuild:  # the bench's step: a build before every frame
                scene.build()
            t.append(scene.render_device(cams[2 + i], w, h, spp, d_rgba=img.data_ptr(), d_hits=hp, timed=True))
        res[name].append(float(np.mean(t)))
        for k in kv:  # back to the library defaults
            R.config_set(k, {"trace.coop_cap": -1, "trace.tile_order": 1, "trace.px_sort": 1, "trace.wg": 256,
                             "trace.coop_lanes": 32, "trace.coop_cap_tiles": -1, "trace.spp_lanes": 2}.get(k, 0))
for name, _ in configs:
    print(f"{name:<22s} mean trace {np.median(res[name]):.4f} ms  (rounds: {' '.join(f'{x:.4f}' for x in res[name])})",
          flush=True)
