"""Median build-stage times (hipEvents) of rt_bvh_build on the soup.
usage: python tools/build_times.py [n] [reps] [key=v,key=v,...]
  keys are rt_config_set knobs, plus lib=<path> (a librtamd variant, e.g.
  from tools/build_exp.sh; default: the in-tree library, or $RT_LIB).
  $RT_CFG adds knobs the same way.  BT_TRACE=1: a 1080p frame of the soup
  (hits + RGBA written, as bench.py's step) is traced before every timed
  build, so each build starts with the trace's data in the caches.
  BT_SCENE=bunny|sponza: that BASELINE substitute scene instead of the soup (n ignored)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
cfgs = [kv for kv in (os.environ.get("RT_CFG", "") + "," + (sys.argv[3] if len(sys.argv) > 3 else "")).split(",") if kv]
knobs = []
for kv in cfgs:
    k, v = kv.split("=", 1)
    if k == "lib":
        os.environ["RT_LIB"] = os.path.abspath(os.path.join(ROOT, v) if not os.path.isabs(v) else v)
    else:
        knobs.append((k, int(v)))

import numpy as np  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402

for k, v in knobs:
    R.config_set(k, v)
if os.environ.get("BT_SCENE"):
    from gpu_raytracer_amd import scenes as _S
    s = R.Scene.from_soup(_S.tris_for(os.environ["BT_SCENE"]))
    n = s.num_tris
else:
    s = R.Scene.generate_soup(n, 1)
between = lambda: None  # noqa: E731
if os.environ.get("BT_TRACE", "0") != "0":
    # BT_TRACE=1: the 1080p1 frame; BT_TRACE=c<k>: the frame of scenes.CONFIGS[k] (c5: 3840x2160x4)
    import torch
    from gpu_raytracer_amd import scenes as S
    bt = os.environ["BT_TRACE"]
    ck = int(bt[1:]) if bt.startswith("c") else 3
    fw, fh, fs = S.CONFIGS[ck].w, S.CONFIGS[ck].h, S.CONFIGS[ck].spp
    v = S.VIEWS[S.CONFIGS[3].scene]
    cam = R.camera_look_at(v.eye, v.at, v.up, v.vfov, fw, fh)
    img = torch.zeros(fw * fh, dtype=torch.int32, device="cuda")
    hits = torch.zeros(fw * fh * fs * 4, dtype=torch.float32, device="cuda")
    s.build()

    nohits = os.environ.get("BT_HITS") == "0"  # the frame writes RGBA only

    def between():
        s.render_device(cam, fw, fh, fs, d_rgba=img.data_ptr(), d_hits=0 if nohits else hits.data_ptr(), timed=True)
rows, tot = [], []
R.config_set("build.stage_events", 1)
for i in range(reps + 3):
    between()
    s.build()
    t = s.build_times()
    if i >= 3:
        rows.append([t.bounds, t.morton, t.sort, t.topology, t.refit, t.wide, t.total])
R.config_set("build.stage_events", 0)
for i in range(reps + 3):
    between()
    ms = s.build()
    if i >= 3:
        tot.append(ms)
m = np.median(np.array(rows), 0) * 1e3
lib = os.path.basename(os.environ.get("RT_LIB", "librtamd.so"))
lib += " " + ",".join(f"{k}={v}" for k, v in knobs) if knobs else ""
lib += (" after-trace" + ("" if os.environ["BT_TRACE"] == "1" else " " + os.environ["BT_TRACE"])
        if os.environ.get("BT_TRACE", "0") != "0" else "")
print(f"{lib:<24s} n={n} us: bounds {m[0]:6.1f} morton {m[1]:6.1f} sort {m[2]:6.1f} topo {m[3]:6.1f} "
      f"refit {m[4]:6.1f} wide {m[5]:5.1f} total(stage events) {m[6]:6.1f}  total {np.median(tot) * 1e3:6.1f}")
