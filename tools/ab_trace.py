"""A/B the trace-kernel variants in ONE process, interleaved rounds (guide
§5.4 rule 24).  usage: python tools/ab_trace.py [rounds] [variants, e.g. 0,2]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
sel = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "2"]
variants = []
for v in sel:
    order = 1
    if "o" in v:  # e.g. 0o0: row-major tile order (default 1: cost-map order)
        v, order = v.split("o")[0], int(v.split("o")[1])
    base = {"trace.tile_order": order}
    tag = "longest-first" if order else "row-major"
    if v == "0":
        variants.append((f"wide ({tag})", {**base, "trace.variant": 0, "trace.wg": 256}))
    elif v == "0s":
        variants.append((f"wide, 64-thread blocks ({tag})", {**base, "trace.variant": 0, "trace.wg": 64}))
    elif v == "2s":
        variants.append((f"binary, 64-thread blocks ({tag})", {**base, "trace.variant": 2, "trace.wg": 64}))
    elif v == "2":
        variants.append((f"binary ({tag})", {**base, "trace.variant": 2, "trace.wg": 256}))
cnts = {}
for name, cfg in variants:
    for k, v in cfg.items():
        R.config_set(k, v)
    cnts[name] = tuple(int(c) for c in s.render_counters(cam, w, h, spp))
    print(name, "kernel work (node records, tri records):", [int(c) for c in s.render_work(cam, w, h, spp)])
print("binary counters", cnts)
assert len(set(cnts.values())) == 1, "variants disagree on work counters"
ref = None
times = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, cfg in variants:
        for k, v in cfg.items():
            R.config_set(k, v)
        ms = [s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True) for _ in range(3)]
        times[name].append(min(ms))
        out = np.concatenate([img.cpu().numpy().view(np.uint32), hits.cpu().numpy().view(np.uint32)])
        if ref is None:
            ref = out.copy()
        assert np.array_equal(out, ref), name
R.config_set("trace.tile_order", 1)
R.config_set("trace.variant", 0)
R.config_set("trace.wg", 256)
for name, _ in variants:
    t = np.array(times[name])
    print(f"{name:<36s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  -> {w*h*spp/np.median(t)/1e3:8.1f} Mrays/s")
