"""One measurement process for tools/ab_libs.py (RT_LIB selects the library).
Prints one JSON line: primary trace ms (longest-first and row-major), the
max-rank tiled trace at P=8, shadow and path frames, 1M build ms, and CRCs of
every output so the libraries can be checked for identical results."""
import json
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd.scenes import SOUP_VIEW as V  # noqa: E402

modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["trace", "rowmajor", "p8", "shadow", "path", "build"]
for kv in os.environ.get("RT_CONFIG", "").split(","):  # e.g. RT_CONFIG=trace.steal=1
    if kv:
        R.config_set(kv.split("=")[0], int(kv.split("=")[1]))
w, h, spp = 1920, 1080, 1
s = R.Scene.generate_soup(1_000_000, 1)
R.Scene.wide_arity = property(lambda self: 4)  # older libraries lack rt_bvh_wide_arity; unused here
s.build()
cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
hits = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
out = {}


def crc(*ts):
    c = 0
    for t in ts:
        c = zlib.crc32(t.cpu().numpy().tobytes(), c)
    return c


def med(f, k):
    return float(np.median([f() for _ in range(k)]))


if "build" in modes:
    out["build"] = med(lambda: s.build(), 10)
if "trace" in modes:
    R.config_set("trace.tile_order", 1)
    out["trace"] = med(lambda: s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True), 12)
    out["crc_trace"] = crc(img, hits)
if "rowmajor" in modes:
    R.config_set("trace.tile_order", 0)
    out["rowmajor"] = med(lambda: s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), timed=True), 8)
    R.config_set("trace.tile_order", 1)
if "moving" in modes:  # the bench's headline sequence: the eye orbiting 0.25 deg per frame
    import bench  # noqa: E402
    cams = [R.camera_look_at(bench.orbit_view(V, i), V.at, V.up, V.vfov, w, h) for i in range(14)]
    for c in cams[:2]:
        s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True)
    out["moving"] = float(np.mean([s.render_device(c, w, h, spp, d_rgba=img.data_ptr(), timed=True) for c in cams[2:]]))
    out["crc_moving"] = crc(img)
for P in (2, 4, 8):  # one rank's tiles, max over ranks (one GPU standing in for each)
    if f"p{P}" not in modes:
        continue
    t = []
    for r in range(P):
        slab = torch.zeros(max(R.tiles_for_rank(w, h, r, P), 1) * 256, dtype=torch.int32, device="cuda")
        t.append(med(lambda: s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), timed=True), 5))
    out[f"p{P}"] = max(t)
if "shadow" in modes:
    out["shadow"] = med(lambda: s.render_shadow_device(cam, w, h, spp, (2.0, 3.0, -2.0), 0.2, d_rgba=img.data_ptr(), timed=True), 6)
    out["crc_shadow"] = crc(img)
if "path" in modes:
    out["path"] = med(lambda: s.render_path_device(cam, w, h, spp, (2.0, 3.0, -2.0), 0.3, 2, d_rgba=img.data_ptr(), timed=True), 4)
    out["crc_path"] = crc(img)
for key in (2, 4, 5):  # another BASELINE config's full frame (static camera, tile order on)
    if f"c{key}" not in modes:
        continue
    import bench  # noqa: E402
    from gpu_raytracer_amd import scenes as S  # noqa: E402
    cf = S.CONFIGS[key]
    vw = S.VIEWS[cf.scene]
    sc = bench.make_scene(R, S, cf)
    sc.build()
    cc = R.camera_look_at(vw.eye, vw.at, vw.up, vw.vfov, cf.w, cf.h)
    im = torch.zeros(cf.w * cf.h, dtype=torch.int32, device="cuda")
    hh = torch.zeros(cf.w * cf.h * cf.spp * 4, dtype=torch.float32, device="cuda")
    f = lambda: sc.render_device(cc, cf.w, cf.h, cf.spp, d_rgba=im.data_ptr(), d_hits=hh.data_ptr(), timed=True)
    f()
    out[f"c{key}"] = med(f, 6)
    out[f"crc_c{key}"] = crc(im, hh)
    sc.close()
    del im, hh
if "work" in modes:  # wide records and triangle records fetched by the primary frame
    wk = s.render_work(cam, w, h, spp)
    out["records"], out["tri_records"] = float(wk[0]), float(wk[1])
print(json.dumps(out), flush=True)
