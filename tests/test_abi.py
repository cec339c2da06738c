"""CPU tests of the C-ABI boundary (librtamd.so): it loads, exports every
symbol include/gpu_raytracer_amd.h declares, its host-side pieces (scene
ingest, camera, OBJ/PPM/hit I/O, tile partition) match the oracle, and its
compute entry points fail loudly (RT_EDEVICE) when no GPU is present -- there
is no CPU fallback.  No compute call runs here."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, bits

HEADER = os.path.join(ROOT, "include", "gpu_raytracer_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported(rt):
    import subprocess
    declared = header_functions()
    assert len(declared) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", rt._lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rt_[a-z0-9_]+)", out))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(rt._lib.EXPORTED) == declared
    for f in declared:
        getattr(rt.lib(), f)  # resolvable through ctypes


def test_library_is_gfx950(rt):
    import subprocess
    blob = open(rt._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert rt.lib().rt_version().decode().endswith("(gfx950)")


def test_camera_matches_oracle(rt, oracle):
    for (eye, at, up, fov, w, h) in [((0.5, 0.5, -1.5), (0.5, 0.5, 0.5), (0, 1, 0), 45, 1920, 1080),
                                     ((278, 273, -800), (278, 273, 0), (0, 1, 0), 39.3077, 256, 256),
                                     ((1, 2, 3), (-4, 0.5, 9), (0.2, 1, 0.1), 70, 333, 77)]:
        c = rt.camera_look_at(eye, at, up, fov, w, h)
        o = oracle.camera_look_at(eye, at, up, fov, w, h)
        assert np.array_equal(bits(rt.camera_array(c)), bits(o.as_array()))


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 100003])
def test_soup_generator_matches_oracle(rt, oracle, n):
    s = rt.Scene.generate_soup(n, 1)
    assert s.num_tris == n
    assert np.array_equal(bits(s.tris()), bits(oracle.soup(n, 1).reshape(-1, 9)))
    s.close()


def test_from_soup_roundtrip(rt):
    t = np.random.default_rng(0).random((123, 9), dtype=np.float32)
    with rt.Scene.from_soup(t) as s:
        assert s.num_tris == 123 and np.array_equal(s.tris(), t)


def test_obj_loader(rt, tmp_path):
    p = tmp_path / "quad.obj"
    p.write_text("# comment\nmtllib x.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\n"
                 "o thing\nusemtl m\nf 1/1/1 2/1/1 3/1/1 4/1/1\nf -4 -2 -1\ns off\n")
    with rt.Scene.load_obj(str(p)) as s:
        t = s.tris()
    exp = np.array([[0, 0, 0, 1, 0, 0, 1, 1, 0], [0, 0, 0, 1, 1, 0, 0, 1, 0], [0, 0, 0, 1, 1, 0, 0, 1, 0]], np.float32)
    assert np.array_equal(t, exp)
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(rt.RtError) as e:
        rt.Scene.load_obj(str(bad))
    assert e.value.status == -3
    with pytest.raises(rt.RtError) as e:
        rt.Scene.load_obj(str(tmp_path / "missing.obj"))
    assert e.value.status == -3


def test_ppm_and_hits_dump(rt, tmp_path):
    rgba = np.arange(4 * 3 * 4, dtype=np.uint8)
    p = tmp_path / "img.ppm"
    rt.dump_ppm(rgba, 4, 3, str(p))
    data = p.read_bytes()
    assert data.startswith(b"P6\n4 3\n255\n")
    assert data[len(b"P6\n4 3\n255\n"):] == rgba.reshape(-1, 4)[:, :3].tobytes()
    hits = np.zeros(5, rt.HIT_DTYPE)
    hits["t"] = np.arange(5)
    hits["prim"] = 0xFFFFFFFF
    q = tmp_path / "h.bin"
    rt.dump_hits(hits, str(q))
    assert q.read_bytes() == hits.tobytes()


@pytest.mark.parametrize("w,h,P", [(1920, 1080, 1), (1920, 1080, 8), (3840, 2160, 8), (17, 33, 3), (16, 16, 4)])
def test_tile_partition(rt, w, h, P):
    nt = ((w + 15) // 16) * ((h + 15) // 16)
    counts = [rt.tiles_for_rank(w, h, r, P) for r in range(P)]
    assert sum(counts) == nt
    assert max(counts) - min(counts) <= 1
    assert rt.tiles_for_rank(w, h, P, P) == 0


def test_invalid_arguments(rt):
    cam = rt.camera_look_at((0, 0, -1), (0, 0, 0), (0, 1, 0), 45, 8, 8)
    with rt.Scene.from_soup(np.zeros((3, 9), np.float32)) as s:
        for args, kw in [((0, 8), {}), ((8, 8), {"ngpus": 0}), ((8, 8), {"ngpus": 65}), ((8, 8, 0), {})]:
            with pytest.raises(rt.RtError) as e:
                s.render(cam, *args, **kw)
            assert e.value.status == -1, (args, kw)
        # an unbuilt scene: RT_EINVAL on a GPU box, RT_EDEVICE without a device
        with pytest.raises(rt.RtError) as e:
            s.render(cam, 8, 8)
        assert e.value.status == (-1 if rt.device_count() else -4)


def test_render_prototype_is_survey_8b(rt):
    """rt_render is exactly SURVEY.md §8(b)'s prototype (SURVEY.md:291-292):
    (scene, cam, w, h, spp, ngpus, hits_out, rgba_out) -- 8 parameters, no
    timing output (that is rt_render_timed's ninth)."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "gpu_raytracer_amd.h")).read()

    def proto(name):
        m = re.search(r"rt_status\s+" + name + r"\s*\(([^)]*)\)\s*;", hdr)
        assert m, name
        return [" ".join(a.split()) for a in m.group(1).split(",")]

    assert proto("rt_render") == [
        "rt_scene* s", "const rt_camera* cam", "uint32_t w", "uint32_t h", "uint32_t spp", "uint32_t ngpus",
        "rt_hit* hits_out", "uint8_t* rgba_out"]
    assert proto("rt_render_timed") == proto("rt_render") + ["double* ms_out"]
    # called with exactly 8 arguments: without a GPU it refuses (RT_EDEVICE)
    # before touching the NULL scene's device
    cam = rt.camera_look_at((0, 0, -1), (0, 0, 0), (0, 1, 0), 45, 8, 8)
    with rt.Scene.from_soup(np.zeros((3, 9), np.float32)) as s:
        st = rt._lib.lib().rt_render(s._h, __import__("ctypes").byref(cam), 8, 8, 1, 1, None, None)
        assert st == (-1 if rt.device_count() else -4)


def test_render_ngpus_beyond_visible_devices(rt):
    """rt_render(ngpus > visible devices) -> RT_EDEVICE (SURVEY.md §8(b):
    multi-GPU is internal to rt_render), checked before any device work."""
    cam = rt.camera_look_at((0, 0, -1), (0, 0, 0), (0, 1, 0), 45, 8, 8)
    with rt.Scene.from_soup(np.zeros((3, 9), np.float32)) as s:
        for ngpus in (rt.device_count() + 1, 64):
            with pytest.raises(rt.RtError) as e:
                s.render(cam, 8, 8, ngpus=ngpus)
            assert e.value.status == -4, ngpus


def test_build_backend_and_mask(rt):
    """rt_bvh_build(scene, backend, device_mask, ms): the CPU backend does not
    exist (RT_EINVAL, never a silent oracle fallback); a mask naming a device
    that is not visible is RT_EDEVICE."""
    with rt.Scene.from_soup(np.zeros((3, 9), np.float32)) as s:
        with pytest.raises(rt.RtError) as e:
            s.build(backend=rt.RT_BACKEND_CPU)
        assert e.value.status == -1 and "no CPU backend" in str(e.value)
        with pytest.raises(rt.RtError) as e:
            s.build(backend=7)
        assert e.value.status == -1
        with pytest.raises(rt.RtError) as e:
            s.build(device_mask=1 << max(rt.device_count(), 1))
        assert e.value.status == -4
        assert s.replicas() == []


def test_no_cpu_fallback(rt):
    """Without a GPU every compute entry point fails loudly with RT_EDEVICE."""
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    tris = np.random.default_rng(1).random((64, 9), dtype=np.float32)
    with rt.Scene.from_soup(tris) as s:
        with pytest.raises(rt.RtError) as e:
            s.build()
        assert e.value.status == -4
    for f in (lambda: rt.stage_bounds(tris), lambda: rt.stage_sort(np.arange(10), np.arange(10)),
              lambda: rt.stage_minmax(np.zeros(2), np.zeros(2))):
        with pytest.raises(rt.RtError) as e:
            f()
        assert e.value.status == -4


def test_obj_loader_robustness(rt, tmp_path):
    """CRLF, continuation lines, comments after data, long lines, relative
    indices, polygon fans and every ignored statement."""
    p = tmp_path / "messy.obj"
    n = 400  # one polygon with n corners on a single very long line
    ang = np.linspace(0.0, 2.0 * np.pi, n, endpoint=False)
    verts = "".join(f"v {np.cos(a):.6f} {np.sin(a):.6f} 0.5 1.0\r\n" for a in ang)
    face = "f " + " ".join(f"{i + 1}/{i + 1}/1" for i in range(n)) + "   # a comment\r\n"
    text = ("# header\r\nmtllib scene.mtl\r\ng grp\r\n" + verts + "vt 0 0\r\nvn 0 0 1\r\nusemtl red\r\n" + face +
            "v 2 0 0\r\nv 2 1 \\\r\n 0\r\nv 3 0 0\r\nf -3//1 -2//1 -1//1\r\nl 1 2\r\np 1\r\ns 1\r\n")
    p.write_bytes(text.encode())
    with rt.Scene.load_obj(str(p)) as s:
        t = s.tris()
    assert t.shape == (n - 2 + 1, 9)
    ring = np.array([[float(f"{np.cos(a):.6f}"), float(f"{np.sin(a):.6f}"), 0.5] for a in ang], np.float32)
    for k in range(1, n - 1):  # fan (0, k, k+1)
        assert np.array_equal(t[k - 1], np.concatenate([ring[0], ring[k], ring[k + 1]]))
    assert np.array_equal(t[-1], np.array([2, 0, 0, 2, 1, 0, 3, 0, 0], np.float32))
    for body, what in [("v 0 0 0\nv 1 0 0\nf 1 2\n", "two corners"), ("v 0 0\n", "short vertex"),
                       ("v 0 0 0\nf 1 1 x\n", "bad index"), ("v 0 0 0\nf 0 1 1\n", "index 0")]:
        bad = tmp_path / "bad.obj"
        bad.write_text(body)
        with pytest.raises(rt.RtError) as e:
            rt.Scene.load_obj(str(bad))
        assert e.value.status == -3, what


def test_rtsoup1_roundtrip(rt, tmp_path):
    t = np.random.default_rng(1).standard_normal((1000, 9)).astype(np.float32)
    t[3, 4] = np.float32(-0.0)
    p = tmp_path / "s.rtsoup"
    with rt.Scene.from_soup(t) as s:
        s.save_soup(str(p))
    raw = p.read_bytes()
    assert raw[:8] == b"RTSOUP1\0" and len(raw) == 24 + 1000 * 36
    assert np.frombuffer(raw[16:24], np.uint64)[0] == 1000
    with rt.Scene.load_soup(str(p)) as s:
        assert np.array_equal(s.tris().view(np.uint32), t.view(np.uint32))
    empty = tmp_path / "e.rtsoup"
    with rt.Scene.from_soup(np.zeros((0, 9), np.float32)) as s:
        s.save_soup(str(empty))
    with rt.Scene.load_soup(str(empty)) as s:
        assert s.num_tris == 0
    for corrupt in (raw[:-4], b"RTSOUP2\0" + raw[8:], raw[:8] + b"\x02" + raw[9:], raw[:20]):
        q = tmp_path / "bad.rtsoup"
        q.write_bytes(corrupt)
        with pytest.raises(rt.RtError) as e:
            rt.Scene.load_soup(str(q))
        assert e.value.status == -3


def test_bvh_cache_rejects_without_device_work(rt, tmp_path):
    """A cache that is not RTBVH1 is refused before any device work."""
    q = tmp_path / "x.rtbvh"
    q.write_bytes(b"not a cache at all, definitely not")
    with rt.Scene.from_soup(np.zeros((3, 9), np.float32)) as s:
        with pytest.raises(rt.RtError) as e:
            s.load_bvh(str(q))
        assert e.value.status == -3


# rt_config_set keys: accepted values, a rejected value each, and the default
# restored afterwards (include/gpu_raytracer_amd.h; INTEGRATION.md "tuning").
CONFIG_KEYS = {
    "trace.variant": ([0, 2], [1, 3, -1], 0),
    "trace.stack_cap": ([0, 1, 14, 16, 18], [-1, 19], 0),
    "trace.wg": ([64, 256], [128], 256),
    "trace.wg_tiles": ([64, 256], [32], 64),
    "trace.tile_order": ([0, 1], [2], 1),
    "trace.px_sort": ([0, 1, 2], [3], 1),
    "trace.spp_lanes": ([0, 1, 2], [3, -1], 2),
    "build.sort": ([0, 1, 2], [3, -1], 2),
    "build.fuse_k01": ([0, 1, 2], [3, -1], 1),
    "build.wide_arity": ([4, 8], [2, 6, 16, -1], 4),
    "build.stage_events": ([0, 1], [2], 0),
    "path.wavefront": ([0, 1], [2], 1),
    "path.wg": ([64, 256], [100], 64),
    "path.sort": ([0, 4], [5], 0),
    "path.batch": ([0, 1 << 20], [-1], 0),
    "render.emulate": ([0, 1], [2], 0),
    "render.rccl1": ([0, 1], [2], 0),
    "trace.coop_cap": ([-1, 0, 1, 96, 1 << 20], [-2, (1 << 20) + 1], -1),
    "trace.coop_cap_tiles": ([-1, 0, 1, 96, 1 << 20], [-2, (1 << 20) + 1], -1),
    "trace.coop_lanes": ([16, 32, 64], [0, 8, 48, 128], 32),
    "trace.coop_max": ([1, 64, 65536, 1 << 24], [0, -1, (1 << 24) + 1], 65536),
    "debug.poison": ([0, 1], [2, -1], 0),
    "debug.lds_scribble": ([0, 1], [2, -1], 0),
    "debug.force_lsb_redo": ([0, 1], [2, -1], 0),
}
# r06: knobs whose non-default settings measured slower
# and served no test-only purpose were removed (profiles/rejected_knobs_r06.patch)
REMOVED_KEYS = ["trace.nt_hits", "trace.sl_mtf", "trace.sl_fold", "trace.coop_order", "trace.order_side",
                "trace.coop_skip", "trace.blocks", "trace.buf_loads", "build.wide_collapse", "build.cross_small",
                "timing.event_fence"]


@pytest.mark.parametrize("key", sorted(CONFIG_KEYS))
def test_config_keys(rt, key):
    """Every tuning knob takes its documented values and rejects others with
    RT_EINVAL (no device needed: the knobs are host-side state)."""
    good, bad, default = CONFIG_KEYS[key]
    try:
        for v in good:
            rt.config_set(key, v)
        for v in bad:
            with pytest.raises(rt.RtError) as e:
                rt.config_set(key, v)
            assert e.value.status == -1
    finally:
        rt.config_set(key, default)


def test_config_unknown_key(rt):
    with pytest.raises(rt.RtError) as e:
        rt.config_set("trace.no_such_knob", 1)
    assert e.value.status == -1


@pytest.mark.parametrize("key", REMOVED_KEYS)
def test_config_removed_keys(rt, key):
    """The pruned knobs are gone: every value is RT_EINVAL."""
    for v in (0, 1, 2):
        with pytest.raises(rt.RtError) as e:
            rt.config_set(key, v)
        assert e.value.status == -1


def test_config_key_count():
    """The library parses exactly the knobs CONFIG_KEYS lists (at most 25,
    VERDICT r05 item 5), so this table and rt_abi.cpp cannot drift apart."""
    import re
    with open(os.path.join(ROOT, "gpu_raytracer_amd", "csrc", "rt_abi.cpp")) as f:
        keys = set(re.findall(r'k == "([a-z_]+\.[a-z_0-9]+)"', f.read()))
    assert keys == set(CONFIG_KEYS)
    assert len(keys) <= 25


def test_wide8_size_cap():
    """RT_WIDE8_MAX_N: the largest n whose 8-ary records' last
    byte offset (n-1) x 96 fits the trace's 32-bit buffer offsets; one more
    triangle would wrap.  (rt_abi.cpp static_asserts the library agrees.)"""
    import re
    with open(os.path.join(ROOT, "include", "gpu_raytracer_amd.h")) as f:
        m = re.search(r"#define RT_WIDE8_MAX_N (\d+)u", f.read())
    cap = int(m.group(1))
    assert (cap - 1) * 96 <= 2**32 - 1 < cap * 96


def test_stream_handles():
    """Python stream arguments: None = the scene's own stream (NULL), an
    explicit 0 (torch's default stream) = the HIP null stream
    (hipStreamLegacy), any other handle passed through."""
    from gpu_raytracer_amd.scene import HIP_STREAM_LEGACY, _stream
    assert _stream(None) is None
    assert _stream(0).value == HIP_STREAM_LEGACY == 1
    assert _stream(0xABC0).value == 0xABC0
