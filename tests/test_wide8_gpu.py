"""GPU tests of the 8-ary wide records (build.wide_arity = 8, K7w8;
SURVEY.md §8(f) row 1 "4/8-wide"): the records restate the greedy
largest-surface cut with up to 8 entries and contain every entry's exact box,
and every kernel that walks them -- the primary full-frame and per-rank tile
kernels, the cooperative heavy-ray pass, shadow rays, both path schedules --
gives the CPU oracle's hits and images bit for bit, including forced stack
overflows, rays with a zero direction component, successive frames with the
tile/pixel order, the BVH cache and the broadcast sections."""
import numpy as np
import pytest

from conftest import bits
from test_wide_gpu import _check_wide

pytestmark = pytest.mark.gpu
SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


@pytest.fixture()
def cfg(R):
    keys = []

    def set_(k, v, default):
        keys.append((k, default))
        R.config_set(k, v)
    set_("build.wide_arity", 8, 4)
    yield set_
    for k, d in reversed(keys):
        R.config_set(k, d)


def _soup_view():
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    return SOUP_VIEW


def _oracle(oracle, tris, view, w, h, spp):
    exp = oracle.build(tris)
    ocam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    return eh, oracle.shade(eh, w, h, spp)


def _same(hits, rgba, eh, er):
    d = np.nonzero(hits["prim"] != eh["prim"])[0]
    assert len(d) == 0, (f"{len(d)} of {len(eh)} prims differ; first {d[:8].tolist()}: got "
                         f"{hits['prim'][d[:8]].tolist()} t {hits['t'][d[:8]].tolist()}, expected "
                         f"{eh['prim'][d[:8]].tolist()} t {eh['t'][d[:8]].tolist()}")
    for f in ("t", "u", "v"):
        assert np.array_equal(bits(hits[f]), bits(eh[f])), f
    assert np.array_equal(rgba, er)


def test_wide8_records(R, oracle):
    rng = np.random.default_rng(5)
    _check_wide(R, oracle.soup(3000, 2).reshape(-1, 9), 8)
    flat = oracle.soup(2000, 4).reshape(-1, 9).copy()
    flat[:, 2::3] = 0.25
    _check_wide(R, flat, 8)
    _check_wide(R, (rng.random((1500, 9)) * 1e-30).astype(np.float32), 8)
    _check_wide(R, (rng.random((1500, 9)) * 3e37 - 1.5e37).astype(np.float32), 8)
    _check_wide(R, np.tile(oracle.soup(1, 3).reshape(-1, 9), (700, 1)), 8)
    for n in (2, 3, 5, 9):  # records with fewer entries than slots
        rec = _check_wide(R, oracle.soup(n, 9).reshape(-1, 9), 8)
        assert rec.shape == (n - 1, 24)


def test_wide8_records_large(R, oracle):
    """A soup spanning many refit blocks: local records (k_topo_refit) and
    crossing ones (k_wide_cross) both restate the cut."""
    _check_wide(R, oracle.soup(40000, 8).reshape(-1, 9), 8)


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("cap", [1, 3, 7, 14, 0])
def test_wide8_render_and_overflow(R, oracle, cfg, variant, cap):
    """cap 1-7 force the overflow hand-off (a record pushes up to 7 entries);
    0 = the whole 18-entry stack; variant 2 = the binary kernel."""
    V = _soup_view()
    tris = oracle.soup(30000, 11).reshape(-1, 9)
    w, h, spp = 96, 64, 2
    eh, er = _oracle(oracle, tris, V, w, h, spp)
    cfg("trace.variant", variant, 0)
    cfg("trace.stack_cap", cap, 0)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        assert s.wide_arity == 8
        hits, rgba, _ = s.render(cam, w, h, spp)
    _same(hits, rgba, eh, er)


def test_wide8_presets_and_zero_directions(R, oracle, cfg):
    from gpu_raytracer_amd import scenes as S
    from test_wide_gpu import _cams
    for tris, view, (w, h, spp) in [(S.cornell_tris(), S.CORNELL_VIEW, (64, 64, 1)),
                                    (S.bunny_substitute_tris(), S.BUNNY_VIEW, (160, 90, 1)),
                                    (S.sponza_substitute_tris(), S.SPONZA_VIEW, (96, 54, 2))]:
        tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
        eh, er = _oracle(oracle, tris, view, w, h, spp)
        cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        with R.Scene.from_soup(tris) as s:
            s.build()
            hits, rgba, _ = s.render(cam, w, h, spp)
        _same(hits, rgba, eh, er)
    tris = oracle.soup(20000, 12).reshape(-1, 9)
    w, h = 64, 48
    for cam, ocam in [
        _cams(R, oracle, (0.5, 0.5, -1.0), (-0.5, 0.0, 1.0), (1.0 / 64, 0.0, 0.0), (0.0, 0.0, 1.0 / 64)),
        _cams(R, oracle, (0.5, 0.5, -1.5), (-10.5 / 64, 0.4, 1.0), (1.0 / 64, 0.0, 0.0), (0.0, -1.0 / 64, 0.0)),
    ]:
        exp = oracle.build(tris)
        eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, 1)
        with R.Scene.from_soup(tris) as s:
            s.build()
            hits, rgba, _ = s.render(cam, w, h, 1)
        _same(hits, rgba, eh, oracle.shade(eh, w, h, 1))


@pytest.mark.parametrize("lanes", [16, 32, 64])
@pytest.mark.parametrize("cap", [1, 4, 24])
def test_wide8_coop_full_frame(R, oracle, cfg, lanes, cap):
    V = _soup_view()
    tris = oracle.soup(40000, 11).reshape(-1, 9)
    w, h, spp = 200, 120, 2
    eh, er = _oracle(oracle, tris, V, w, h, spp)
    cfg("trace.coop_cap", cap, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(cam, w, h, spp)
            _same(hits, rgba, eh, er)


@pytest.mark.parametrize("lanes", [16, 64])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_wide8_tiles(R, oracle, cfg, P, lanes):
    """One rank's tiles (64-thread blocks, Moller-Trumbore first, heavy-ray
    queue at the tile cap), emulated P-rank frames, three successive frames."""
    V = _soup_view()
    tris = oracle.soup(30000, 14).reshape(-1, 9)
    w, h, spp = 170, 90, 2
    eh, er = _oracle(oracle, tris, V, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.coop_cap_tiles", 6, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(cam, w, h, spp, ngpus=P)
            _same(hits, rgba, eh, er)


@pytest.mark.parametrize("lanes", [16, 64])
def test_wide8_coop_frontier_handoff(R, oracle, cfg, lanes):
    base = oracle.soup(8, 21).reshape(-1, 9)
    tris = np.concatenate([np.repeat(base, 75, axis=0), oracle.soup(2000, 22).reshape(-1, 9) * 0.05 + 0.45])
    tris = np.ascontiguousarray(tris, np.float32)
    V = _soup_view()
    w, h = 96, 64
    eh, er = _oracle(oracle, tris, V, w, h, 1)
    cfg("trace.coop_cap", 1, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render(cam, w, h, 1)
    _same(hits, rgba, eh, er)


@pytest.mark.parametrize("cap", [2, 0])
def test_wide8_shadow(R, oracle, cfg, cap):
    from gpu_raytracer_amd.scenes import LIGHTS
    V = _soup_view()
    tris = oracle.soup(40000, 31).reshape(-1, 9)
    w, h, spp = 128, 96, 2
    exp = oracle.build(tris)
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, er, _ = oracle.render_shadow(exp["nodes"], tris, ocam, w, h, spp, LIGHTS["soup"], 0.2)
    cfg("trace.stack_cap", cap, 0)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render_shadow(cam, w, h, spp, LIGHTS["soup"], 0.2)
    assert np.array_equal(hits["prim"], eh["prim"])
    assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
    assert np.array_equal(rgba, er)


@pytest.mark.parametrize("wave", [0, 1])
@pytest.mark.parametrize("cap", [3, 0])
def test_wide8_path(R, oracle, cfg, wave, cap):
    from gpu_raytracer_amd.scenes import LIGHTS
    V = _soup_view()
    tris = oracle.soup(30000, 41).reshape(-1, 9)
    w, h, spp, depth, sky = 96, 64, 2, 3, 0.3
    exp = oracle.build(tris)
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, er, ecnt = oracle.render_path(exp["nodes"], tris, ocam, w, h, spp, LIGHTS["soup"], sky, depth)
    cfg("path.wavefront", wave, 1)
    cfg("trace.stack_cap", cap, 0)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render_path(cam, w, h, spp, LIGHTS["soup"], sky, depth)
        work = s.render_path_work(cam, w, h, spp, LIGHTS["soup"], sky, depth)
    assert np.array_equal(hits["prim"], eh["prim"])
    assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
    assert np.array_equal(rgba, er)
    assert work[2] == ecnt[2]


def test_wide8_cache_roundtrip_and_arity_switch(R, oracle, cfg, tmp_path):
    """An 8-ary BVH cache restores 8-ary records (renders identically) even
    when the current setting is 4-ary, and a 4-ary one the other way round."""
    V = _soup_view()
    tris = oracle.soup(20000, 51).reshape(-1, 9)
    w, h = 80, 60
    eh, er = _oracle(oracle, tris, V, w, h, 1)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    p8, p4 = str(tmp_path / "b8.rtbvh"), str(tmp_path / "b4.rtbvh")
    with R.Scene.from_soup(tris) as s:
        s.build()
        s.save_bvh(p8)
    cfg("build.wide_arity", 4, 4)
    with R.Scene.from_soup(tris) as s:
        s.build()
        s.save_bvh(p4)
        s.load_bvh(p8)
        assert s.wide_arity == 8
        hits, rgba, _ = s.render(cam, w, h, 1)
        _same(hits, rgba, eh, er)
    cfg("build.wide_arity", 8, 4)
    with R.Scene.from_soup(tris) as s:
        s.load_bvh(p4)
        assert s.wide_arity == 4
        hits, rgba, _ = s.render(cam, w, h, 1)
        _same(hits, rgba, eh, er)


def test_wide8_headline_1m(R, oracle, cfg):
    """soup-1M 1080p, full frame and 8 emulated ranks' tiles (heavy-ray queue
    at its default cap), successive frames."""
    V = _soup_view()
    tris = oracle.soup(1_000_000, 1).reshape(-1, 9)
    w, h = 1920, 1080
    eh, er = _oracle(oracle, tris, V, w, h, 1)
    cfg("render.emulate", 1, 0)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for P in (1, 8, 8):
            hits, rgba, _ = s.render(cam, w, h, 1, ngpus=P)
            _same(hits, rgba, eh, er)
