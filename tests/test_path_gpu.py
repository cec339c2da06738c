"""GPU tests of the path mode ("simple path tracing";
contract in DESIGN.md "Path mode"): diffuse paths with next-event estimation,
bit-exact against the CPU oracle's orc_render_path -- images, primary hits and
the number of rays traced -- for the wide and the binary traversal, both
workgroup shapes, forced stack overflows and several path depths."""
import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu
SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    yield rt
    rt.config_set("trace.variant", 0)
    rt.config_set("trace.stack_cap", 0)
    rt.config_set("trace.wg", 256)
    rt.config_set("path.wg", 64)
    rt.config_set("path.wavefront", 1)
    rt.config_set("path.sort", 0)
    rt.config_set("path.batch", 0)


def _cam_pair(R, oracle, eye, w00, du, dv):
    c, o = R._lib.rt_camera(), oracle.Camera()
    for name, v in (("eye", eye), ("w00", w00), ("du", du), ("dv", dv)):
        for k in range(3):
            getattr(c, name)[k] = float(np.float32(v[k]))
            getattr(o, name)[k] = float(np.float32(v[k]))
    return c, o


def _check(R, oracle, tris, view, light, w, h, spp, depth, sky=0.3, variant=0, cap=14, wg=64, cams=None, wave=None):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    exp = oracle.build(tris)
    ocam = cams[1] if cams else oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, er, ecnt = oracle.render_path(exp["nodes"], tris, ocam, w, h, spp, light, sky, depth)
    R.config_set("trace.variant", variant)
    R.config_set("trace.stack_cap", cap)
    R.config_set("path.wg", wg)
    if wave is not None:
        R.config_set("path.wavefront", wave)
    cam = cams[0] if cams else R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render_path(cam, w, h, spp, light, sky, depth)
        work = s.render_path_work(cam, w, h, spp, light, sky, depth)
    assert np.array_equal(hits["prim"], eh["prim"])
    assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
    assert np.array_equal(rgba, er)
    assert work[2] == ecnt[2]                     # same rays, so the same paths
    if variant == 2:                              # binary traversal: the oracle's own work
        assert work[0] == ecnt[0] and work[1] == ecnt[1]
    return er, ecnt


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("cap", [2, 14])
@pytest.mark.parametrize("wave", [0, 1])
def test_path_soup(R, oracle, variant, cap, wave):
    from gpu_raytracer_amd.scenes import SOUP_VIEW, LIGHTS
    tris = oracle.soup(30000, 51).reshape(-1, 9)
    img, cnt = _check(R, oracle, tris, SOUP_VIEW, LIGHTS["soup"], 96, 64, 2, 2, variant=variant, cap=cap, wave=wave)
    assert cnt[2] > 2 * 96 * 64 * 2
    assert len(np.unique(img.reshape(-1, 4)[:, :3].astype(np.int64).sum(1))) > 50


@pytest.mark.parametrize("depth", [0, 1, 4])
@pytest.mark.parametrize("wg,wave", [(64, 0), (256, 0), (64, 1)])
def test_path_presets(R, oracle, depth, wg, wave):
    from gpu_raytracer_amd import scenes as S
    for name, tris, (w, h) in [("cornell", S.cornell_tris(), (64, 64)),
                               ("bunny", S.bunny_substitute_tris(), (96, 54)),
                               ("sponza", S.sponza_substitute_tris(), (64, 36))]:
        _check(R, oracle, tris, S.VIEWS[name], S.LIGHTS[name], w, h, 2, depth, wg=wg, wave=wave)


@pytest.mark.parametrize("wave", [0, 1])
def test_path_edge_cases(R, oracle, wave):
    """Light inside the soup / at the eye, sky 0 and 1, 1- and 2-triangle
    scenes, a camera with exactly-zero direction components."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = oracle.soup(4000, 52).reshape(-1, 9)
    for light, sky in [((0.5, 0.5, 0.5), 0.0), (SOUP_VIEW.eye, 1.0)]:
        _check(R, oracle, tris, SOUP_VIEW, light, 48, 32, 1, 3, sky, wave=wave)
    for n in (1, 2):
        _check(R, oracle, oracle.soup(n, 53).reshape(-1, 9), SOUP_VIEW, (2.0, 3.0, -2.0), 32, 24, 1, 2, wave=wave)
    # d.x == 0 exactly on pixel column 10 (w00.x = -10.5/64, du.x = 1/64)
    cams = _cam_pair(R, oracle, (0.5, 0.5, -1.5), (-10.5 / 64, 0.4, 1.0), (1.0 / 64, 0.0, 0.0), (0.0, -1.0 / 64, 0.0))
    _check(R, oracle, tris, None, (0.5, 2.0, -1.0), 48, 48, 1, 2, cams=cams, wave=wave)


@pytest.mark.parametrize("wave", [0, 1])
def test_path_large_depth_and_spp(R, oracle, wave):
    from gpu_raytracer_amd import scenes as S
    _check(R, oracle, S.cornell_tris(), S.CORNELL_VIEW, S.LIGHTS["cornell"], 32, 32, 8, 8, wave=wave)


@pytest.mark.parametrize("sort", [0, 1, 2, 4])
def test_path_wavefront_matches(R, oracle, sort):
    """The wavefront schedule with ray reordering: the same image, hits and
    ray count as the oracle, and the same per-ray work as the megakernel."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW, LIGHTS
    tris = oracle.soup(30000, 54).reshape(-1, 9)
    R.config_set("path.sort", sort)
    R.config_set("path.wavefront", 0)
    tr = np.ascontiguousarray(tris, np.float32)
    cam = R.camera_look_at(SOUP_VIEW.eye, SOUP_VIEW.at, SOUP_VIEW.up, SOUP_VIEW.vfov, 80, 48)
    with R.Scene.from_soup(tr) as s:
        s.build()
        mega = s.render_path_work(cam, 80, 48, 2, LIGHTS["soup"], 0.3, 3)
    R.config_set("path.wavefront", 1)
    _, cnt = _check(R, oracle, tris, SOUP_VIEW, LIGHTS["soup"], 80, 48, 2, 3)
    with R.Scene.from_soup(tr) as s:
        s.build()
        wave = s.render_path_work(cam, 80, 48, 2, LIGHTS["soup"], 0.3, 3)
    assert np.array_equal(wave, mega)


@pytest.mark.parametrize("variant,sort", [(0, 0), (0, 1), (2, 0)])
def test_path_wavefront_batches_and_presets(R, oracle, variant, sort):
    """Small batches (several per frame, partial last batch), binary traversal,
    presets, spp 3 and depths 0 and 5."""
    from gpu_raytracer_amd import scenes as S
    R.config_set("path.wavefront", 1)
    R.config_set("path.sort", sort)
    R.config_set("path.batch", 256 * 3 * 5)
    for name, tris, (w, h), depth in [("cornell", S.cornell_tris(), (70, 50), 5),
                                      ("bunny", S.bunny_substitute_tris(), (96, 54), 0),
                                      ("sponza", S.sponza_substitute_tris(), (64, 36), 2)]:
        _check(R, oracle, tris, S.VIEWS[name], S.LIGHTS[name], w, h, 3, depth, variant=variant)
