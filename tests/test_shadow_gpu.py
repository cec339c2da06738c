"""GPU tests of the shadow mode (contract in
DESIGN.md "Shadow mode"): one any-hit shadow ray per primary hit, Lambert +
ambient shading -- bit-exact against the CPU oracle's orc_render_shadow for
the wide and the binary traversal, with forced stack overflows."""
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


def _check(R, oracle, tris, view, light, w, h, spp, variant=0, cap=14, ambient=0.2):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    exp = oracle.build(tris)
    ocam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, er, _ = oracle.render_shadow(exp["nodes"], tris, ocam, w, h, spp, light, ambient)
    R.config_set("trace.variant", variant)
    R.config_set("trace.stack_cap", cap)
    cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render_shadow(cam, w, h, spp, light, ambient)
    assert np.array_equal(hits["prim"], eh["prim"])
    assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
    assert np.array_equal(rgba, er)
    return er


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("cap", [2, 14])
def test_shadow_soup(R, oracle, variant, cap):
    from gpu_raytracer_amd.scenes import SOUP_VIEW, LIGHTS
    tris = oracle.soup(40000, 31).reshape(-1, 9)
    img = _check(R, oracle, tris, SOUP_VIEW, LIGHTS["soup"], 128, 96, 2, variant, cap)
    lum = img.reshape(-1, 4)[:, :3].astype(np.int64).sum(1)
    assert (lum > 0).sum() > 1000           # lit and shadowed pixels both present
    assert len(np.unique(lum)) > 50


@pytest.mark.parametrize("variant", [0, 2])
def test_shadow_presets(R, oracle, variant):
    from gpu_raytracer_amd import scenes as S
    for name, tris, (w, h) in [("cornell", S.cornell_tris(), (96, 96)),
                               ("bunny", S.bunny_substitute_tris(), (160, 90)),
                               ("sponza", S.sponza_substitute_tris(), (96, 54))]:
        _check(R, oracle, tris, S.VIEWS[name], S.LIGHTS[name], w, h, 1, variant)


def test_shadow_edge_lights(R, oracle):
    """Light inside the soup, on a triangle's plane, and at the eye; ambient 0 and 1."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = oracle.soup(5000, 32).reshape(-1, 9)
    for light, amb in [((0.5, 0.5, 0.5), 0.2), (tuple(float(x) for x in tris[10, :3]), 0.0),
                       (SOUP_VIEW.eye, 1.0), ((0.5, 0.5, -1.5), 0.5)]:
        _check(R, oracle, tris, SOUP_VIEW, light, 64, 48, 1, 0, 14, amb)


def test_shadow_empty_and_single(R, oracle):
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    _check(R, oracle, oracle.soup(1, 33).reshape(-1, 9), SOUP_VIEW, (2.0, 3.0, -2.0), 32, 24, 1)
    _check(R, oracle, oracle.soup(2, 33).reshape(-1, 9), SOUP_VIEW, (2.0, 3.0, -2.0), 32, 24, 1)


def test_shadow_work_counts(R, oracle):
    from gpu_raytracer_amd.scenes import SOUP_VIEW, LIGHTS
    tris = oracle.soup(100000, 34).reshape(-1, 9)
    w, h = 160, 90
    cam = R.camera_look_at(SOUP_VIEW.eye, SOUP_VIEW.at, SOUP_VIEW.up, SOUP_VIEW.vfov, w, h)
    R.config_set("trace.variant", 0)
    with R.Scene.from_soup(tris) as s:
        s.build()
        prim = s.render_work(cam, w, h, 1)
        both = s.render_shadow_work(cam, w, h, 1, LIGHTS["soup"], 0.2)
    assert both[0] > prim[0] and both[1] > prim[1]
