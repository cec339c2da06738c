"""GPU tests with poisoned device memory (rt_config_set("debug.poison", 1)):
every buffer the library allocates is filled with 0xFF bytes before first
use, so a kernel that reads a byte nothing wrote -- a record slot, a map
entry, a hit -- reads the same wrong value every run instead of whatever the
allocator recycled.  Under poison the build (sorted indices, every node,
every 4-/8-ary wide record) and the trace (hits, images; full frames, one
rank's tiles with the heavy-ray queue, successive frames) must still equal
the CPU oracle bit for bit.  VERDICT r02 "What's weak" 2: the one recorded
wrong-hit failure (8-ary, Cornell 64x64, fresh scene) is re-run here on the
same scenes with every allocation poisoned."""
import numpy as np
import pytest

from conftest import bits
from test_wide_gpu import _check_wide

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


@pytest.fixture()
def poison(R):
    R.config_set("debug.poison", 1)
    yield
    for k, v in (("debug.poison", 0), ("build.wide_arity", 4), ("render.emulate", 0),
                 ("trace.coop_cap", -1), ("trace.coop_cap_tiles", -1)):
        R.config_set(k, v)


def _scenes(oracle):
    from gpu_raytracer_amd import scenes as S
    out = [("cornell", S.cornell_tris(), S.CORNELL_VIEW, (64, 64, 1)),
           ("bunny", S.bunny_substitute_tris(), S.BUNNY_VIEW, (160, 90, 1)),
           ("sponza", S.sponza_substitute_tris(), S.SPONZA_VIEW, (96, 54, 2))]
    for n in (2, 3, 5, 9, 32):
        out.append((f"soup{n}", oracle.soup(n, 60 + n), S.SOUP_VIEW, (48, 32, 1)))
    return [(name, np.ascontiguousarray(t, np.float32).reshape(-1, 9), v, f) for name, t, v, f in out]


def _same(name, hits, rgba, eh, er):
    d = np.nonzero(hits["prim"] != eh["prim"])[0]
    assert len(d) == 0, (f"{name}: {len(d)} of {len(eh)} prims differ; first {d[:8].tolist()}: got "
                         f"{hits['prim'][d[:8]].tolist()}, expected {eh['prim'][d[:8]].tolist()}")
    for f in ("t", "u", "v"):
        assert np.array_equal(bits(hits[f]), bits(eh[f])), (name, f)
    assert np.array_equal(rgba, er), name


@pytest.mark.parametrize("arity", [4, 8])
def test_poisoned_build_and_render(R, oracle, poison, arity):
    for name, tris, view, (w, h, spp) in _scenes(oracle):
        _check_wide(R, tris, arity)  # every record restates the cut (poison stays on)
        exp = oracle.build(tris)
        ocam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
        er = oracle.shade(eh, w, h, spp)
        cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        R.config_set("build.wide_arity", arity)
        with R.Scene.from_soup(tris) as s:
            s.build()
            assert s.wide_arity == arity
            got = s.read_bvh()
            assert np.array_equal(got["vals"], exp["vals"]), name
            assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32)), name
            for frame in range(2):  # the second frame runs the tile and pixel order
                hits, rgba, _ = s.render(cam, w, h, spp)
                _same(f"{name} frame {frame}", hits, rgba, eh, er)


@pytest.mark.parametrize("arity", [4, 8])
def test_poisoned_tiles_and_queue(R, oracle, poison, arity):
    """One rank's tiles (emulated P = 3 and 8) with the heavy-ray queue at a
    low cap, and a full frame with the queue on: queue entries, counters,
    slabs and order maps all start poisoned."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(20000, 71).reshape(-1, 9)
    w, h, spp = 130, 70, 2
    exp = oracle.build(tris)
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    er = oracle.shade(eh, w, h, spp)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    R.config_set("build.wide_arity", arity)
    R.config_set("render.emulate", 1)
    R.config_set("trace.coop_cap_tiles", 6)
    R.config_set("trace.coop_cap", 6)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for P in (1, 3, 3, 8, 8, 1):
            hits, rgba, _ = s.render(cam, w, h, spp, ngpus=P)
            _same(f"P={P}", hits, rgba, eh, er)
