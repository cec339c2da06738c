"""Randomised parity (seeded, bounded): random scenes -- uniform soups,
clustered and flat soups, near-degenerate slivers, the Cornell and bunny
presets -- seen from random cameras (eye anywhere on a sphere around the
scene, including inside its box), rendered with random settings (4-/8-ary
records, traversal variant, stack cap, heavy-ray queue cap and lanes, spp,
emulated ranks P = 1/2/3/8) for two successive frames, against the CPU
oracle: every hit (t, u, v, prim bit for bit) and the image.  A complement
to the targeted tests: the combinations nobody wrote down."""
import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu

KNOBS = {"build.wide_arity": 4, "trace.variant": 0, "trace.stack_cap": 0, "trace.coop_cap": -1,
         "trace.coop_cap_tiles": -1, "trace.coop_lanes": 32, "render.emulate": 0}


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    yield rt
    for k, v in KNOBS.items():
        rt.config_set(k, v)


def _scene(oracle, rng):
    from gpu_raytracer_amd import scenes as S
    kind = int(rng.integers(0, 6))
    if kind == 0:
        return np.ascontiguousarray(S.cornell_tris(), np.float32).reshape(-1, 9)
    if kind == 1:
        return np.ascontiguousarray(S.bunny_substitute_tris(), np.float32).reshape(-1, 9)
    n = int(rng.integers(2, 20000))
    t = oracle.soup(n, int(rng.integers(1, 10_000))).reshape(-1, 9).copy()
    if kind == 3:    # a few dense clusters
        c = rng.random((4, 3)).astype(np.float32)
        k = rng.integers(0, 4, n)
        t = (t - t.reshape(-1, 3, 3).mean(1).repeat(3, 0).reshape(-1, 9)) * 0.3 + np.tile(c[k], 3)
    elif kind == 4:  # flat: every vertex on one plane
        t[:, 1::3] = np.float32(0.5)
    elif kind == 5:  # slivers: v2 nearly on the line v0-v1
        t[:, 6:9] = t[:, 0:3] + (t[:, 3:6] - t[:, 0:3]) * np.float32(0.5) + np.float32(1e-6)
    return np.ascontiguousarray(t, np.float32)


def _camera(R, oracle, tris, rng, w, h):
    lo, hi = tris.reshape(-1, 3).min(0).astype(np.float64), tris.reshape(-1, 3).max(0).astype(np.float64)
    c, ext = (lo + hi) / 2, float(np.linalg.norm(hi - lo)) + 1e-3
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    eye = c + u * ext * float(rng.uniform(0.3, 2.0))   # sometimes inside the box
    at = c + rng.normal(size=3) * ext * 0.1
    up = rng.normal(size=3)
    fov = float(rng.uniform(20, 80))
    if np.linalg.norm(np.cross(at - eye, up)) < 1e-6:
        up = np.array([0.0, 0.0, 1.0]) if abs(u[2]) < 0.9 else np.array([1.0, 0.0, 0.0])
    return (R.camera_look_at(tuple(eye), tuple(at), tuple(up), fov, w, h),
            oracle.camera_look_at(eye, at, up, fov, w, h))


@pytest.mark.parametrize("seed", range(24))
def test_random_scene_camera_settings(R, oracle, seed):
    rng = np.random.default_rng(1000 + seed)
    tris = _scene(oracle, rng)
    w, h, spp = int(rng.integers(8, 160)), int(rng.integers(8, 120)), int(rng.integers(1, 4))
    cam, ocam = _camera(R, oracle, tris, rng, w, h)
    knobs = {"build.wide_arity": int(rng.choice([4, 8])), "trace.variant": int(rng.choice([0, 0, 2])),
             "trace.stack_cap": int(rng.choice([0, 0, 1, 3])), "trace.coop_cap": int(rng.choice([-1, 0, 2, 24, 96])),
             "trace.coop_cap_tiles": int(rng.choice([-1, 0, 4])), "trace.coop_lanes": int(rng.choice([16, 32, 64]))}
    P = int(rng.choice([1, 1, 2, 3, 8]))
    exp = oracle.build(tris)
    eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    er = oracle.shade(eh, w, h, spp)
    try:
        for k, v in knobs.items():
            R.config_set(k, v)
        R.config_set("render.emulate", 1 if P > 1 else 0)
        with R.Scene.from_soup(tris) as s:
            s.build()
            for frame in range(2):
                hits, rgba, _ = s.render(cam, w, h, spp, ngpus=P)
                d = np.nonzero(hits["prim"] != eh["prim"])[0]
                assert len(d) == 0, (f"seed {seed} frame {frame} n {len(tris)} {w}x{h}x{spp} P {P} {knobs}: "
                                     f"{len(d)} prims differ, first {d[:6].tolist()}")
                for f in ("t", "u", "v"):
                    assert np.array_equal(bits(hits[f]), bits(eh[f])), f
                assert np.array_equal(rgba, er)
    finally:
        for k, v in KNOBS.items():
            R.config_set(k, v)
