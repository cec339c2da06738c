"""Cooperative heavy rays (trace.coop_cap / trace.coop_cap_tiles, DESIGN.md
"Cooperative heavy rays"): primary rays still traversing after the cap are
queued and finished by k_trace_coop, a group of 16/32/64 lanes per ray, folding the leaves in
§9.7 preorder.  Every frame must stay bit-identical to the CPU oracle (hits
and RGBA) whatever the cap, the queue capacity (a full queue leaves rays to
their own lane), the samples per pixel (a pixel resumes at its deferred
sample with the colour sums of the earlier ones), the full-frame and the
per-rank tiled kernels, successive frames (tile/pixel order on), and the
frontier hand-off to the binary traversal (a scene of identical triangles,
whose boxes all overlap, overflows the frontier)."""
import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu


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
    yield set_
    for k, d in reversed(keys):
        R.config_set(k, d)


def _frame(oracle, tris, view, w, h, spp):
    exp = oracle.build(tris)
    cam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, cam, w, h, spp)
    return eh, oracle.shade(eh, w, h, spp)


def _same_hits(a, b):
    return all(np.array_equal(bits(a[k]), bits(b[k])) for k in ("t", "u", "v", "prim"))


def _soup_view():
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    return SOUP_VIEW


@pytest.mark.parametrize("lanes", [16, 32, 64])
@pytest.mark.parametrize("cap", [1, 2, 5, 16, 40])
@pytest.mark.parametrize("spp", [1, 3])
def test_coop_full_frame(R, oracle, cfg, cap, spp, lanes):
    V = _soup_view()
    tris = oracle.soup(40000, 11).reshape(-1, 9)
    w, h = 200, 120
    eh, er = _frame(oracle, tris, V, w, h, spp)
    cfg("trace.coop_cap", cap, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(3):  # frames 2 and 3 also run the tile and pixel order
            hits, rgba, _ = s.render(cam, w, h, spp)
            assert np.array_equal(rgba, er), (cap, spp, frame)
            assert _same_hits(hits, eh), (cap, spp, frame)


def test_coop_changes_work_not_result(R, oracle, cfg):
    """The queue really runs: the kernels' own fetch counters change with the
    cap (the cooperative pass speculates), the image does not."""
    V = _soup_view()
    tris = oracle.soup(40000, 12).reshape(-1, 9)
    w, h = 160, 96
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        base = s.render_work(cam, w, h, 1)
        _, img0, _ = s.render(cam, w, h, 1)
        cfg("trace.coop_cap", 2, -1)
        coop = s.render_work(cam, w, h, 1)
        _, img1, _ = s.render(cam, w, h, 1)
    assert np.array_equal(img0, img1)
    assert not np.array_equal(base, coop)


@pytest.mark.parametrize("qmax", [1, 7, 100])
def test_coop_queue_full(R, oracle, cfg, qmax):
    V = _soup_view()
    tris = oracle.soup(30000, 13).reshape(-1, 9)
    w, h, spp = 150, 100, 2
    eh, er = _frame(oracle, tris, V, w, h, spp)
    cfg("trace.coop_max", qmax, 65536)
    cfg("trace.coop_cap", 3, -1)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(2):
            hits, rgba, _ = s.render(cam, w, h, spp)
            assert np.array_equal(rgba, er), (qmax, frame)
            assert _same_hits(hits, eh), (qmax, frame)


@pytest.mark.parametrize("lanes", [16, 64])
@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("cap", [2, 24])
def test_coop_tiles(R, oracle, cfg, P, cap, lanes):
    """One rank's tiles (packed slabs, 64-thread blocks) through the queue:
    emulated P-rank frames == the oracle, three successive frames."""
    V = _soup_view()
    tris = oracle.soup(30000, 14).reshape(-1, 9)
    w, h, spp = 170, 90, 2
    eh, er = _frame(oracle, tris, V, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.coop_cap_tiles", cap, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(cam, w, h, spp, ngpus=P)
            assert np.array_equal(rgba, er), (P, cap, frame)
            assert _same_hits(hits, eh), (P, cap, frame)


@pytest.mark.parametrize("lanes", [16, 32, 64])
def test_coop_frontier_handoff(R, oracle, cfg, lanes):
    """All-overlapping boxes (600 copies of a few triangles, and a cluster):
    the frontier outgrows its 256 entries and hands over to the binary
    traversal from its head entry -- still the oracle's hits."""
    base = oracle.soup(8, 21).reshape(-1, 9)
    tris = np.concatenate([np.repeat(base, 75, axis=0), oracle.soup(2000, 22).reshape(-1, 9) * 0.05 + 0.45])
    tris = np.ascontiguousarray(tris, np.float32)
    V = _soup_view()
    w, h = 96, 64
    eh, er = _frame(oracle, tris, V, w, h, 1)
    cfg("trace.coop_cap", 1, -1)
    cfg("trace.coop_lanes", lanes, 32)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render(cam, w, h, 1)
    assert np.array_equal(rgba, er)
    assert _same_hits(hits, eh)


def test_coop_headline_1m(R, oracle, cfg):
    """The soup-1M 1080p frame with the tile default cap applied to the full
    frame (the rays past 48 wide steps, ~10 % of the frame) == the oracle."""
    V = _soup_view()
    tris = oracle.soup(1_000_000, 1).reshape(-1, 9)
    w, h = 1920, 1080
    eh, er = _frame(oracle, tris, V, w, h, 1)
    cfg("trace.coop_cap", 48, -1)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(2):
            hits, rgba, _ = s.render(cam, w, h, 1)
            assert np.array_equal(rgba, er), frame
            assert _same_hits(hits, eh), frame


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("cap", [0, 14, 15, 16])
def test_tile_stack_depths(R, oracle, cfg, P, cap):
    """One rank's tiles run 64-thread blocks with 16-entry stacks (14 for the
    256-thread full frames) and the 1-spp kernel: stack depths up to 16,
    through the overflow hand-off and the queue, == the oracle, on a scene of
    overlapping clusters."""
    base = oracle.soup(8, 21).reshape(-1, 9)
    tris = np.concatenate([np.repeat(base, 40, axis=0), oracle.soup(20000, 22).reshape(-1, 9) * 0.3 + 0.35,
                           oracle.soup(20000, 23).reshape(-1, 9)])
    tris = np.ascontiguousarray(tris, np.float32)
    V = _soup_view()
    w, h = 112, 80
    eh, er = _frame(oracle, tris, V, w, h, 1)
    cfg("render.emulate", 1, 0)
    cfg("trace.stack_cap", cap, 0)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(2):
            hits, rgba, _ = s.render(cam, w, h, 1, ngpus=P)
            assert np.array_equal(rgba, er), (P, cap, frame)
            assert _same_hits(hits, eh), (P, cap, frame)


def test_orbit_frame_8_ranks_1m(R, oracle, cfg):
    """The bench's orbiting camera at step 8 (soup-1M 1080p), where a few
    rays need more than 14 stack entries: the emulated 8-rank frame (16-entry
    tile stacks) and the full frame (14 entries, binary hand-off) == the
    oracle over the whole image."""
    import bench
    V = _soup_view()
    tris = oracle.soup(1_000_000, 1).reshape(-1, 9)
    w, h = 1920, 1080
    eye = bench.orbit_view(V, 8)

    class _V:
        pass
    view = _V()
    view.eye, view.at, view.up, view.vfov = eye, V.at, V.up, V.vfov
    eh, er = _frame(oracle, tris, view, w, h, 1)
    cfg("render.emulate", 1, 0)
    cam = R.camera_look_at(eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for P in (8, 1):
            hits, rgba, _ = s.render(cam, w, h, 1, ngpus=P)
            assert np.array_equal(rgba, er), P
            assert _same_hits(hits, eh), P


def test_order_with_queue(R, oracle, cfg):
    """A queue-on frame's next tile order is sorted by k_trace_coop's block 0
    (the side-stream and fold-block alternatives were removed in r06,
    profiles/rejected_knobs_r06.patch) -- four successive frames each, full
    frames and one rank's tiles (P = 3), and full frames on torch's default
    stream with no host sync between them: every frame == the oracle."""
    import torch
    V = _soup_view()
    tris = oracle.soup(40000, 12).reshape(-1, 9)
    w, h, spp = 210, 118, 1
    eh, er = _frame(oracle, tris, V, w, h, spp)
    cfg("trace.coop_cap", 16, -1)
    cfg("trace.coop_cap_tiles", 24, -1)
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(4):
            hits, rgba, _ = s.render(cam, w, h, spp)
            assert np.array_equal(rgba, er), ("full", frame)
            assert _same_hits(hits, eh), ("full", frame)
        cfg("render.emulate", 1, 0)
        for frame in range(4):
            hits, rgba, _ = s.render(cam, w, h, spp, ngpus=3)
            assert np.array_equal(rgba, er), ("tiles", frame)
        cur = torch.cuda.current_stream()
        imgs = [torch.zeros(w * h, dtype=torch.int32, device="cuda") for _ in range(4)]
        for img in imgs:
            s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), stream=cur.cuda_stream)
        torch.cuda.synchronize()
        for i, img in enumerate(imgs):
            assert np.array_equal(img.cpu().numpy().view(np.uint8), er), ("null stream", i)


def test_coop_skip_probe_frames(R, oracle, cfg):
    """The queue skip (automatic caps): a shape whose queue-on frame queued
    fewer than 64 rays runs its next 15 frames without the queue (the order
    folded in k_trace), then probes with it again; a heavy shape keeps it.
    20 frames of a light scene (the bunny substitute's sphere) and of a soup,
    every one == the oracle."""
    from gpu_raytracer_amd import scenes as S
    for tris, view in ((np.ascontiguousarray(S.tris_for("bunny"), np.float32).reshape(-1, 9), S.VIEWS["bunny"]),
                       (oracle.soup(40000, 13).reshape(-1, 9), _soup_view())):
        w, h, spp = 160, 96, 1
        eh, er = _frame(oracle, tris, view, w, h, spp)
        cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        with R.Scene.from_soup(tris) as s:
            s.build()
            for frame in range(20):
                hits, rgba, _ = s.render(cam, w, h, spp)
                assert np.array_equal(rgba, er), frame
                assert _same_hits(hits, eh), frame
