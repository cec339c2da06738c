"""Samples in lanes (trace.spp_lanes, k_trace_sl; DESIGN.md (e) "Samples in
lanes for one rank's tiles"): at 2/4/8/16 spp a pixel's samples are traced
by adjacent lanes, one ray each, and its colour is the loop's ordered sum
over them (shuffles); a sample the heavy-ray queue takes is finished by
k_trace_coop alone (kCoopOne) and its pixel's colour by k_coop_resolve from
the hits.  Every frame must equal the CPU oracle bit for bit -- hits and
RGBA -- across the queue caps (many queued samples, several per pixel), a
full or tiny queue, no hits buffer (queue off), forced stack overflows
(binary hand-off), odd frame sizes, successive frames (tile order), the
per-rank tiles and full frames (spp_lanes = 2, the default; 1 = tiles only)."""
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


def _view():
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    return SOUP_VIEW


def _frame(oracle, tris, w, h, spp):
    V = _view()
    exp = oracle.build(tris)
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, cam, w, h, spp)
    return eh, oracle.shade(eh, w, h, spp)


def _cam(R, w, h):
    V = _view()
    return R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)


def _same_hits(a, b):
    return all(np.array_equal(bits(a[k]), bits(b[k])) for k in ("t", "u", "v", "prim"))


@pytest.fixture(scope="module")
def scene30k(oracle):
    return oracle.soup(30000, 21).reshape(-1, 9)


@pytest.mark.parametrize("spp", [2, 4, 8, 16])
@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("cap", [0, 1, 6])
def test_spp_lanes_tiles(R, oracle, cfg, scene30k, spp, P, cap):
    """Emulated P-rank frames through k_trace_sl: queue off (cap 0), every
    sample queued after 1 step (most pixels resolved from hits), and a cap
    that queues a fraction; three successive frames (tile order on: with the
    queue off, block 0 of the second frame sorts the order the third uses)."""
    w, h = 70, 45
    eh, er = _frame(oracle, scene30k, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.coop_cap_tiles", cap, -1)
    with R.Scene.from_soup(scene30k) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=P)
            assert np.array_equal(rgba, er), (spp, P, cap, frame)
            assert _same_hits(hits, eh), (spp, P, cap, frame)


@pytest.mark.parametrize("qmax", [1, 9, 200])
def test_spp_lanes_queue_capacity(R, oracle, cfg, scene30k, qmax):
    """A queue that fills: the samples that find their shard full trace on
    in their own lane, the others are resolved."""
    w, h, spp, P = 90, 50, 4, 3
    eh, er = _frame(oracle, scene30k, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.coop_cap_tiles", 2, -1)
    cfg("trace.coop_max", qmax, 65536)
    with R.Scene.from_soup(scene30k) as s:
        s.build()
        hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=P)
        assert np.array_equal(rgba, er), qmax
        assert _same_hits(hits, eh), qmax


def test_spp_lanes_rgba_only(R, oracle, cfg, scene30k):
    """No hits buffer: the queue needs the hits to resolve, so it is off and
    every sample finishes in its lane -- the image still equals the oracle."""
    w, h, spp = 64, 40, 4
    _, er = _frame(oracle, scene30k, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.coop_cap_tiles", 1, -1)
    with R.Scene.from_soup(scene30k) as s:
        s.build()
        for P in (2, 8):
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, hits=False, ngpus=P)
            assert hits is None
            assert np.array_equal(rgba, er), P


@pytest.mark.parametrize("stack", [1, 3])
def test_spp_lanes_stack_overflow(R, oracle, cfg, scene30k, stack):
    """Stack caps 1/3 send most rays through the binary hand-off, with and
    without the queue in front of it."""
    w, h, spp = 60, 44, 8
    eh, er = _frame(oracle, scene30k, w, h, spp)
    cfg("render.emulate", 1, 0)
    cfg("trace.stack_cap", stack, 0)
    with R.Scene.from_soup(scene30k) as s:
        s.build()
        for cap in (0, 4):
            R.config_set("trace.coop_cap_tiles", cap)
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=3)
            assert np.array_equal(rgba, er), (stack, cap)
            assert _same_hits(hits, eh), (stack, cap)
        R.config_set("trace.coop_cap_tiles", -1)


@pytest.mark.parametrize("spp", [2, 4, 16])
@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("wg", [64, 256])
def test_spp_lanes_full_frames(R, oracle, cfg, scene30k, spp, cap, wg):
    """trace.spp_lanes = 2: full frames too (256- and 64-thread blocks), with
    and without the queue; odd frame size; three frames."""
    w, h = 77, 41
    eh, er = _frame(oracle, scene30k, w, h, spp)
    cfg("trace.spp_lanes", 2, 2)
    cfg("trace.coop_cap", cap, -1)
    cfg("trace.wg", wg, 256)
    with R.Scene.from_soup(scene30k) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp)
            assert np.array_equal(rgba, er), (spp, cap, wg, frame)
            assert _same_hits(hits, eh), (spp, cap, wg, frame)


def test_spp_lanes_equals_loop_kernel(R, cfg):
    """The same frame of a 300K soup through k_trace_sl and through the loop
    kernel (spp_lanes = 0), per rank at P = 8 and in full: identical slabs,
    hits and images (no oracle: a device-only comparison at a larger size)."""
    import torch
    w, h, spp, P = 480, 270, 4, 8
    cam = _cam(R, w, h)
    with R.Scene.generate_soup(300_000, 3) as s:
        s.build()
        outs = {}
        for mode in (0, 1):
            R.config_set("trace.spp_lanes", mode)
            got = []
            for r in range(P):
                nb = R.tiles_for_rank(w, h, r, P)
                slab = torch.zeros(nb * 256, dtype=torch.int32, device="cuda")
                sh = torch.zeros(nb * 256 * spp * 4, dtype=torch.float32, device="cuda")
                torch.cuda.synchronize()  # the zero fills, before the scene's stream writes
                for _ in range(3):  # the third frame runs the order sorted in the second's block 0
                    s.render_tiles_device(cam, w, h, spp, r, P, slab.data_ptr(), sh.data_ptr())
                torch.cuda.synchronize()
                got.append((slab.cpu().numpy().copy(), sh.cpu().numpy().view(np.uint32).copy()))
            outs[mode] = got
        full = {}
        for mode in (0, 2):
            R.config_set("trace.spp_lanes", mode)
            img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
            hb = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            for _ in range(2):
                s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hb.data_ptr())
            torch.cuda.synchronize()
            full[mode] = (img.cpu().numpy().copy(), hb.cpu().numpy().view(np.uint32).copy())
        R.config_set("trace.spp_lanes", 2)
        for r in range(P):
            assert np.array_equal(outs[0][r][0], outs[1][r][0]), r
            assert np.array_equal(outs[0][r][1], outs[1][r][1]), r
        assert np.array_equal(full[0][0], full[2][0])
        assert np.array_equal(full[0][1], full[2][1])


def test_spp_lanes_folded_order_large_frames(R, cfg):
    """k_trace_sl full frames sort the next frame's tile order in their block
    0 (a loop over any tile count): 9216 tiles, five frames
    (the order is sorted in frame 2 on, used from frame 3), each identical to
    the loop kernel's frame -- a tile the order dropped or repeated would
    leave its pixels unwritten (device-only comparison)."""
    import torch
    w, h, spp = 2048, 1152, 2
    cam = _cam(R, w, h)
    with R.Scene.generate_soup(300_000, 3) as s:
        s.build()
        ref = None
        for mode in (0, 2):
            cfg("trace.spp_lanes", mode, 2)
            for f in range(5):
                img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
                hb = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
                # the zero fills run on torch's stream, which the scene's stream does not wait for (and
                # torch's default stream has handle 0, i.e. "the scene's stream" to render_device)
                torch.cuda.synchronize()
                s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hb.data_ptr())
                torch.cuda.synchronize()
                got = (img.cpu().numpy().copy(), hb.cpu().numpy().view(np.uint32).copy())
                if ref is None:
                    ref = got
                    assert np.count_nonzero(ref[0]) == w * h  # alpha 255 everywhere
                if not np.array_equal(got[0], ref[0]):
                    d = np.nonzero(got[0] != ref[0])[0]
                    tiles = np.unique((d // w // 16) * 128 + (d % w) // 16)
                    pytest.fail(f"mode {mode} frame {f}: {d.size} pixels differ in {tiles.size} tiles "
                                f"{tiles[:8].tolist()}; first {[(int(p % w), int(p // w)) for p in d[:6]]}: got "
                                f"{[hex(int(v) & 0xFFFFFFFF) for v in got[0][d[:6]]]} expected "
                                f"{[hex(int(v) & 0xFFFFFFFF) for v in ref[0][d[:6]]]}; hit records of the first: got "
                                f"{got[1].reshape(-1, 4)[d[0] * spp:(d[0] + 1) * spp].tolist()} expected "
                                f"{ref[1].reshape(-1, 4)[d[0] * spp:(d[0] + 1) * spp].tolist()}")
                if not np.array_equal(got[1], ref[1]):
                    d = np.nonzero(got[1] != ref[1])[0]
                    rec = np.unique(d // 4)
                    px = rec // spp
                    pytest.fail(f"mode {mode} frame {f}: {d.size} words in {rec.size} hit records differ "
                                f"(fields {np.bincount(d % 4, minlength=4).tolist()}); first records "
                                f"{[(int(r), int(p % w), int(p // w)) for r, p in zip(rec[:6], px[:6])]}: got "
                                f"{got[1].reshape(-1, 4)[rec[:3]].tolist()} expected {ref[1].reshape(-1, 4)[rec[:3]].tolist()}; "
                                f"distinct tiles {np.unique((px // w // 16) * 128 + (px % w) // 16).size}")
