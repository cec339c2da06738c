"""rt_render(ngpus) -- the in-library multi-GPU render (SURVEY.md §3(iii),
§8(e)): BVH replicas, tile t on replica t mod P, packed slabs gathered to the
primary (RCCL ncclGather over xGMI), unpacked there.  Every frame must equal
the single-GPU render and the CPU oracle bit-for-bit.

On a one-GPU box the RCCL code path runs with a 1-rank communicator
(render.rccl1) and the P-rank logic with every replica on the one device
(render.emulate: device copies instead of RCCL); real P-device RCCL runs when
the box has P GPUs.  Also: rt_bvh_build's device mask, rt_stage_refit, and
ordering of device work across caller streams."""
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


def _cam(R, w, h):
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    return R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)


def _oracle_frame(oracle, tris, w, h, spp):
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    exp = oracle.build(tris)
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, cam, w, h, spp)
    return eh, oracle.shade(eh, w, h, spp)


def _same_hits(a, b):
    return all(np.array_equal(bits(a[k]), bits(b[k])) for k in ("t", "u", "v", "prim"))


def test_rccl_single_rank(R, oracle, cfg):
    """rt_render(ngpus=1) through the tiled + RCCL path: dlopen of RCCL,
    ncclCommInitAll over one device, grouped ncclGather of the RGBA and hit
    slabs, both unpack kernels -- == the oracle."""
    cfg("render.rccl1", 1, 0)
    tris = oracle.soup(20000, 5).reshape(-1, 9)
    w, h, spp = 123, 77, 2
    eh, er = _oracle_frame(oracle, tris, w, h, spp)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for _ in range(3):  # later frames: tile order from the previous frame's map
            hits, rgba, ms = s.render(_cam(R, w, h), w, h, spp)
            assert ms > 0
            assert np.array_equal(rgba, er)
            assert _same_hits(hits, eh)


@pytest.mark.parametrize("P", [2, 3, 8])
def test_emulated_ranks(R, oracle, cfg, P):
    """P ranks on one device (render.emulate): P replicas built (bit-identical
    BVHs), per-rank tile deal and tile order over 3 successive frames, gather,
    unpack -- every frame == the oracle, hits included."""
    cfg("render.emulate", 1, 0)
    tris = oracle.soup(30000, 7).reshape(-1, 9)
    w, h, spp = 250, 138, 1
    eh, er = _oracle_frame(oracle, tris, w, h, spp)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for frame in range(3):
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=P)
            assert np.array_equal(rgba, er), (P, frame)
            assert _same_hits(hits, eh), (P, frame)
        assert s.replicas() == [0] * P


def test_emulated_ranks_spp_and_odd_frames(R, oracle, cfg):
    cfg("render.emulate", 1, 0)
    tris = oracle.soup(5000, 9).reshape(-1, 9)
    with R.Scene.from_soup(tris) as s:
        s.build()
        for (w, h, spp, P) in [(17, 33, 3, 3), (16, 16, 1, 4), (1, 1, 1, 2), (64, 8, 4, 8)]:
            eh, er = _oracle_frame(oracle, tris, w, h, spp)
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=P)
            assert np.array_equal(rgba, er), (w, h, spp, P)
            assert _same_hits(hits, eh), (w, h, spp, P)


def test_real_multi_gpu(R, oracle):
    """Real RCCL across devices (runs only on a box with >= 2 GPUs)."""
    nd = R.device_count()
    if nd < 2:
        pytest.skip("one GPU: real multi-device RCCL covered by the 8-GPU driver run")
    tris = oracle.soup(50000, 3).reshape(-1, 9)
    w, h, spp = 320, 200, 1
    eh, er = _oracle_frame(oracle, tris, w, h, spp)
    with R.Scene.from_soup(tris) as s:
        s.build(device_mask=(1 << nd) - 1)
        assert s.replicas() == list(range(nd))
        for P in sorted({2, nd}):
            hits, rgba, _ = s.render(_cam(R, w, h), w, h, spp, ngpus=P)
            assert np.array_equal(rgba, er) and _same_hits(hits, eh), P


def test_build_device_mask(R, oracle):
    tris = oracle.soup(3000, 2).reshape(-1, 9)
    with R.Scene.from_soup(tris) as s:
        s.build(device_mask=1)
        assert s.replicas() == [0]
        got = s.read_bvh()
    exp = oracle.build(tris)
    assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32))


@pytest.mark.parametrize("n,seed,clustered", [(1, 1, False), (2, 1, False), (777, 3, False), (100003, 4, False),
                                              (60000, 5, True)])
def test_stage_refit(R, oracle, n, seed, clustered):
    """rt_stage_refit (K4..K7w over given sorted keys/vals) == the oracle's
    node records: children, escape links and every AABB bit-exact."""
    tris = oracle.soup(n, seed).reshape(-1, 9)
    if clustered:  # many equal Morton keys: long equal-key runs cross refit blocks
        tris = (np.round(tris * 8.0) / 8.0).astype(np.float32)
    exp = oracle.build(tris)
    nodes = R.stage_refit(exp["keys"], exp["vals"], tris)
    assert np.array_equal(nodes.view(np.uint32), exp["nodes"].view(np.uint32))


def test_caller_stream_ordering(R, oracle):
    """Device renders on two different caller streams, then a rebuild and a
    free without a host sync in between: the library orders them (the second
    stream waits for the first, the rebuild for both) -- images stay exact."""
    import torch
    tris = oracle.soup(40000, 6).reshape(-1, 9)
    w, h, spp = 200, 120, 1
    _, er = _oracle_frame(oracle, tris, w, h, spp)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    img = [torch.zeros(w * h, dtype=torch.int32, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()  # the zero fill (torch's stream) before the scene's stream writes
    s = R.Scene.from_soup(tris)
    s.build()
    cam = _cam(R, w, h)
    for i in range(4):
        st = (a, b)[i % 2]
        s.render_device(cam, w, h, spp, d_rgba=img[i].data_ptr(), stream=st.cuda_stream)
    s.build()
    s.close()  # waits for the caller-stream work before freeing
    torch.cuda.synchronize()
    for i in range(4):
        assert np.array_equal(img[i].cpu().numpy().view(np.uint8), er), i


def test_default_stream_handle_is_the_null_stream(R, oracle):
    """torch's default stream has handle 0, which the C ABI's NULL would read
    as the scene's own (non-blocking) stream: the Python layer passes an
    explicit 0 as hipStreamLegacy, so a render on
    torch.cuda.current_stream().cuda_stream runs after torch's zero fills of
    its buffers and before torch's reads of them -- no host sync in between
    (bench.py's N > 1 frame queues trace, RCCL gather and unpack this way)."""
    import torch
    tris = oracle.soup(40000, 8).reshape(-1, 9)
    w, h, spp = 640, 360, 2
    eh, er = _oracle_frame(oracle, tris, w, h, spp)
    cur = torch.cuda.current_stream()
    assert cur.cuda_stream == 0  # the case this test is about
    with R.Scene.from_soup(tris) as s:
        s.build()
        cam = _cam(R, w, h)
        for _ in range(3):
            img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
            hb = torch.zeros(w * h * spp * 4, dtype=torch.float32, device="cuda")
            s.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hb.data_ptr(), stream=cur.cuda_stream)
            img2, hb2 = img.clone(), hb.clone()  # torch's reads, queued behind the render
            img.fill_(0)
            hb.fill_(0)
            torch.cuda.synchronize()
            assert np.array_equal(img2.cpu().numpy().view(np.uint8), er)
            prim = hb2.view(-1, 4)[:, 3].view(torch.int32).cpu().numpy().view(np.uint32)
            assert np.array_equal(prim, eh["prim"])


def test_tiles_on_the_null_stream(R, oracle):
    """bench.py's N > 1 frame: rt_render_tiles_device on torch's default
    stream (handle 0 -> hipStreamLegacy), then an unpack on the same stream,
    no host sync between -- for three ranks of a P = 3 frame, three frames
    each (tile order, heavy-ray queue): the unpacked image == the oracle's."""
    import torch
    tris = oracle.soup(40000, 9).reshape(-1, 9)
    w, h, spp, P = 250, 138, 1, 3
    _, er = _oracle_frame(oracle, tris, w, h, spp)
    cur = torch.cuda.current_stream()
    tmax = max(R.tiles_for_rank(w, h, r, P) for r in range(P))
    with R.Scene.from_soup(tris) as s:
        s.build()
        cam = _cam(R, w, h)
        for _ in range(3):
            slabs = torch.zeros((P, tmax * 256), dtype=torch.int32, device="cuda")
            hits = torch.zeros((P, tmax * 256 * spp * 4), dtype=torch.float32, device="cuda")
            for r in range(P):
                s.render_tiles_device(cam, w, h, spp, r, P, slabs[r].data_ptr(), hits[r].data_ptr(),
                                      stream=cur.cuda_stream)
            img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
            R.unpack_tiles_device(slabs.data_ptr(), tmax, w, h, P, img.data_ptr(), 0, cur.cuda_stream)
            got = img.clone()
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint8), er)
