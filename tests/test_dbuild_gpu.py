"""Distributed BVH build (rt_dbuild_*, DESIGN.md
"Distributed build") on the MI355X: P ranks emulated on one GPU -- P threads
of one process, each with its own scene, exchanging by device copies
(dist.ThreadExchange), and P processes over gloo (dist.Exchange, bytes
staged through host memory).  Every rank's BVH must equal rt_bvh_build's bit
for bit: sorted keys and indices, every node (box, child, escape link), every
K7w wide record, the build bounds -- and a frame rendered from it must equal
the one rendered from the single build (hits and RGBA).  Up to 1M triangles
the distributed result is also compared with the CPU oracle's build
directly (keys, indices, parents, every node), and one case runs the RCCL
exchange (dist.Exchange under 'nccl', a 1-rank group: device tensors for
every collective, incl. the small host arrays)."""
import os
import socket
import threading

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


def _frame(R, s, w=160, h=96):
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    return s.render(cam, w, h, 2)


def _check_oracle(oracle, got, n, seed):
    """The distributed build against the oracle's (not only against the HIP
    single build): sorted keys/indices, parents and all 2n-1 nodes."""
    exp = oracle.build(oracle.soup(n, seed).reshape(-1, 9))
    b = got.read_bvh()
    assert np.array_equal(b["keys"], exp["keys"]), "keys vs oracle"
    assert np.array_equal(b["vals"], exp["vals"]), "vals vs oracle"
    assert np.array_equal(b["parent"], exp["parent"]), "parents vs oracle"
    assert np.array_equal(b["nodes"].view(np.uint32), exp["nodes"].view(np.uint32)), "nodes vs oracle"


def _check(R, ref, got, nref):
    a, b = ref.read_bvh(), got.read_bvh()
    for k in ("keys", "vals", "parent", "lo", "hi", "inv"):
        assert np.array_equal(np.asarray(a[k]).view(np.uint32), np.asarray(b[k]).view(np.uint32)), k
    assert np.array_equal(a["nodes"].view(np.uint32), b["nodes"].view(np.uint32)), "nodes"
    if nref >= 2:
        assert np.array_equal(ref.read_wide(), got.read_wide()), "wide records"
    ha, ia, _ = _frame(R, ref)
    hb, ib, _ = _frame(R, got)
    assert np.array_equal(ia, ib), "image"
    assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32)), "hits"


@pytest.mark.parametrize("P,n", [(2, 1_000_000), (3, 200_003), (8, 100_000), (8, 1_000_000), (2, 10_000_000),
                                 (4, 700), (3, 2)])
def test_dbuild_threads(R, oracle, P, n):
    import torch
    from gpu_raytracer_amd import dist as D
    seed = 41
    ref = R.Scene.generate_soup(n, seed)
    ref.build()
    scenes = [R.Scene.generate_soup(n, seed) for _ in range(P)]
    hub = D.ThreadExchange.Hub(P)
    errs, infos = [None] * P, [None] * P

    def run(r):
        try:
            torch.cuda.set_device(0)
            infos[r] = D.distributed_build(D.LibStages(scenes[r], "cuda:0"), D.ThreadExchange(hub, r))
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
            hub.bar.abort()
    th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th)
    for e in errs:
        if e is not None:
            raise e
    for r in (0, P - 1):
        _check(R, ref, scenes[r], n)
    if n <= 1_000_000:
        _check_oracle(oracle, scenes[P - 1], n, seed)
    if n > 512:
        assert infos[0]["crossing"] > 0
    for s in scenes + [ref]:
        s.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proc(rank, world, port, n, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        import gpu_raytracer_amd as R
        from gpu_raytracer_amd import dist as D
        s = R.Scene.generate_soup(n, 43)
        D.distributed_build(D.LibStages(s, "cuda:0"), D.Exchange(stage=True))
        ref = R.Scene.generate_soup(n, 43)
        ref.build()
        try:
            _check(R, ref, s, n)
            q.put((rank, "ok"))
        except AssertionError as e:
            q.put((rank, str(e)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_dbuild_gloo_processes(R):
    """P = 2 processes on the one GPU over gloo: the driver as bench.py runs it."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_proc, args=(r, 2, port, 300_000, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=10) for _ in range(2))
    assert res == {0: "ok", 1: "ok"}, res


def _proc_nccl(port, n, q):
    """One rank over 'nccl' (RCCL): every collective of the driver runs on
    device tensors, incl. gather_small's host arrays."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import gpu_raytracer_amd as R
        from gpu_raytracer_amd import dist as D
        from oracle import oracle as O
        s = R.Scene.generate_soup(n, 47)
        ex = D.Exchange()
        assert ex.device is not None and ex.device.type == "cuda"
        boxes = ex.gather_small(np.arange(6, dtype=np.float32))
        assert boxes.shape == (1, 6) and np.array_equal(boxes[0], np.arange(6, dtype=np.float32))
        D.distributed_build(D.LibStages(s, "cuda:0"), ex)
        try:
            _check_oracle(O, s, n, 47)
            q.put("ok")
        except AssertionError as e:
            q.put(str(e))
    finally:
        dist.destroy_process_group()


def test_dbuild_nccl_exchange(R):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_proc_nccl, args=(_free_port(), 50_000, q))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0, p.exitcode
    assert q.get(timeout=10) == "ok"
