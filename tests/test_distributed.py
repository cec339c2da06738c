"""N>1 path on CPU: world_size-2 (and 3) 'gloo' process groups run the same
tile partition + slab gather (gpu_raytracer_amd.dist) that bench.py drives
over RCCL; each rank's slab is the oracle render of its tiles, and rank 0's
unpacked image must equal the single-process oracle image bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, w, h, spp, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpu_raytracer_amd import dist as D
        from gpu_raytracer_amd.scenes import SOUP_VIEW as V
        from oracle import oracle as O, tiles_np
        tris = O.soup(n, 3)
        b = O.build(tris)
        cam = O.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
        hits, _ = O.trace(b["nodes"], tris, cam, w, h, spp, nthreads=1)
        full = O.shade(hits, w, h, spp).view(np.uint32)
        st = D.slab_tiles(w, h, world)
        slab = torch.from_numpy(tiles_np.pack(full, w, h, rank, world, st).view(np.int32))
        got = D.gather_slabs(slab, rank, world)
        if rank == 0:
            img = tiles_np.unpack(got.numpy().view(np.uint32), w, h, world, st)
            q.put(bool(np.array_equal(img, full)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, 70, 45), (3, 64, 48)])
def test_gloo_tile_gather(world, w, h):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 3000, w, h, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_partition_helpers():
    from gpu_raytracer_amd import dist as D
    for (w, h, P) in [(1920, 1080, 8), (3840, 2160, 8), (17, 33, 3)]:
        assert sum(D.tiles_of_rank(w, h, r, P) for r in range(P)) == D.tiles_total(w, h)
        assert sum(D.rays_of_rank(w, h, 2, r, P) for r in range(P)) == w * h * 2


def _dbuild_worker(rank, world, port, n, seed, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpu_raytracer_amd import dist as D
        from gpu_raytracer_amd import _lib as L
        from oracle import oracle as O
        from oracle.dbuild_np import NumpyStages
        tris = O.soup(n, seed).reshape(-1, 9)
        st = NumpyStages(tris)
        info = D.distributed_build(st, D.Exchange())
        exp = O.build(tris)
        # the device phases write internal nodes only; leaf L0 + k is derived
        # from triangle record k {v0, v1, v2, prim, esc} (k_leaf_nodes)
        got_nodes = st.arr(L.RT_DB_NODES).copy()
        ts = st.arr(L.RT_DB_TRI_S)
        lv, v = got_nodes[n - 1:], ts[:, :9].reshape(-1, 3, 3)
        lv["lo"] = np.fmin(np.fmin(v[:, 0], v[:, 1]), v[:, 2])
        lv["hi"] = np.fmax(np.fmax(v[:, 0], v[:, 1]), v[:, 2])
        lv["a"], lv["esc"] = ts[:, 9].view(np.uint32), ts[:, 10].view(np.uint32)
        ok = {
            "keys": np.array_equal(st.arr(L.RT_DB_KEYS), exp["keys"]),
            "vals": np.array_equal(st.arr(L.RT_DB_VALS), exp["vals"]),
            "nodes": np.array_equal(got_nodes.view(np.uint32), exp["nodes"].view(np.uint32)),
            "tri_s": np.array_equal(st.arr(L.RT_DB_TRI_S)[:, :9], tris[exp["vals"]])
            and np.array_equal(st.arr(L.RT_DB_TRI_S)[:, 9].view(np.uint32), exp["vals"]),
            "crossing": info["crossing"] > 0 or n <= 512,
            "exchanged": info["bytes_in"] > 0,
        }
        q.put((rank, ok))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,seed", [(2, 20000, 31), (3, 7001, 32), (2, 300, 33), (4, 5, 34)])
def test_gloo_distributed_build(world, n, seed):
    """the distributed-build driver (Morton-prefix
    partition, all-to-all of (key, index), per-rank refit blocks, share
    gathers, crossing-node merge) on world_size CPU ranks over gloo, with
    the numpy restatement of the device phases: every rank ends with the
    single-process oracle's BVH, bit for bit (sorted keys/indices, every
    node's box, child and escape link, the leaf triangle records)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dbuild_worker, args=(r, world, port, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=10) for _ in range(world))
    for r in range(world):
        assert all(res[r].values()), (r, res[r])


def test_split_buckets():
    from gpu_raytracer_amd import dist as D
    h = np.zeros(1024, np.int64)
    h[[3, 500, 501, 1000]] = [10, 5, 5, 10]
    for P in (1, 2, 3, 8):
        cut = D.split_buckets(h, P)
        assert cut[0] == 0 and cut[-1] == 1024 and np.all(np.diff(cut) >= 0)
        assert sum(h[cut[d]:cut[d + 1]].sum() for d in range(P)) == h.sum()
    assert list(D.split_buckets(np.ones(1024), 4)) == [0, 256, 512, 768, 1024]
    for n, P in ((1_000_000, 8), (10, 3), (1, 2), (513, 2)):
        sh = [D.dbuild_shares_of(n, r, P) for r in range(P)]
        assert sh[0][0] == 0 and sh[-1][1] == n and all(sh[r][1] == sh[r + 1][0] for r in range(P - 1))
        assert sh[0][4] == 0 and sh[-1][5] == n and all(sh[r][5] == sh[r + 1][4] for r in range(P - 1))
