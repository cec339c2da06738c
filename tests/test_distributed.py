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
