"""Multi-GPU image-tile sharding: one process per GPU.

Tile t (16x16 pixels, row-major over the image) belongs to rank t mod P; the
BVH is replicated (every rank builds it -- the build is deterministic, so the
replicas are bit-identical).  Each rank traces its tiles into a packed slab
[tile][256 px] on its GPU (rt_render_tiles_device); the single exchange is a
gather of the equal-size slabs to rank 0 over torch.distributed -- backend
'nccl', which is RCCL over xGMI on MI355X -- followed by rt_unpack_tiles_device.
The gather helper is backend-agnostic so the CPU tests drive it with 'gloo'.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

TILE = 16


def tiles_total(w: int, h: int) -> int:
    return ((w + TILE - 1) // TILE) * ((h + TILE - 1) // TILE)


def tiles_of_rank(w: int, h: int, rank: int, nranks: int) -> int:
    nt = tiles_total(w, h)
    return 0 if rank >= nt else (nt - rank + nranks - 1) // nranks


def slab_tiles(w: int, h: int, nranks: int) -> int:
    """Tiles per (padded, equal-size) slab: the largest rank share."""
    return max(1, max(tiles_of_rank(w, h, r, nranks) for r in range(nranks)))


def rays_of_rank(w: int, h: int, spp: int, rank: int, nranks: int) -> int:
    tx = (w + TILE - 1) // TILE
    n = 0
    for t in range(rank, tiles_total(w, h), nranks):
        x0, y0 = (t % tx) * TILE, (t // tx) * TILE
        n += min(TILE, w - x0) * min(TILE, h - y0)
    return n * spp


class _DeviceBytes:
    """A library-owned device buffer seen by torch without a copy
    (__cuda_array_interface__; the HIP device pointer on ROCm)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2}


def bvh_tensors(scene, device) -> list:
    """The scene's device BVH sections (rt_bvh_device_sections) as uint8
    tensors aliasing the library's buffers."""
    return [torch.as_tensor(_DeviceBytes(p, n), device=device) for p, n in scene.device_sections() if n]


def broadcast_bvh(scene, device, src: int = 0) -> int:
    """SURVEY.md §8(e)'s alternative to the replicated build: rank `src` has
    built; every other rank has called scene.prepare().  Broadcasts the BVH
    sections in place (RCCL over xGMI with the 'nccl' backend) and marks the
    receivers built.  Returns the bytes moved per receiver."""
    ts = bvh_tensors(scene, device)
    for t in ts:
        dist.broadcast(t, src=src)
    if dist.get_rank() != src:
        torch.cuda.synchronize(device)
        scene.mark_built()
    return sum(t.numel() for t in ts)


def gather_slabs(slab: torch.Tensor, rank: int, world: int, gather_list=None, out: torch.Tensor | None = None):
    """Gather every rank's slab (same shape) to rank 0.  On rank 0 returns the
    concatenation [rank][slab] (written into `out` when given)."""
    if world == 1:
        return slab
    if rank == 0:
        if out is not None and gather_list is None:
            # receive straight into out's [rank] rows (views): no concatenation copy
            gather_list = list(out.view(world, -1).unbind(0))
        if gather_list is None:
            gather_list = [torch.empty_like(slab) for _ in range(world)]
        dist.gather(slab, gather_list, dst=0)
        if out is None:
            return torch.cat(gather_list)
        if gather_list[0].data_ptr() != out.data_ptr():
            torch.cat(gather_list, out=out)
        return out
    dist.gather(slab, None, dst=0)
    return None
