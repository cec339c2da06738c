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


# ---------------------------------------------------------------- distributed build
# SURVEY.md §8(f) row 4 (DESIGN.md "Distributed build"): the BVH built by P
# ranks together instead of replicated, bit-identical to rt_bvh_build.  The
# phases are librtamd's rt_dbuild_* (LibStages); this module only moves the
# bytes between them.  The same driver runs over any stage backend with the
# LibStages interface -- the CPU tests plug in a numpy restatement of the
# phases (oracle/dbuild_np.py, test infrastructure) and run it with gloo.
import numpy as _np  # noqa: E402

from . import _lib as _L  # noqa: E402


def split_buckets(total_hist, nranks: int) -> _np.ndarray:
    """Rank d owns the top-10-bit key buckets [cut[d], cut[d + 1]): the
    cumulative count split as evenly as whole buckets allow (a Morton-prefix
    partition of the key space)."""
    c = _np.concatenate([[0], _np.cumsum(_np.asarray(total_hist, _np.int64))])
    n = int(c[-1])
    cut = [0]
    for d in range(1, nranks):
        b = int(_np.searchsorted(c, -(-n * d // nranks), side="left"))
        cut.append(min(max(b, cut[-1]), 1024))
    cut.append(1024)
    return _np.asarray(cut, _np.int64)


class LibStages:
    """librtamd's rt_dbuild_* phases on one rank's scene, with its exchange
    buffers seen by torch without a copy (int32 views on `device`)."""

    def __init__(self, scene, device):
        self.s, self.dev = scene, device
        self.n = scene.num_tris

    def bounds(self, rank, P):
        return self.s.dbuild_bounds(rank, P)

    def keys(self, rank, P, boxes):
        return self.s.dbuild_keys(rank, P, boxes)

    def sort(self, count):
        self.s.dbuild_sort(count)

    def subtrees(self, rank, P):
        return self.s.dbuild_subtrees(rank, P)

    def merge(self, total):
        self.s.dbuild_merge(total)

    def buf(self, which) -> torch.Tensor:
        p, nbytes = self.s.dbuild_buffer(which)
        if not nbytes:
            return torch.empty(0, dtype=torch.int32, device=self.dev)
        return torch.as_tensor(_DeviceBytes(p, nbytes), device=self.dev).view(torch.int32)

    def sync(self):
        torch.cuda.synchronize(self.dev)


class Exchange:
    """The collectives the distributed build needs, over the default process
    group.  stage=True (gloo with device buffers) moves the bytes through
    host memory.  Under 'nccl' (RCCL) every collective needs device tensors:
    the small host arrays (boxes, histograms, counts) go through `device`
    (default: the current GPU)."""

    def __init__(self, stage: bool = False, device=None):
        self.stage = stage
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.bytes_in = 0  # bytes this rank received
        self.device = None
        if dist.get_backend() == "nccl":
            self.device = torch.device(device) if device is not None else \
                torch.device("cuda", torch.cuda.current_device())

    def gather_small(self, arr) -> _np.ndarray:
        a = torch.from_numpy(_np.ascontiguousarray(arr).copy())
        if self.device is not None:
            a = a.to(self.device)
        out = [torch.empty_like(a) for _ in range(self.world)]
        dist.all_gather(out, a)
        return _np.stack([o.cpu().numpy() for o in out])

    def alltoallv(self, send: torch.Tensor, scounts, recv: torch.Tensor, rcounts):
        self.bytes_in += 4 * (sum(rcounts) - rcounts[self.rank])
        if self.stage:
            r = torch.empty(int(sum(rcounts)), dtype=send.dtype)
            dist.all_to_all_single(r, send.cpu(), list(map(int, rcounts)), list(map(int, scounts)))
            recv.copy_(r)
        else:
            dist.all_to_all_single(recv, send, list(map(int, rcounts)), list(map(int, scounts)))

    def share(self, buf: torch.Tensor, ranges):
        """Element range q of buf (written by rank q) broadcast from rank q
        to every rank, in place."""
        for q, (lo, hi) in enumerate(ranges):
            if hi <= lo:
                continue
            view = buf[lo:hi]
            if q != self.rank:
                self.bytes_in += 4 * (hi - lo)
            if self.stage:
                h = view.cpu()
                dist.broadcast(h, src=q)
                if q != self.rank:
                    view.copy_(h)
            else:
                dist.broadcast(view, src=q)


def distributed_build(st, ex: Exchange) -> dict:
    """SPMD distributed BVH build (include/gpu_raytracer_amd.h, rt_dbuild_*):
    every rank calls this with its own stage backend `st` over the same soup;
    afterwards every rank's scene holds the BVH rt_bvh_build would make.
    Returns this rank's counts (bytes received, crossing nodes)."""
    rank, P, n = ex.rank, ex.world, st.n
    sync = getattr(st, "sync", lambda: None)
    # 1. global centroid bounds from every rank's slice box
    boxes = ex.gather_small(st.bounds(rank, P))
    # 2. Morton codes; the Morton-prefix partition; all-to-all of (key, index)
    hist = st.keys(rank, P, boxes).astype(_np.int64)
    hists = ex.gather_small(hist)
    cut = split_buckets(hists.sum(0), P)
    scount = [int(hist[cut[d]:cut[d + 1]].sum()) for d in range(P)]
    rcount = [int(hists[q, cut[rank]:cut[rank + 1]].sum()) for q in range(P)]
    ns, nr = sum(scount), sum(rcount)
    sync()
    for a, b in ((_L.RT_DB_SEND_KEYS, _L.RT_DB_RECV_KEYS), (_L.RT_DB_SEND_VALS, _L.RT_DB_RECV_VALS)):
        ex.alltoallv(st.buf(a)[:ns], scount, st.buf(b)[:nr], rcount)
    sync()
    # 3. sort the received runs -> this rank's run of the global order; gather
    st.sort(nr)
    seg = [int(hists[:, cut[d]:cut[d + 1]].sum()) for d in range(P)]
    off = _np.concatenate([[0], _np.cumsum(seg)]).astype(_np.int64)
    ranges = [(int(off[q]), int(off[q + 1])) for q in range(P)]
    for src, dst in ((_L.RT_DB_RECV_KEYS, _L.RT_DB_KEYS), (_L.RT_DB_RECV_VALS, _L.RT_DB_VALS)):
        full = st.buf(dst)
        full[ranges[rank][0]:ranges[rank][1]].copy_(st.buf(src)[:nr])
        sync()
        ex.share(full, ranges)
    sync()
    # 4. this rank's refit blocks, then every section's shares
    nc = st.subtrees(rank, P)
    shares = [dbuild_shares_of(n, q, P) for q in range(P)]
    ni = max(n - 1, 0)
    # wide records: 16 words (4-ary) or 24 (8-ary, build.wide_arity)
    wwpe = len(st.buf(_L.RT_DB_WIDE)) // ni if ni else 16
    secs = [  # (buffer, int32 words per element, [(lo, hi) element range per rank])
        (_L.RT_DB_NODES, 8, [(s[4], min(s[5], ni)) for s in shares]),  # internal nodes (leaves live in tri_s)
        (_L.RT_DB_TRI_S, 12, [(s[4], s[5]) for s in shares]),
        (_L.RT_DB_WIDE, wwpe, [(s[4], min(s[5], ni)) for s in shares]),
        (_L.RT_DB_TOPO, 4, [(s[4], min(s[5], ni)) for s in shares]),
        (_L.RT_DB_PRE, 6, [(s[4], s[5]) for s in shares]),
        (_L.RT_DB_SUF, 6, [(s[4], s[5]) for s in shares]),
        (_L.RT_DB_TOTALS, 6, [(s[2], s[3]) for s in shares]),
    ]
    sync()
    for which, wpe, rg in secs:
        ex.share(st.buf(which), [(lo * wpe, hi * wpe) for lo, hi in rg])
    ncs = ex.gather_small(_np.array([nc], _np.int64))[:, 0]
    coff = _np.concatenate([[0], _np.cumsum(ncs)]).astype(_np.int64)
    allc = st.buf(_L.RT_DB_CROSS_ALL)
    allc[int(coff[rank]):int(coff[rank + 1])].copy_(st.buf(_L.RT_DB_CROSS)[:nc])
    sync()
    ex.share(allc, [(int(coff[q]), int(coff[q + 1])) for q in range(P)])
    sync()
    # 5. every crossing node
    st.merge(int(coff[-1]))
    return dict(bytes_in=ex.bytes_in, crossing=int(coff[-1]), cut=cut.tolist())


def dbuild_shares_of(n: int, rank: int, nranks: int) -> tuple:
    """rt_dbuild_shares (a host function: no device needed)."""
    from .scene import dbuild_shares
    return dbuild_shares(n, rank, nranks)


class ThreadExchange:
    """Exchange between P ranks that are threads of one process (one GPU
    standing in for P: the multi-rank emulation of tests/test_dbuild_gpu.py
    and tools/dbuild_emulate.py).  Bytes move by device copies; construct one
    shared `ThreadExchange.Hub(P)` and one ThreadExchange(hub, rank) per
    thread."""

    class Hub:
        def __init__(self, world: int):
            import threading
            self.world = world
            self.bar = threading.Barrier(world)
            self.slots = [None] * world

    def __init__(self, hub: "ThreadExchange.Hub", rank: int):
        self.hub, self.rank, self.world = hub, rank, hub.world
        self.bytes_in = 0

    def _post(self, x):
        self.hub.slots[self.rank] = x
        self.hub.bar.wait()
        got = list(self.hub.slots)
        return got

    def _done(self):
        torch.cuda.synchronize()
        self.hub.bar.wait()

    def gather_small(self, arr) -> _np.ndarray:
        got = self._post(_np.ascontiguousarray(arr).copy())
        self._done()
        return _np.stack(got)

    def alltoallv(self, send, scounts, recv, rcounts):
        got = self._post((send, list(map(int, scounts))))
        o = 0
        for q in range(self.world):
            sq, cq = got[q]
            start = sum(cq[:self.rank])
            n = cq[self.rank]
            recv[o:o + n].copy_(sq[start:start + n])
            if q != self.rank:
                self.bytes_in += 4 * n
            o += n
        self._done()

    def share(self, buf, ranges):
        got = self._post(buf)
        for q, (lo, hi) in enumerate(ranges):
            if q != self.rank and hi > lo:
                buf[lo:hi].copy_(got[q][lo:hi])
                self.bytes_in += 4 * (hi - lo)
        self._done()
