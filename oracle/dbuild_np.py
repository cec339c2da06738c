"""Numpy restatement of the distributed-build phases (rt_dbuild_*,
include/gpu_raytracer_amd.h; DESIGN.md "Distributed build").

TEST INFRASTRUCTURE ONLY (same rules as oracle/rt_oracle.c): the stage
backend that lets tests/test_distributed.py run gpu_raytracer_amd.dist's
distributed_build driver -- the partition, the all-to-all, the share gathers
and the merge -- on CPU ranks over gloo, and compare the BVH every rank ends
with against the single-process oracle build.  Each phase restates what the
device phase computes on the rank's share:
  bounds   -- centroid box of the rank's triangle slice (§9.2, fmin/fmax);
  keys     -- §9.3 Morton codes of the slice against the global box, the
              slice sorted by (key, index), its top-10-bit bucket histogram;
  sort     -- the received (key, index) pairs sorted stably (§9.4);
  subtrees -- for the rank's 256-leaf refit blocks: leaf nodes and leaf
              triangle records, the topology of the internal nodes there
              (§9.5, §9.6), boxes of the nodes whose range lies inside one
              block, the per-block prefix/suffix/total boxes and the list of
              nodes whose range crosses blocks;
  merge    -- every crossing node's box = suffix(l) U middle block totals U
              prefix(r) (exact min/max, so equal to §9.6's post-order refit).
Wide (K7w) records are not restated here (the GPU tests check them); the
WIDE buffer stays zero.  Buffers are numpy arrays seen by torch without a
copy (int32 views), like LibStages' device buffers."""
from __future__ import annotations

import numpy as np
import torch

from gpu_raytracer_amd import _lib as L
from gpu_raytracer_amd.dist import dbuild_shares_of
from oracle import oracle as O
from oracle import oracle_np as N

T = 256  # leaves per refit block (kRefitT)


def _union(lo, hi):
    """exact box of a set of boxes (rows).  np.fmin/np.fmax ignore NaN like
    §9.1's min/max; the soups these tests build have no signed zeros, where
    the two could differ."""
    return np.fmin.reduce(lo, axis=0).astype(np.float32), np.fmax.reduce(hi, axis=0).astype(np.float32)


class NumpyStages:
    def __init__(self, tris: np.ndarray):
        self.tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
        n = self.n = self.tris.shape[0]
        ni = max(n - 1, 0)
        m = -(-n // T)
        self.m = m
        self._b = {
            L.RT_DB_SEND_KEYS: np.zeros(n, np.uint32), L.RT_DB_SEND_VALS: np.zeros(n, np.uint32),
            L.RT_DB_RECV_KEYS: np.zeros(n, np.uint32), L.RT_DB_RECV_VALS: np.zeros(n, np.uint32),
            L.RT_DB_KEYS: np.zeros(n, np.uint32), L.RT_DB_VALS: np.zeros(n, np.uint32),
            L.RT_DB_NODES: np.zeros(max(2 * n - 1, 0), O.NODE_DTYPE), L.RT_DB_TRI_S: np.zeros((n, 12), np.float32),
            L.RT_DB_WIDE: np.zeros((ni, 16), np.uint32), L.RT_DB_TOPO: np.zeros((ni, 4), np.uint32),
            L.RT_DB_PRE: np.zeros((n, 6), np.float32), L.RT_DB_SUF: np.zeros((n, 6), np.float32),
            L.RT_DB_TOTALS: np.zeros((m, 6), np.float32),
            L.RT_DB_CROSS: np.zeros(max(n, 1), np.uint32), L.RT_DB_CROSS_ALL: np.zeros(max(n, 1), np.uint32),
        }
        self.bmin, self.bmax = N.tri_bounds(self.tris)

    def buf(self, which) -> torch.Tensor:
        return torch.from_numpy(self._b[which].view(np.uint8).reshape(-1)).view(torch.int32)

    def arr(self, which):
        return self._b[which]

    # 1.
    def bounds(self, rank, P):
        a, b = dbuild_shares_of(self.n, rank, P)[:2]
        c = (self.bmin[a:b] + self.bmax[a:b]) * np.float32(0.5)
        lo, hi = _union(c, c) if b > a else (np.full(3, np.inf, np.float32), np.full(3, -np.inf, np.float32))
        return np.concatenate([lo, hi]).astype(np.float32)

    # 2.
    def keys(self, rank, P, boxes):
        boxes = np.asarray(boxes, np.float32).reshape(P, 6)
        lo, _ = _union(boxes[:, :3], boxes[:, :3])
        _, hi = _union(boxes[:, 3:], boxes[:, 3:])
        inv = np.where(hi > lo, np.float32(1) / np.where(hi > lo, hi - lo, np.float32(1)), np.float32(0))
        inv = inv.astype(np.float32)
        a, b = dbuild_shares_of(self.n, rank, P)[:2]
        k, _ = O.morton(self.tris[a:b], lo, inv)
        v = np.arange(a, b, dtype=np.uint32)
        o = np.argsort(k, kind="stable")
        self._b[L.RT_DB_SEND_KEYS][: b - a] = k[o]
        self._b[L.RT_DB_SEND_VALS][: b - a] = v[o]
        return np.bincount(k >> 20, minlength=1024).astype(np.uint32)

    # 3.
    def sort(self, count):
        k = self._b[L.RT_DB_RECV_KEYS][:count].copy()
        v = self._b[L.RT_DB_RECV_VALS][:count].copy()
        o = np.argsort(k, kind="stable")
        self._b[L.RT_DB_RECV_KEYS][:count] = k[o]
        self._b[L.RT_DB_RECV_VALS][:count] = v[o]

    # 4.
    def subtrees(self, rank, P):
        n = self.n
        keys, vals = self._b[L.RT_DB_KEYS], self._b[L.RT_DB_VALS]
        _, _, b0, b1, k0, k1 = dbuild_shares_of(n, rank, P)
        nodes, tri_s = self._b[L.RT_DB_NODES], self._b[L.RT_DB_TRI_S]
        pre, suf, tot = self._b[L.RT_DB_PRE], self._b[L.RT_DB_SUF], self._b[L.RT_DB_TOTALS]
        topo = self._b[L.RT_DB_TOPO]
        L0 = n - 1
        left, right, rlo, rhi, parent = O.karras(keys) if n > 1 else ([], [], [], [], np.zeros(1, np.uint32))
        esc = O.escape(n, left, right, parent) if n > 1 else np.array([0xFFFFFFFF], np.uint32)
        lmin, lmax = self.bmin[vals[k0:k1]], self.bmax[vals[k0:k1]]
        # leaf-ordered triangle records {v0, v1, v2, prim, leaf escape, 0}: the
        # device writes no leaf nodes (leaf_nodes() derives them)
        tri_s[k0:k1, :9] = self.tris[vals[k0:k1]]
        tri_s[k0:k1, 9] = vals[k0:k1].view(np.float32)
        tri_s[k0:k1, 10] = esc[L0 + k0:L0 + k1].view(np.float32)
        cross = []
        for blk in range(b0, b1):
            B0, B1 = blk * T, min(blk * T + T, n)
            bl, bh = lmin[B0 - k0:B1 - k0], lmax[B0 - k0:B1 - k0]
            # every prefix / suffix inside the block
            pre[B0:B1, :3] = np.fmin.accumulate(bl, axis=0)
            pre[B0:B1, 3:] = np.fmax.accumulate(bh, axis=0)
            suf[B0:B1, :3] = np.fmin.accumulate(bl[::-1], axis=0)[::-1]
            suf[B0:B1, 3:] = np.fmax.accumulate(bh[::-1], axis=0)[::-1]
            tot[blk] = pre[B1 - 1]
            for i in range(B0, min(B1, n - 1)):  # internal nodes of the block
                l, r = int(rlo[i]), int(rhi[i])
                topo[i] = (left[i], esc[i], l, r)
                if l >= B0 and r < B1:
                    a, b = _union(bl[l - B0:r - B0 + 1], bh[l - B0:r - B0 + 1])
                    nodes[i] = (a, b, left[i], esc[i])
                else:
                    cross.append(i)
        c = self._b[L.RT_DB_CROSS]
        c[: len(cross)] = cross
        return len(cross)

    # 5.
    def merge(self, total):
        nodes, topo = self._b[L.RT_DB_NODES], self._b[L.RT_DB_TOPO]
        pre, suf, tot = self._b[L.RT_DB_PRE], self._b[L.RT_DB_SUF], self._b[L.RT_DB_TOTALS]
        for i in self._b[L.RT_DB_CROSS_ALL][:total]:
            l, r = int(topo[i, 2]), int(topo[i, 3])
            rows = [suf[l], pre[r]] + [tot[j] for j in range(l // T + 1, r // T)]
            rows = np.stack(rows)
            a, b = _union(rows[:, :3], rows[:, 3:])
            nodes[i] = (a, b, topo[i, 0], topo[i, 1])
