"""Host-side Python mirror of the librtamd C-ABI (include/gpu_raytracer_amd.h).

Thin numpy-facing wrappers: no compute happens in Python, every call goes to
the gfx950 kernels through ctypes, and errors surface as RtError carrying the
library's status and message.  Names follow the ABI:
scene ingest -> rt_bvh_build -> rt_render -> framebuffer/hit dumps, plus the
per-stage entry points the parity tests drive.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import RT_BACKEND_HIP, SENTINEL, call, lib, rt_build_times, rt_camera

NODE_DTYPE = np.dtype([("lo", "<f4", (3,)), ("hi", "<f4", (3,)), ("a", "<u4"), ("esc", "<u4")])
HIT_DTYPE = np.dtype([("t", "<f4"), ("u", "<f4"), ("v", "<f4"), ("prim", "<u4")])
TILE = 16


def _p(a: np.ndarray) -> C.c_void_p:
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return C.c_void_p(a.ctypes.data)


def camera_look_at(eye, at, up, vfov_deg: float, w: int, h: int) -> rt_camera:
    """SURVEY.md §9.7 ray frame (double on the host, rounded to float)."""
    cam = rt_camera()
    e, a, u = (np.ascontiguousarray(x, dtype=np.float64) for x in (eye, at, up))
    call("rt_camera_look_at", _p(e), _p(a), _p(u), float(vfov_deg), int(w), int(h), C.byref(cam))
    return cam


def camera_array(cam: rt_camera) -> np.ndarray:
    return np.array([list(cam.eye), list(cam.w00), list(cam.du), list(cam.dv)], dtype=np.float32)


# hipStreamLegacy: the HIP null stream.  Stream handles are ints as torch
# gives them (torch.cuda.current_stream().cuda_stream), and torch's default
# stream IS the null stream, handle 0 -- which the C ABI's NULL would read as
# "the scene's own stream", unordered with the caller's work.  So None selects
# the scene's stream and an explicit 0 the null stream.
HIP_STREAM_LEGACY = 1


def _stream(stream):
    if stream is None:
        return None
    return C.c_void_p(int(stream) if int(stream) != 0 else HIP_STREAM_LEGACY)


@dataclass
class BuildTimes:
    bounds: float
    morton: float
    sort: float
    topology: float
    refit: float
    wide: float
    total: float
    sort_kind: int = 2   # 0 LSB, 1 MSB, 2 tile-bucketed gather (the sort later builds use)
    fused_k01: int = 0   # the last build ran K0 + K1 as one launch
    fused_fallback: int = 0  # its fused barrier gave up and the build was redone with two launches
    lsb_redo: int = 0    # a gather bucket overflowed and the build was redone with the LSB sort


class Scene:
    """Opaque rt_scene handle: host soup + device-resident BVH on one GPU."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle

    # -- ingest
    @classmethod
    def from_soup(cls, tris: np.ndarray) -> "Scene":
        t = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        h = C.c_void_p()
        call("rt_scene_from_soup", _p(t) if len(t) else None, len(t), C.byref(h))
        return cls(h)

    @classmethod
    def load_obj(cls, path: str) -> "Scene":
        h = C.c_void_p()
        call("rt_scene_load_obj", path.encode(), C.byref(h))
        return cls(h)

    @classmethod
    def load_soup(cls, path: str) -> "Scene":
        """RTSOUP1 binary triangle soup."""
        h = C.c_void_p()
        call("rt_scene_load_soup", path.encode(), C.byref(h))
        return cls(h)

    def save_soup(self, path: str) -> None:
        call("rt_scene_save_soup", self._h, path.encode())

    @classmethod
    def generate_soup(cls, n: int, seed: int = 1) -> "Scene":
        h = C.c_void_p()
        call("rt_scene_generate_soup", int(n), int(seed), C.byref(h))
        return cls(h)

    def close(self) -> None:
        if self._h:
            lib().rt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def num_tris(self) -> int:
        n = C.c_uint32()
        call("rt_scene_num_tris", self._h, C.byref(n))
        return n.value

    def tris(self) -> np.ndarray:
        out = np.empty((self.num_tris, 9), np.float32)
        if len(out):
            call("rt_scene_get_tris", self._h, _p(out))
        return out

    def set_device(self, device: int) -> None:
        call("rt_scene_set_device", self._h, int(device))

    # -- build
    def build(self, device_mask: int = 0, backend: int = RT_BACKEND_HIP) -> float:
        """rt_bvh_build: replicas on the devices of device_mask (0 = the
        scene's device); returns the device time of the (longest) build."""
        ms = C.c_double()
        call("rt_bvh_build", self._h, int(backend), int(device_mask), C.byref(ms))
        return ms.value

    def replicas(self) -> list:
        """Devices holding a built BVH replica, primary first."""
        cnt = C.c_uint32()
        call("rt_bvh_replicas", self._h, 0, None, C.byref(cnt))
        devs = (C.c_int * max(cnt.value, 1))()
        call("rt_bvh_replicas", self._h, cnt.value, devs, C.byref(cnt))
        return [int(devs[i]) for i in range(cnt.value)]

    def save_bvh(self, path: str) -> None:
        """RTBVH1 cache of the built BVH."""
        call("rt_bvh_save", self._h, path.encode())

    def load_bvh(self, path: str) -> None:
        """Restore a cached BVH built for these same triangles (instead of build())."""
        call("rt_bvh_load", self._h, path.encode())

    def build_times(self) -> BuildTimes:
        t = rt_build_times()
        call("rt_bvh_build_times_sized", self._h, C.byref(t), C.sizeof(t))
        return BuildTimes(t.bounds, t.morton, t.sort, t.topology, t.refit, t.wide, t.total, t.sort_kind, t.fused_k01,
                          t.fused_fallback, t.lsb_redo)

    @property
    def wide_arity(self) -> int:
        """Arity of the built wide records: 4 (K7w) or 8 (K7w8)."""
        a = C.c_uint32()
        call("rt_bvh_wide_arity", self._h, C.byref(a))
        return a.value

    def read_wide(self) -> np.ndarray:
        """Wide records as uint32[(n-1), 16] (4-ary K7w) or uint32[(n-1), 24]
        (8-ary K7w8); layouts: csrc/rt_device.h."""
        n = self.num_tris
        words = 24 if self.wide_arity == 8 else 16
        rec = np.zeros((max(n - 1, 1), words), np.uint32)
        call("rt_bvh_read_wide", self._h, _p(rec))
        return rec[: max(n - 1, 0)]

    def read_bvh(self) -> dict:
        n = self.num_tris
        tot = max(2 * n - 1, 0)
        nodes = np.zeros(max(tot, 1), NODE_DTYPE)
        keys = np.zeros(max(n, 1), np.uint32)
        vals = np.zeros(max(n, 1), np.uint32)
        parent = np.zeros(max(tot, 1), np.uint32)
        bounds = np.zeros(9, np.float32)
        call("rt_bvh_read", self._h, _p(nodes), _p(keys), _p(vals), _p(parent), _p(bounds))
        return dict(nodes=nodes[:tot], keys=keys[:n], vals=vals[:n], parent=parent[:tot],
                    lo=bounds[0:3].copy(), hi=bounds[3:6].copy(), inv=bounds[6:9].copy())

    # -- render
    def render(self, cam: rt_camera, w: int, h: int, spp: int = 1, hits: bool = True, rgba: bool = True,
               ngpus: int = 1):
        """Returns (hits[h*w*spp] HIT_DTYPE or None, rgba[h*w*4] uint8 or None, frame_ms).
        ngpus > 1: the in-library multi-GPU render (replicas + RCCL gather)."""
        hb = np.zeros(w * h * spp, HIT_DTYPE) if hits else None
        rb = np.zeros(w * h * 4, np.uint8) if rgba else None
        ms = C.c_double()
        call("rt_render_timed", self._h, C.byref(cam), w, h, spp, int(ngpus), _p(hb) if hits else None,
             _p(rb) if rgba else None, C.byref(ms))
        return hb, rb, ms.value

    def render_shadow(self, cam: rt_camera, w: int, h: int, spp: int, light, ambient: float,
                      hits: bool = True):
        """Shadow mode: (primary hits or None, shaded rgba, ms)."""
        hb = np.zeros(w * h * spp, HIT_DTYPE) if hits else None
        rb = np.zeros(w * h * 4, np.uint8)
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        ms = C.c_double()
        call("rt_render_shadow", self._h, C.byref(cam), _p(L), float(ambient), w, h, spp,
             _p(hb) if hits else None, _p(rb), C.byref(ms))
        return hb, rb, ms.value

    def render_shadow_device(self, cam, w, h, spp, light, ambient, d_rgba: int = 0, d_hits: int = 0,
                             stream: int | None = None, timed: bool = False):
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        ms = C.c_double()
        call("rt_render_shadow_device", self._h, C.byref(cam), _p(L), float(ambient), w, h, spp,
             C.c_void_p(d_hits) if d_hits else None, C.c_void_p(d_rgba) if d_rgba else None,
             _stream(stream), C.byref(ms) if timed else None)
        return ms.value if timed else None

    def render_shadow_work(self, cam, w, h, spp, light, ambient) -> np.ndarray:
        c = np.zeros(2, np.uint64)
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        call("rt_render_shadow_work", self._h, C.byref(cam), _p(L), float(ambient), w, h, spp, _p(c))
        return c

    def render_path(self, cam: rt_camera, w: int, h: int, spp: int, light, sky: float, max_depth: int,
                    hits: bool = True):
        """Path mode: (primary hits or None, path-traced rgba, ms)."""
        hb = np.zeros(w * h * spp, HIT_DTYPE) if hits else None
        rb = np.zeros(w * h * 4, np.uint8)
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        ms = C.c_double()
        call("rt_render_path", self._h, C.byref(cam), _p(L), float(sky), int(max_depth), w, h, spp,
             _p(hb) if hits else None, _p(rb), C.byref(ms))
        return hb, rb, ms.value

    def render_path_device(self, cam, w, h, spp, light, sky, max_depth, d_rgba: int = 0, d_hits: int = 0,
                           stream: int | None = None, timed: bool = False):
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        ms = C.c_double()
        call("rt_render_path_device", self._h, C.byref(cam), _p(L), float(sky), int(max_depth), w, h, spp,
             C.c_void_p(d_hits) if d_hits else None, C.c_void_p(d_rgba) if d_rgba else None,
             _stream(stream), C.byref(ms) if timed else None)
        return ms.value if timed else None

    def render_path_work(self, cam, w, h, spp, light, sky, max_depth) -> np.ndarray:
        """Path-mode kernel work: node records, tri records, rays traced."""
        c = np.zeros(3, np.uint64)
        L = np.ascontiguousarray(light, np.float32).reshape(3)
        call("rt_render_path_work", self._h, C.byref(cam), _p(L), float(sky), int(max_depth), w, h, spp, _p(c))
        return c

    def prepare(self):
        """Upload + allocate without building (a receiver of a broadcast BVH)."""
        call("rt_bvh_prepare", self._h)

    def device_sections(self):
        """[(device pointer, bytes)] of the BVH buffers (RTBVH1 sections)."""
        cnt = C.c_uint32()
        call("rt_bvh_device_sections", self._h, 0, None, None, C.byref(cnt))
        ptrs = (C.c_void_p * cnt.value)()
        sizes = (C.c_uint64 * cnt.value)()
        call("rt_bvh_device_sections", self._h, cnt.value, ptrs, sizes, C.byref(cnt))
        return [(int(ptrs[i] or 0), int(sizes[i])) for i in range(cnt.value)]

    def mark_built(self):
        call("rt_bvh_mark_built", self._h)

    # ---- distributed build phases (rt_dbuild_*; driven by dist.distributed_build)
    def dbuild_bounds(self, rank: int, nranks: int) -> np.ndarray:
        box = np.zeros(6, np.float32)
        call("rt_dbuild_bounds", self._h, rank, nranks, _p(box))
        return box

    def dbuild_keys(self, rank: int, nranks: int, boxes: np.ndarray) -> np.ndarray:
        boxes = np.ascontiguousarray(boxes, np.float32).reshape(nranks, 6)
        hist = np.zeros(1024, np.uint32)
        call("rt_dbuild_keys", self._h, rank, nranks, _p(boxes), _p(hist))
        return hist

    def dbuild_sort(self, count: int) -> None:
        call("rt_dbuild_sort", self._h, int(count))

    def dbuild_subtrees(self, rank: int, nranks: int) -> int:
        nc = C.c_uint32()
        call("rt_dbuild_subtrees", self._h, rank, nranks, C.byref(nc))
        return nc.value

    def dbuild_merge(self, ncross_total: int) -> None:
        call("rt_dbuild_merge", self._h, int(ncross_total))

    def dbuild_buffer(self, which: int):
        """(device pointer, bytes) of an exchange buffer (RT_DB_*)."""
        p, b = C.c_void_p(), C.c_uint64()
        call("rt_dbuild_buffer", self._h, int(which), C.byref(p), C.byref(b))
        return int(p.value or 0), int(b.value)

    def render_counters(self, cam: rt_camera, w: int, h: int, spp: int = 1) -> np.ndarray:
        """§9.7 binary-traversal counters (the oracle's): nodes fetched, tris tested."""
        c = np.zeros(2, np.uint64)
        call("rt_render_counters", self._h, C.byref(cam), w, h, spp, _p(c))
        return c

    def render_work(self, cam: rt_camera, w: int, h: int, spp: int = 1) -> np.ndarray:
        """The configured trace kernel's own fetches: node records, triangle records."""
        c = np.zeros(2, np.uint64)
        call("rt_render_work", self._h, C.byref(cam), w, h, spp, _p(c))
        return c

    def render_device(self, cam, w, h, spp, d_rgba: int = 0, d_hits: int = 0, stream: int | None = None,
                      timed: bool = False):
        """Full-image render into device buffers (device pointers as ints) on
        `stream` (None: the scene's own stream; an int handle, 0 = the null
        stream, e.g. torch.cuda.current_stream().cuda_stream)."""
        ms = C.c_double()
        call("rt_render_device", self._h, C.byref(cam), w, h, spp, C.c_void_p(d_hits) if d_hits else None,
             C.c_void_p(d_rgba) if d_rgba else None, _stream(stream),
             C.byref(ms) if timed else None)
        return ms.value if timed else None

    def render_tiles_counters(self, cam, w, h, spp, rank, nranks) -> np.ndarray:
        c = np.zeros(2, np.uint64)
        call("rt_render_tiles_counters", self._h, C.byref(cam), w, h, spp, rank, nranks, _p(c))
        return c

    def render_tiles_work(self, cam, w, h, spp, rank, nranks) -> np.ndarray:
        """The trace kernel's own fetches (records, triangle records) for one rank's tiles."""
        c = np.zeros(2, np.uint64)
        call("rt_render_tiles_work", self._h, C.byref(cam), w, h, spp, rank, nranks, _p(c))
        return c

    def step_map(self, w, h, spp=1, rank=0, nranks=1) -> np.ndarray:
        """Per-pixel wide-traversal step counts of the previous full frame of
        this shape, tile-slot-major (rt_render_step_map)."""
        nb = tiles_for_rank(w, h, rank, nranks)
        out = np.zeros(nb * 256, np.uint16)
        call("rt_render_step_map", self._h, w, h, spp, rank, nranks, _p(out), out.size)
        return out

    def render_tiles_device(self, cam, w, h, spp, rank, nranks, d_rgba: int, d_hits: int = 0,
                            stream: int | None = None, timed: bool = False):
        ms = C.c_double()
        call("rt_render_tiles_device", self._h, C.byref(cam), w, h, spp, rank, nranks, C.c_void_p(d_rgba),
             C.c_void_p(d_hits) if d_hits else None, _stream(stream),
             C.byref(ms) if timed else None)
        return ms.value if timed else None

    def stream(self) -> int:
        s = C.c_void_p()
        call("rt_scene_stream", self._h, C.byref(s))
        return s.value or 0

    def sync(self) -> None:
        call("rt_scene_sync", self._h)


def dbuild_shares(n: int, rank: int, nranks: int) -> tuple:
    """(tri_lo, tri_hi, block_lo, block_hi, leaf_lo, leaf_hi) of one rank
    (rt_dbuild_shares)."""
    out = np.zeros(6, np.uint32)
    call("rt_dbuild_shares", int(n), int(rank), int(nranks), _p(out))
    return tuple(int(x) for x in out)


def tiles_for_rank(w: int, h: int, rank: int, nranks: int) -> int:
    return int(lib().rt_tiles_for_rank(w, h, rank, nranks))


def unpack_tiles_device(d_slabs: int, tiles_per_slab: int, w: int, h: int, nranks: int, d_rgba: int,
                        device: int = 0, stream: int = 0) -> None:
    call("rt_unpack_tiles_device", C.c_void_p(d_slabs), tiles_per_slab, w, h, nranks, C.c_void_p(d_rgba),
         int(device), C.c_void_p(stream) if stream else None)


def dump_ppm(rgba: np.ndarray, w: int, h: int, path: str) -> None:
    call("rt_framebuffer_dump_ppm", _p(np.ascontiguousarray(rgba, np.uint8)), w, h, path.encode())


def dump_hits(hits: np.ndarray, path: str) -> None:
    h = np.ascontiguousarray(hits, HIT_DTYPE)
    call("rt_hits_dump", _p(h) if len(h) else None, len(h), path.encode())


def config_set(key: str, value: int) -> None:
    """Process-wide tuning knob (see rt_config_set in the header)."""
    call("rt_config_set", key.encode(), int(value))


def device_count() -> int:
    return int(lib().rt_device_count())


# -- per-stage entry points (parity tests) -------------------------------
def stage_bounds(tris: np.ndarray, device: int = 0):
    t = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    out = np.zeros(9, np.float32)
    call("rt_stage_bounds", device, _p(t) if len(t) else None, len(t), _p(out))
    return out[0:3].copy(), out[3:6].copy(), out[6:9].copy()


def stage_morton(tris, lo, inv, device: int = 0):
    t = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    n = len(t)
    k = np.zeros(max(n, 1), np.uint32)
    v = np.zeros(max(n, 1), np.uint32)
    call("rt_stage_morton", device, _p(t) if n else None, n, _p(np.ascontiguousarray(lo, np.float32)),
         _p(np.ascontiguousarray(inv, np.float32)), _p(k), _p(v))
    return k[:n], v[:n]


def stage_sort(keys, vals, device: int = 0):
    k = np.array(keys, np.uint32, copy=True)
    v = np.array(vals, np.uint32, copy=True)
    call("rt_stage_sort", device, _p(k) if len(k) else None, _p(v) if len(v) else None, len(k))
    return k, v


def stage_topology(sorted_keys, device: int = 0):
    k = np.ascontiguousarray(sorted_keys, np.uint32)
    n = len(k)
    topo = np.zeros((max(n - 1, 1), 4), np.uint32)
    parent = np.zeros(max(2 * n - 1, 1), np.uint32)
    lesc = np.zeros(max(n, 1), np.uint32)
    call("rt_stage_topology", device, _p(k) if n else None, n, _p(topo), _p(parent), _p(lesc))
    return topo[: max(n - 1, 0)], parent[: max(2 * n - 1, 0)], lesc[:n]


def stage_refit(sorted_keys, sorted_vals, tris, device: int = 0) -> np.ndarray:
    """K5 + K6 (+ K7w) over sorted keys/vals: the (2n-1) node records."""
    k = np.ascontiguousarray(sorted_keys, np.uint32)
    v = np.ascontiguousarray(sorted_vals, np.uint32)
    t = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    n = len(k)
    if len(v) != n or len(t) != n:
        raise ValueError("keys, vals and tris must have the same length")
    nodes = np.zeros(max(2 * n - 1, 1), NODE_DTYPE)
    call("rt_stage_refit", device, _p(k) if n else None, _p(v) if n else None, _p(t) if n else None, n, _p(nodes))
    return nodes[: max(2 * n - 1, 0)]


def stage_trace(nodes, tris, cam: rt_camera, w, h, spp=1, device: int = 0):
    t = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    nd = np.ascontiguousarray(nodes, NODE_DTYPE)
    n = len(t)
    hits = np.zeros(w * h * spp, HIT_DTYPE)
    rgba = np.zeros(w * h * 4, np.uint8)
    cnt = np.zeros(2, np.uint64)
    call("rt_stage_trace", device, _p(nd) if n else None, n, _p(t) if n else None, C.byref(cam), w, h, spp,
         _p(hits), _p(rgba), _p(cnt))
    return hits, rgba, cnt


def stage_intersect(o, d, tri, t_best, device: int = 0):
    o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
    tri = np.ascontiguousarray(tri, np.float32).reshape(-1, 9)
    tb = np.ascontiguousarray(t_best, np.float32).reshape(-1)
    n = len(o)
    hit = np.zeros(max(n, 1), np.uint32)
    tuv = np.zeros((max(n, 1), 3), np.float32)
    call("rt_stage_intersect", device, n, _p(o), _p(d), _p(tri), _p(tb), _p(hit), _p(tuv))
    return hit[:n].astype(bool), tuv[:n]


def stage_minmax(a, b, device: int = 0):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    out = np.zeros((max(len(a), 1), 2), np.float32)
    call("rt_stage_minmax", device, len(a), _p(a), _p(b), _p(out))
    return out[: len(a), 0].copy(), out[: len(a), 1].copy()


__all__ = ["Scene", "config_set", "camera_look_at", "camera_array", "tiles_for_rank", "unpack_tiles_device", "dump_ppm",
           "dump_hits", "device_count", "stage_bounds", "stage_morton", "stage_sort", "stage_topology",
           "stage_refit", "stage_trace", "stage_intersect", "stage_minmax", "NODE_DTYPE", "HIT_DTYPE", "SENTINEL"]
