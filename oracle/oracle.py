"""ctypes binding of the C oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py -- never by the product package
(gpu_raytracer_amd/).  Parity vs upstream SoslanGM/gpu_raytracer is UNPINNED
(the reference at /root/reference is a code-less stub); this
oracle restates SURVEY.md §9 and is pinned by the KATs of SURVEY.md §4/§9.8 and
by the independent numpy restatement in oracle/oracle_np.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
SENTINEL = 0xFFFFFFFF

NODE_DTYPE = np.dtype([("lo", "<f4", (3,)), ("hi", "<f4", (3,)), ("a", "<u4"), ("esc", "<u4")])
HIT_DTYPE = np.dtype([("t", "<f4"), ("u", "<f4"), ("v", "<f4"), ("prim", "<u4")])
assert NODE_DTYPE.itemsize == 32 and HIT_DTYPE.itemsize == 16


class Camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("w00", C.c_float * 3), ("du", C.c_float * 3), ("dv", C.c_float * 3)]

    def as_array(self) -> np.ndarray:
        return np.array([list(self.eye), list(self.w00), list(self.du), list(self.dv)], dtype=np.float32)


class Bounds(C.Structure):
    _fields_ = [("lo", C.c_float * 3), ("hi", C.c_float * 3), ("inv", C.c_float * 3)]


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def use_native_build() -> str:
    """Switch this process to the -march=native build of the same source
    (bench.py's timed CPU baseline; compiled on the host that runs it).
    Must be called before the first lib()."""
    global _LIB_PATH
    if _lib is not None:
        raise RuntimeError("oracle already loaded")
    subprocess.run(["make", "-s", "-C", _HERE, "native"], check=True)
    _LIB_PATH = os.path.join(_HERE, "build", "liboracle_native.so")
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build_oracle()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        u32, u64, f32, i32 = C.c_uint32, C.c_uint64, C.c_float, C.c_int
        L.orc_soup_generate.argtypes = [u32, u64, P]
        L.orc_camera_look_at.argtypes = [P, P, P, C.c_double, u32, u32, C.POINTER(Camera)]
        L.orc_centroid_bounds.argtypes = [P, u32, P, P, P]
        L.orc_expand10.argtypes = [u32]
        L.orc_expand10.restype = u32
        L.orc_morton3.argtypes = [u32, u32, u32]
        L.orc_morton3.restype = u32
        L.orc_morton.argtypes = [P, u32, P, P, P, P]
        L.orc_radix_sort.argtypes = [P, P, u32, P, P]
        L.orc_delta.argtypes = [P, u32, C.c_int64, C.c_int64]
        L.orc_delta.restype = i32
        L.orc_karras.argtypes = [P, u32, P, P, P, P, P]
        L.orc_escape.argtypes = [u32, P, P, P, P]
        L.orc_refit_pack.argtypes = [P, u32, P, P, P, P, P]
        L.orc_build.argtypes = [P, u32, P, P, P, P, C.POINTER(Bounds)]
        L.orc_build.restype = i32
        L.orc_pcg_hash.argtypes = [u32]
        L.orc_pcg_hash.restype = u32
        L.orc_fmin.argtypes = [f32, f32]
        L.orc_fmin.restype = f32
        L.orc_fmax.argtypes = [f32, f32]
        L.orc_fmax.restype = f32
        L.orc_intersect_tri.argtypes = [P, P, P, f32, P, P, P]
        L.orc_intersect_tri.restype = i32
        L.orc_trace.argtypes = [P, u32, P, C.POINTER(Camera), u32, u32, u32, u32, u32, P, P, i32]
        L.orc_shade.argtypes = [P, u32, u32, u32, P]
        L.orc_render_shadow.argtypes = [P, u32, P, C.POINTER(Camera), u32, u32, u32, P, f32, P, P, P, i32]
        L.orc_render_path.argtypes = [P, u32, P, C.POINTER(Camera), u32, u32, u32, P, f32, u32, P, P, P, i32]
        L.orc_debug_fail_spawn.argtypes = [i32]
        _lib = L
    return _lib


def default_threads() -> int:
    """Host threads for the oracle's traces: the CPUs this process may use,
    at most 16 (the GPU box's CPU share; os.cpu_count() shows the machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def soup(n: int, seed: int = 1) -> np.ndarray:
    t = np.empty((n, 9), dtype=np.float32)
    lib().orc_soup_generate(n, seed, _p(t))
    return t


def camera_look_at(eye, at, up, vfov_deg, w, h) -> Camera:
    cam = Camera()
    e = np.asarray(eye, dtype=np.float64)
    a = np.asarray(at, dtype=np.float64)
    u = np.asarray(up, dtype=np.float64)
    lib().orc_camera_look_at(_p(e), _p(a), _p(u), float(vfov_deg), w, h, C.byref(cam))
    return cam


def centroid_bounds(tris: np.ndarray):
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    lo, hi, inv = (np.empty(3, np.float32) for _ in range(3))
    lib().orc_centroid_bounds(_p(tris), tris.shape[0], _p(lo), _p(hi), _p(inv))
    return lo, hi, inv


def morton(tris: np.ndarray, lo, inv):
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    n = tris.shape[0]
    keys = np.empty(n, np.uint32)
    vals = np.empty(n, np.uint32)
    lo = np.ascontiguousarray(lo, np.float32)
    inv = np.ascontiguousarray(inv, np.float32)
    lib().orc_morton(_p(tris), n, _p(lo), _p(inv), _p(keys), _p(vals))
    return keys, vals


def radix_sort(keys: np.ndarray, vals: np.ndarray):
    k = np.array(keys, dtype=np.uint32, copy=True)
    v = np.array(vals, dtype=np.uint32, copy=True)
    n = k.shape[0]
    tk = np.empty(max(n, 1), np.uint32)
    tv = np.empty(max(n, 1), np.uint32)
    lib().orc_radix_sort(_p(k), _p(v), n, _p(tk), _p(tv))
    return k, v


def karras(keys: np.ndarray):
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    n = keys.shape[0]
    m = max(n - 1, 1)
    left, right, rlo, rhi = (np.zeros(m, np.uint32) for _ in range(4))
    parent = np.zeros(max(2 * n - 1, 1), np.uint32)
    lib().orc_karras(_p(keys), n, _p(left), _p(right), _p(rlo), _p(rhi), _p(parent))
    k = max(n - 1, 0)
    return left[:k], right[:k], rlo[:k], rhi[:k], parent[: max(2 * n - 1, 0)]


def escape(n: int, left, right, parent):
    esc = np.zeros(max(2 * n - 1, 1), np.uint32)
    l = np.ascontiguousarray(left, np.uint32) if len(left) else np.zeros(1, np.uint32)
    r = np.ascontiguousarray(right, np.uint32) if len(right) else np.zeros(1, np.uint32)
    lib().orc_escape(n, _p(l), _p(r), _p(np.ascontiguousarray(parent, np.uint32)), _p(esc))
    return esc[: max(2 * n - 1, 0)]


def build(tris: np.ndarray):
    """Full oracle build. Returns dict(nodes, keys, vals, parent, lo, hi, inv)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    n = tris.shape[0]
    nodes = np.zeros(max(2 * n - 1, 1), NODE_DTYPE)
    keys = np.zeros(max(n, 1), np.uint32)
    vals = np.zeros(max(n, 1), np.uint32)
    parent = np.zeros(max(2 * n - 1, 1), np.uint32)
    b = Bounds()
    rc = lib().orc_build(_p(tris), n, _p(nodes), _p(keys), _p(vals), _p(parent), C.byref(b))
    if rc != 0:
        raise MemoryError("orc_build failed")
    return dict(nodes=nodes[: max(2 * n - 1, 0)], keys=keys[:n], vals=vals[:n],
                parent=parent[: max(2 * n - 1, 0)], lo=np.array(b.lo[:], np.float32),
                hi=np.array(b.hi[:], np.float32), inv=np.array(b.inv[:], np.float32))


def trace(nodes, tris, cam: Camera, w, h, spp=1, row0=0, row_step=1, nthreads=None, hits=None):
    """Returns (hits[h*w*spp] HIT_DTYPE, counters[2] = nodes fetched, tris tested)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    n = tris.shape[0]
    if hits is None:
        hits = np.zeros(max(w * h * spp, 1), HIT_DTYPE)
        hits["t"] = np.inf
        hits["prim"] = SENTINEL
    cnt = np.zeros(2, np.uint64)
    nd = np.ascontiguousarray(nodes) if len(nodes) else np.zeros(1, NODE_DTYPE)
    tr = tris if n else np.zeros((1, 9), np.float32)
    nthreads = nthreads or default_threads()
    lib().orc_trace(_p(nd), n, _p(tr), C.byref(cam), w, h, spp, row0, row_step, _p(hits), _p(cnt), int(nthreads))
    return hits[: w * h * spp], cnt


def render_shadow(nodes, tris, cam: Camera, w, h, spp, light, ambient, nthreads=None):
    """Shadow mode: returns (primary hits, rgba, shadow counters)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    n = tris.shape[0]
    hits = np.zeros(max(w * h * spp, 1), HIT_DTYPE)
    hits["t"] = np.inf
    hits["prim"] = SENTINEL
    rgba = np.zeros(max(w * h * 4, 1), np.uint8)
    cnt = np.zeros(2, np.uint64)
    nd = np.ascontiguousarray(nodes) if len(nodes) else np.zeros(1, NODE_DTYPE)
    tr = tris if n else np.zeros((1, 9), np.float32)
    L = np.ascontiguousarray(light, np.float32).reshape(3)
    nthreads = nthreads or default_threads()
    lib().orc_render_shadow(_p(nd), n, _p(tr), C.byref(cam), w, h, spp, _p(L), float(ambient), _p(hits), _p(rgba),
                            _p(cnt), int(nthreads))
    return hits[: w * h * spp], rgba[: w * h * 4], cnt


def render_path(nodes, tris, cam: Camera, w, h, spp, light, sky, max_depth, nthreads=None):
    """Path mode: returns (primary hits, rgba, counters[nodes, tris, rays])."""
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    n = tris.shape[0]
    hits = np.zeros(max(w * h * spp, 1), HIT_DTYPE)
    rgba = np.zeros(max(w * h * 4, 1), np.uint8)
    cnt = np.zeros(3, np.uint64)
    nd = np.ascontiguousarray(nodes) if len(nodes) else np.zeros(1, NODE_DTYPE)
    tr = tris if n else np.zeros((1, 9), np.float32)
    L = np.ascontiguousarray(light, np.float32).reshape(3)
    nthreads = nthreads or default_threads()
    lib().orc_render_path(_p(nd), n, _p(tr), C.byref(cam), w, h, spp, _p(L), float(sky), int(max_depth), _p(hits),
                          _p(rgba), _p(cnt), int(nthreads))
    return hits[: w * h * spp], rgba[: w * h * 4], cnt


def shade(hits, w, h, spp=1):
    rgba = np.zeros(max(w * h * 4, 1), np.uint8)
    lib().orc_shade(_p(np.ascontiguousarray(hits)), w, h, spp, _p(rgba))
    return rgba[: w * h * 4]


def intersect_tri(o, d, tri, t_best=np.inf):
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    tri = np.ascontiguousarray(tri, np.float32).reshape(9)
    t, u, v = (np.zeros(1, np.float32) for _ in range(3))
    hit = lib().orc_intersect_tri(_p(o), _p(d), _p(tri), float(t_best), _p(t), _p(u), _p(v))
    return bool(hit), float(t[0]), float(u[0]), float(v[0])
