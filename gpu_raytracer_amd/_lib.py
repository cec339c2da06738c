"""ctypes loader for librtamd.so (the C-ABI declared in include/gpu_raytracer_amd.h).

The library is built in-tree (``make -C gpu_raytracer_amd`` or
``__graft_entry__.build()``) into ``gpu_raytracer_amd/lib/librtamd.so``.  There
is no fallback: if the library is missing or cannot be loaded this module
raises, and every compute entry point of the library itself returns
RT_EDEVICE when no gfx950 device is visible.

torch is imported (when installed) BEFORE the library is dlopen'ed so that the
process holds exactly one HIP runtime: torch's bundled libamdhip64.so carries
the SONAME libamdhip64.so.7 that librtamd.so links against, so the loader
reuses it instead of mapping /opt/rocm's copy beside it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

try:  # one HIP runtime per process (see module docstring)
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the ABI itself
    _torch = None

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RT_LIB overrides the library path (diagnostic stamp build, tools/diag_stamps.py)
LIB_PATH = os.environ.get("RT_LIB") or os.path.join(PKG_DIR, "lib", "librtamd.so")

RT_OK, RT_EINVAL, RT_ENOMEM, RT_EIO, RT_EDEVICE, RT_ECOMM = 0, -1, -2, -3, -4, -5
RT_BACKEND_CPU, RT_BACKEND_HIP = 0, 1
SENTINEL = 0xFFFFFFFF
_STATUS_NAMES = {0: "RT_OK", -1: "RT_EINVAL", -2: "RT_ENOMEM", -3: "RT_EIO", -4: "RT_EDEVICE", -5: "RT_ECOMM"}

# every symbol the header declares (checked by tests/test_abi.py)
EXPORTED = [
    "rt_scene_from_soup", "rt_scene_load_obj", "rt_scene_generate_soup", "rt_scene_load_soup",
    "rt_scene_save_soup", "rt_bvh_save", "rt_bvh_load", "rt_scene_num_tris",
    "rt_scene_get_tris", "rt_scene_set_device", "rt_scene_free", "rt_camera_look_at", "rt_bvh_build",
    "rt_bvh_build_times", "rt_bvh_build_times_sized", "rt_bvh_read", "rt_bvh_read_wide", "rt_bvh_wide_arity", "rt_render", "rt_render_timed", "rt_render_counters",
    "rt_render_work", "rt_render_device",
    "rt_render_shadow", "rt_render_shadow_device", "rt_render_shadow_work",
    "rt_render_path", "rt_render_path_device", "rt_render_path_work",
    "rt_bvh_prepare", "rt_bvh_device_sections", "rt_bvh_mark_built", "rt_bvh_replicas",
    "rt_render_tiles_counters", "rt_render_tiles_work", "rt_render_step_map", "rt_tiles_for_rank",
    "rt_render_tiles_device", "rt_unpack_tiles_device", "rt_scene_stream", "rt_scene_sync",
    "rt_stage_bounds", "rt_stage_morton", "rt_stage_sort", "rt_stage_topology", "rt_stage_refit", "rt_stage_trace",
    "rt_stage_intersect", "rt_stage_minmax", "rt_framebuffer_dump_ppm", "rt_hits_dump",
    "rt_config_set", "rt_last_error", "rt_device_count", "rt_version",
    "rt_dbuild_shares", "rt_dbuild_bounds", "rt_dbuild_keys", "rt_dbuild_sort", "rt_dbuild_subtrees",
    "rt_dbuild_merge", "rt_dbuild_buffer",
]
# rt_dbuild_buffer selectors (include/gpu_raytracer_amd.h)
(RT_DB_SEND_KEYS, RT_DB_SEND_VALS, RT_DB_RECV_KEYS, RT_DB_RECV_VALS, RT_DB_KEYS, RT_DB_VALS, RT_DB_NODES,
 RT_DB_TRI_S, RT_DB_WIDE, RT_DB_TOPO, RT_DB_PRE, RT_DB_SUF, RT_DB_TOTALS, RT_DB_CROSS, RT_DB_CROSS_ALL) = range(15)


class RtError(RuntimeError):
    def __init__(self, status: int, func: str, msg: str):
        self.status = status
        super().__init__(f"{func} -> {_STATUS_NAMES.get(status, status)}: {msg}")


class rt_camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("w00", C.c_float * 3), ("du", C.c_float * 3), ("dv", C.c_float * 3)]


class rt_build_times(C.Structure):
    _fields_ = ([(k, C.c_double) for k in ("bounds", "morton", "sort", "topology", "refit", "wide", "total")] +
                [("sort_kind", C.c_uint32), ("fused_k01", C.c_uint32), ("fused_fallback", C.c_uint32),
                 ("lsb_redo", C.c_uint32)])


def build_library(verbose: bool = False) -> str:
    """Compile librtamd.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    r = subprocess.run(["make", "-j8", "-C", PKG_DIR], capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("building librtamd.so failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return LIB_PATH


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` or __graft_entry__.build(). "
            "There is no CPU fallback.")
    L = C.CDLL(LIB_PATH)
    P, u32, u64, i32, dbl = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_double
    PP = C.POINTER(C.c_void_p)
    cam = C.POINTER(rt_camera)
    sig = {
        "rt_scene_from_soup": [P, u32, PP],
        "rt_scene_load_obj": [C.c_char_p, PP],
        "rt_scene_load_soup": [C.c_char_p, PP],
        "rt_scene_save_soup": [P, C.c_char_p],
        "rt_bvh_save": [P, C.c_char_p],
        "rt_bvh_load": [P, C.c_char_p],
        "rt_scene_generate_soup": [u32, u64, PP],
        "rt_scene_num_tris": [P, C.POINTER(u32)],
        "rt_scene_get_tris": [P, P],
        "rt_scene_set_device": [P, i32],
        "rt_camera_look_at": [P, P, P, dbl, u32, u32, cam],
        "rt_bvh_build": [P, i32, u32, C.POINTER(dbl)],
        "rt_bvh_replicas": [P, u32, P, C.POINTER(u32)],
        "rt_bvh_build_times": [P, C.POINTER(rt_build_times)],
        "rt_bvh_build_times_sized": [P, C.POINTER(rt_build_times), C.c_size_t],
        "rt_bvh_read": [P, P, P, P, P, P],
        "rt_bvh_read_wide": [P, P],
        "rt_bvh_wide_arity": [P, C.POINTER(u32)],
        "rt_render": [P, cam, u32, u32, u32, u32, P, P],
        "rt_render_timed": [P, cam, u32, u32, u32, u32, P, P, C.POINTER(dbl)],
        "rt_render_counters": [P, cam, u32, u32, u32, P],
        "rt_render_work": [P, cam, u32, u32, u32, P],
        "rt_render_shadow": [P, cam, P, C.c_float, u32, u32, u32, P, P, C.POINTER(dbl)],
        "rt_render_shadow_device": [P, cam, P, C.c_float, u32, u32, u32, P, P, P, C.POINTER(dbl)],
        "rt_render_shadow_work": [P, cam, P, C.c_float, u32, u32, u32, P],
        "rt_render_path": [P, cam, P, C.c_float, u32, u32, u32, u32, P, P, C.POINTER(dbl)],
        "rt_render_path_device": [P, cam, P, C.c_float, u32, u32, u32, u32, P, P, P, C.POINTER(dbl)],
        "rt_render_path_work": [P, cam, P, C.c_float, u32, u32, u32, u32, P],
        "rt_bvh_prepare": [P],
        "rt_bvh_device_sections": [P, u32, P, P, P],
        "rt_bvh_mark_built": [P],
        "rt_render_device": [P, cam, u32, u32, u32, P, P, P, C.POINTER(dbl)],
        "rt_render_tiles_counters": [P, cam, u32, u32, u32, u32, u32, P],
        "rt_render_tiles_work": [P, cam, u32, u32, u32, u32, u32, P],
        "rt_render_step_map": [P, u32, u32, u32, u32, u32, P, C.c_size_t],
        "rt_render_tiles_device": [P, cam, u32, u32, u32, u32, u32, P, P, P, C.POINTER(dbl)],
        "rt_unpack_tiles_device": [P, u32, u32, u32, u32, P, i32, P],
        "rt_scene_stream": [P, PP],
        "rt_scene_sync": [P],
        "rt_stage_bounds": [i32, P, u32, P],
        "rt_stage_morton": [i32, P, u32, P, P, P, P],
        "rt_stage_sort": [i32, P, P, u32],
        "rt_stage_topology": [i32, P, u32, P, P, P],
        "rt_stage_refit": [i32, P, P, P, u32, P],
        "rt_stage_trace": [i32, P, u32, P, cam, u32, u32, u32, P, P, P],
        "rt_stage_intersect": [i32, u32, P, P, P, P, P, P],
        "rt_stage_minmax": [i32, u32, P, P, P],
        "rt_framebuffer_dump_ppm": [P, u32, u32, C.c_char_p],
        "rt_hits_dump": [P, C.c_size_t, C.c_char_p],
        "rt_config_set": [C.c_char_p, C.c_int64],
        "rt_dbuild_shares": [u32, u32, u32, P],
        "rt_dbuild_bounds": [P, u32, u32, P],
        "rt_dbuild_keys": [P, u32, u32, P, P],
        "rt_dbuild_sort": [P, u32],
        "rt_dbuild_subtrees": [P, u32, u32, C.POINTER(u32)],
        "rt_dbuild_merge": [P, u32],
        "rt_dbuild_buffer": [P, i32, PP, C.POINTER(u64)],
    }
    for name, args in sig.items():
        if os.environ.get("RT_LIB") and not hasattr(L, name):
            continue  # an older library under A/B (tools/ab_libs.py): bind what it has
        f = getattr(L, name)
        f.argtypes = args
        f.restype = i32
    L.rt_scene_free.argtypes = [P]
    L.rt_scene_free.restype = None
    L.rt_tiles_for_rank.argtypes = [u32, u32, u32, u32]
    L.rt_tiles_for_rank.restype = u32
    L.rt_last_error.argtypes = []
    L.rt_last_error.restype = C.c_char_p
    L.rt_device_count.argtypes = []
    L.rt_device_count.restype = i32
    L.rt_version.argtypes = []
    L.rt_version.restype = C.c_char_p
    _lib = L
    return L


def check(status: int, func: str) -> None:
    if status != RT_OK:
        msg = lib().rt_last_error()
        raise RtError(status, func, msg.decode() if msg else "")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
