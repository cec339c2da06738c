"""gpu_raytracer_amd -- MI355X-native (gfx950) BVH build + ray trace.

The hot path lives in librtamd.so: hand-written HIP kernels
behind the C-ABI in include/gpu_raytracer_amd.h.  This package is the Python
side of that boundary (ctypes) plus the scene presets used by bench.py; it
contains no compute and no CPU fallback.
"""
from ._lib import RT_BACKEND_CPU, RT_BACKEND_HIP, RtError, build_library, lib, SENTINEL  # noqa: F401
from .scene import (  # noqa: F401
    HIT_DTYPE, NODE_DTYPE, Scene, camera_array, config_set, camera_look_at, device_count, dump_hits, dump_ppm,
    stage_bounds, stage_intersect, stage_minmax, stage_morton, stage_refit, stage_sort, stage_topology, stage_trace,
    tiles_for_rank, unpack_tiles_device,
)
from . import scenes  # noqa: F401

__version__ = "0.1.0"
