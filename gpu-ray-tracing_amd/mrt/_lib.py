"""ctypes bindings of the two in-tree native libraries.

lib/libmrt.so       include/mrt.h       (gfx950 traversal kernels + C-ABI; the hot path)
lib/libmrt_host.so  include/mrt_host.h  (scenes, SBVH builder, Compact2, ray generation)

Both are built by ``make -C gpu-ray-tracing_amd`` (``__graft_entry__.build()``).
There is no fallback: if a library is missing, importing the part of the
package that needs it raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.environ.get("MRT_LIB_DIR") or os.path.join(PKG_DIR, "lib")
TRACE_LIB_PATH = os.path.join(LIB_DIR, "libmrt.so")
# A variant directory (tools/build_variant.sh) holds only libmrt.so; the host
# library then comes from the regular build.
HOST_LIB_PATH = os.path.join(LIB_DIR if os.path.exists(os.path.join(LIB_DIR, "libmrt_host.so"))
                             else os.path.join(PKG_DIR, "lib"), "libmrt_host.so")

# include/mrt.h
MRT_TRACE_ANY_HIT = 1 << 0
MRT_TRACE_EXACT_RCP = 1 << 1
MRT_TRACE_LOCKSTEP_OFF = 1 << 2
MRT_TRACE_STATS = 1 << 3
MRT_TRACE_SECONDARY = 1 << 4
MRT_ERR_INVALID_ARG = 1
MRT_ERR_STACK_OVERFLOW = 6

vp, i32, i64, u32, f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_float


class LaunchCfg(C.Structure):
    _fields_ = [("waves_per_cu", i32), ("fetch_threshold", i32), ("num_queues", i32), ("lds_stack", i32),
                ("lane_groups", i32), ("wide", i32), ("spec_slack", i32), ("static_rounds", i32), ("autotune", i32),
                ("tail_lanes", i32), ("queue_shared", i32), ("queue_block", i32), ("ray_sort", i32),
                ("queue_xcc_mask", i32)]


class TraceInfo(C.Structure):
    _fields_ = [("kernel_ms", f32), ("grid_waves", i32), ("block_threads", i32),
                ("lds_stack_entries", i32), ("wide", i32), ("num_queues", i32), ("fetch_threshold", i32), ("stack_overflows", i32), ("node_bytes", i32),
                ("autotune_candidate", i32), ("autotune_locked", i32), ("stack_capacity", i32)]


class BindInfo(C.Structure):
    _fields_ = [("bind_ms", C.c_double), ("wide_bytes", i64), ("wide_format", i32), ("stack_capacity", i32),
                ("stack_bound", i32)]


class TunedSchedule(C.Structure):
    _fields_ = [("num_rays", i32), ("variant", i32), ("candidate", i32), ("version", i32)]


MRT_TUNE_VERSION = 11


class HostCamera(C.Structure):
    _fields_ = [("position", f32 * 3), ("forward", f32 * 3), ("up", f32 * 3),
                ("fov_deg", f32), ("near_dist", f32), ("far_dist", f32)]


class BuildParams(C.Structure):
    _fields_ = [("sah_node_cost", f32), ("sah_triangle_cost", f32), ("min_leaf_size", i32),
                ("max_leaf_size", i32), ("split_alpha", f32), ("threads", i32)]


class BvhStats(C.Structure):
    _fields_ = [("inner_nodes", i64), ("leaf_nodes", i64), ("tri_refs", i64), ("max_depth", i64),
                ("sah_cost", f32), ("build_seconds", C.c_double)]


# (name, restype, argtypes) of every symbol include/mrt.h declares.
TRACE_SYMBOLS = [
    ("mrt_tracer_create", i32, [i32, C.POINTER(vp)]),
    ("mrt_tracer_destroy", i32, [vp]),
    ("mrt_tracer_bind", i32, [vp, vp, i64, vp, i64, vp, i64]),
    ("mrt_tracer_unbind", i32, [vp]),
    ("mrt_tracer_set_config", i32, [vp, C.POINTER(LaunchCfg)]),
    ("mrt_tracer_get_config", i32, [vp, C.POINTER(LaunchCfg)]),
    ("mrt_tracer_bind_info", i32, [vp, C.POINTER(BindInfo)]),
    ("mrt_tracer_tune_export", i32, [vp, C.POINTER(TunedSchedule), i32, C.POINTER(i32)]),
    ("mrt_tracer_tune_import", i32, [vp, C.POINTER(TunedSchedule), i32]),
    ("mrt_tracer_trace", i32, [vp, vp, vp, i32, u32, vp, vp]),
    ("mrt_tracer_trace_timed", i32, [vp, vp, vp, i32, u32, vp, vp, C.POINTER(TraceInfo)]),
    ("mrt_tracer_stack_overflows", i32, [vp, C.POINTER(i64), i32]),
    ("mrt_derive_wide_nodes", i32, [vp, i64, vp, i64, i32, vp, i64, C.POINTER(i64)]),
    ("mrt_bind_bvh", i32, [vp, i64, vp, i64, vp, i64]),
    ("mrt_unbind_bvh", i32, []),
    ("mrt_trace", i32, [vp, vp, i32, i32, vp, C.POINTER(f32)]),
    ("mrt_error_string", C.c_char_p, [i32]),
    ("mrt_last_error_detail", C.c_char_p, []),
    ("mrt_version", i32, []),
    ("mrt_device_count", i32, []),
    ("mrt_raygen_primary", i32, [C.POINTER(f32), C.POINTER(f32), f32, i32, i32, vp, vp, vp, vp, vp]),
    ("mrt_raygen_primary_subpixel", i32, [C.POINTER(f32), C.POINTER(f32), f32, i32, i32, f32, f32, vp, vp, vp, vp,
                                          vp]),
    ("mrt_raygen_ao", i32, [vp, vp, i32, vp, i64, i32, f32, u32, vp, vp, vp, vp]),
    ("mrt_raygen_ao_blocks", i32, [vp, vp, i32, vp, i64, i32, f32, vp, i32, i32, vp, i32, i32, i64, vp, vp]),
    ("mrt_shard_blocks", i32, [vp, i32, i32, i32, i32, i32, i32, vp, i32, C.POINTER(i32), C.POINTER(i64), vp]),
    ("mrt_count_hits", i32, [vp, i32, vp, vp]),
    ("mrt_reconstruct", i32, [i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    ("mrt_selftest_exact_rcp", i32, [C.POINTER(C.c_uint64)]),
    ("bind_CudaBVHTexture", None, [vp, i64, vp, i64, vp, i64]),
    ("unbind_CudaBVHTexture", None, []),
    ("launch_tracingKernel", f32, [i32, vp, C.c_int, C.c_bool, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    ("copy_tracing_results", None, [vp, vp, i32]),
    ("launch_reconstructKernel", None, [i32, vp]),
    ("launch_rayGenPrimaryKernel", None, [i32, vp]),
    ("launch_rayGenAOKernel", None, [i32, vp]),
    ("launch_countHitsKernel", i32, [i32, vp, vp]),
]

# (name, restype, argtypes) of every symbol include/mrt_host.h declares.
HOST_SYMBOLS = [
    ("mrth_scene_synthetic", i32, [C.c_char_p, i64, C.c_uint64, C.POINTER(vp)]),
    ("mrth_scene_load_obj", i32, [C.c_char_p, C.POINTER(vp)]),
    ("mrth_scene_from_arrays", i32, [vp, i64, vp, i64, C.POINTER(vp)]),
    ("mrth_scene_destroy", None, [vp]),
    ("mrth_scene_num_triangles", i64, [vp]),
    ("mrth_scene_num_vertices", i64, [vp]),
    ("mrth_scene_copy_arrays", i32, [vp, vp, vp, vp]),
    ("mrth_scene_camera", i32, [vp, C.POINTER(HostCamera), C.POINTER(f32)]),
    ("mrth_scene_tri_colors", i32, [vp, vp, vp]),
    ("mrth_default_build_params", None, [C.POINTER(BuildParams)]),
    ("mrth_fw_hash_buffer", u32, [vp, i64]),
    ("mrth_scene_hash", u32, [vp]),
    ("mrth_bvh_cache_name", i32, [vp, C.POINTER(BuildParams), C.c_char_p]),
    ("mrth_bvh_build", i32, [vp, C.POINTER(BuildParams), C.POINTER(vp)]),
    ("mrth_bvh_load", i32, [C.c_char_p, C.POINTER(vp)]),
    ("mrth_bvh_save", i32, [vp, C.c_char_p]),
    ("mrth_bvh_from_buffers", i32, [vp, i64, vp, i64, vp, i64, C.POINTER(vp)]),
    ("mrth_bvh_destroy", None, [vp]),
    ("mrth_bvh_buffers", i32, [vp, C.POINTER(vp), C.POINTER(i64), C.POINTER(vp), C.POINTER(i64),
                               C.POINTER(vp), C.POINTER(i64)]),
    ("mrth_bvh_get_stats", i32, [vp, C.POINTER(BvhStats)]),
    ("mrth_woopify", None, [C.POINTER(f32), C.POINTER(f32), C.POINTER(f32), C.POINTER(f32)]),
    ("mrth_pixel_table", i32, [i32, i32, vp]),
    ("mrth_primary_rays", i32, [C.POINTER(HostCamera), i32, i32, vp, vp]),
    ("mrth_primary_rays_subpixel", i32, [C.POINTER(HostCamera), i32, i32, f32, f32, vp, vp]),
    ("mrth_camera_nscreen_to_world", i32, [C.POINTER(HostCamera), i32, i32, C.POINTER(f32)]),
    ("mrth_camera_decode_signature", i32, [C.c_char_p, C.POINTER(HostCamera), C.POINTER(f32), C.POINTER(i32)]),
    ("mrth_ao_rays", i32, [vp, vp, i64, vp, i32, f32, u32, vp]),
    ("mrth_count_hits", i64, [vp, i64]),
    ("mrth_last_error", C.c_char_p, []),
]

_trace_lib = None
_host_lib = None


def _load(path: str, symbols):
    if not os.path.exists(path):
        raise RuntimeError(f"native library {path} is missing: run `make -C {PKG_DIR}` "
                           f"(or __graft_entry__.build()); there is no Python fallback")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, res, args in symbols:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def trace_lib():
    global _trace_lib
    if _trace_lib is None:
        _trace_lib = _load(TRACE_LIB_PATH, TRACE_SYMBOLS)
    return _trace_lib


def host_lib():
    global _host_lib
    if _host_lib is None:
        _host_lib = _load(HOST_LIB_PATH, HOST_SYMBOLS)
    return _host_lib


class MrtError(RuntimeError):
    pass


def check(rc: int) -> None:
    if rc != 0:
        lib = trace_lib()
        raise MrtError(f"mrt error {rc} ({lib.mrt_error_string(rc).decode()}): "
                       f"{lib.mrt_last_error_detail().decode()}")


def check_host(rc: int) -> None:
    if rc != 0:
        raise MrtError(f"mrt_host error {rc}: {host_lib().mrth_last_error().decode()}")
