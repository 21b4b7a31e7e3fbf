"""ctypes access to the CPU oracle (oracle/build/liboracle.so) — test
infrastructure only: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg are the only callers."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        vp, i64 = C.c_void_p, C.c_int64
        L.oracle_trace.restype = C.c_double
        L.oracle_trace.argtypes = [vp, vp, i64, C.c_int, vp, i64, vp, i64, vp, vp, C.c_int]
        L.oracle_woop_hit.restype = C.c_int
        L.oracle_woop_hit.argtypes = [vp, vp, i64, i64, C.c_float, C.POINTER(C.c_float)]
        L.oracle_brute_force.restype = None
        L.oracle_brute_force.argtypes = [vp, vp, i64, C.c_int, vp, i64, vp]
        L.oracle_tri_colors.restype = None
        L.oracle_tri_colors.argtypes = [vp, i64, vp, vp]
        L.oracle_tri_colors_mat.restype = None
        L.oracle_tri_colors_mat.argtypes = [vp, vp, i64, vp, vp]
        L.oracle_reconstruct.restype = None
        L.oracle_reconstruct.argtypes = [C.c_int] * 4 + [vp] * 7
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data


def trace(rays, nodes, woop, tri_index, any_hit=False, stats=False, threads=1):
    """Returns (results int32[n,4] with pads zero, stats int32[n,4] or None, seconds)."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    nodes = np.ascontiguousarray(nodes).view(np.int32)
    woop = np.ascontiguousarray(woop).view(np.int32)
    tri = np.ascontiguousarray(tri_index, np.int32)
    n = len(rays)
    res = np.zeros((n, 4), np.int32)
    st = np.zeros((n, 4), np.int32) if stats else None
    secs = lib().oracle_trace(_p(rays), _p(res), n, int(any_hit), _p(nodes), nodes.nbytes, _p(woop), woop.nbytes,
                              _p(tri), _p(st) if stats else None, threads)
    return res, st, secs


def woop_hit(ray, woop, slot, tmax):
    ray = np.ascontiguousarray(ray, np.float32).reshape(8)
    woop = np.ascontiguousarray(woop).view(np.int32)
    t = C.c_float()
    hit = lib().oracle_woop_hit(_p(ray), _p(woop), woop.nbytes, int(slot), float(tmax), C.byref(t))
    return bool(hit), float(t.value)


def brute_force(rays, woop, tri_index, any_hit=False):
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    woop = np.ascontiguousarray(woop).view(np.int32)
    tri = np.ascontiguousarray(tri_index, np.int32)
    res = np.zeros((len(rays), 4), np.int32)
    lib().oracle_brute_force(_p(rays), _p(res), len(rays), int(any_hit), _p(woop), woop.nbytes, _p(tri))
    return res


def tri_colors(normals, diffuse=None):
    """Scene::Scene colour tables (material, shaded) as uint32 ABGR; diffuse: (n, 4)
    per-triangle Material::diffuse, None = the default 0.75 grey."""
    normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
    n = normals.shape[0]
    mat = np.empty(n, np.uint32)
    sh = np.empty(n, np.uint32)
    if diffuse is None:
        lib().oracle_tri_colors(_p(normals), n, _p(mat), _p(sh))
    else:
        d = np.ascontiguousarray(diffuse, np.float32).reshape(n, 4)
        lib().oracle_tri_colors_mat(_p(normals), _p(d), n, _p(mat), _p(sh))
    return mat, sh


def reconstruct(ray_type, num_rays_per_primary, primary_slot_to_id, primary_results, batch_results,
                tri_material, tri_shaded, num_pixels, batch_id_to_slot=None, first_primary=0, num_primary=None):
    """reconstructKernel on the CPU; returns num_pixels uint32 ABGR (untouched pixels 0)."""
    s2i = np.ascontiguousarray(primary_slot_to_id, np.int32)
    pres = np.ascontiguousarray(primary_results, np.int32).reshape(-1, 4)
    bres = np.ascontiguousarray(batch_results, np.int32).reshape(-1, 4)
    mat = np.ascontiguousarray(tri_material, np.uint32)
    sh = np.ascontiguousarray(tri_shaded, np.uint32)
    if num_primary is None:
        num_primary = s2i.shape[0] - first_primary
    b2s = None if batch_id_to_slot is None else np.ascontiguousarray(batch_id_to_slot, np.int32)
    pix = np.zeros(num_pixels, np.uint32)
    lib().oracle_reconstruct(ray_type, num_rays_per_primary, first_primary, num_primary, _p(s2i), _p(pres),
                             None if b2s is None else _p(b2s), _p(bres), _p(mat), _p(sh), _p(pix))
    return pix
