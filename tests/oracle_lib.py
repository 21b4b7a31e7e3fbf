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
        L.oracle_woop_hit_rcp.restype = C.c_int
        L.oracle_woop_hit_rcp.argtypes = [vp, vp, i64, i64, C.c_float, C.c_int, C.POINTER(C.c_float)]
        L.oracle_check_hits.restype = i64
        L.oracle_check_hits.argtypes = [vp, vp, vp, i64, vp, i64, vp, C.c_int, vp]
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


def woop_hit_rcp(ray, woop, slot, tmax, rcp_ulps):
    """The Woop test with 1/Dz moved by rcp_ulps ulps (oracle_woop_hit_rcp)."""
    ray = np.ascontiguousarray(ray, np.float32).reshape(8)
    woop = np.ascontiguousarray(woop).view(np.int32)
    t = C.c_float()
    hit = lib().oracle_woop_hit_rcp(_p(ray), _p(woop), woop.nbytes, int(slot), float(tmax), int(rcp_ulps),
                                    C.byref(t))
    return bool(hit), float(t.value)


def invalid_hits(rays, res, woop, tri_index, which=None, rcp_ulps=0):
    """Indices (into rays) of reported results that are not genuine: a hit {id, t} no
    triangle with that triIndex reproduces under the Woop test of the ray against its
    (tmin, tmax) with 1/Dz within rcp_ulps ulps of 1/Dz, or a miss whose t is not the
    ray's tmax (oracle_check_hits). which: the rays to check (default: all)."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    res = np.ascontiguousarray(res, np.int32).reshape(-1, 4)
    woop = np.ascontiguousarray(woop).view(np.int32)
    tri = np.ascontiguousarray(tri_index, np.int32)
    idx = np.arange(len(rays), dtype=np.int64) if which is None else np.ascontiguousarray(which, np.int64)
    ok = np.zeros(len(idx), np.uint8)
    if len(idx):
        lib().oracle_check_hits(_p(rays), _p(res), _p(idx), len(idx), _p(woop), woop.nbytes, _p(tri), int(rcp_ulps),
                                _p(ok))
    return idx[ok == 0]


def _ulps(a, b):
    ia, ib = (int(np.float32(x).view(np.int32)) for x in (a, b))
    ia = -(ia & 0x7FFFFFFF) if ia < 0 else ia
    ib = -(ib & 0x7FFFFFFF) if ib < 0 else ib
    return abs(ia - ib)


def classify_fast_rcp(rays, gpu, want, woop, tri_index, limit=20000):
    """SURVEY.md §8(a) Note 3: closest-hit results of the fast-reciprocal mode
    (v_rcp_f32, the analogue of the reference's rcp.approx) against the oracle's
    correctly rounded ones. A ray agrees when its id is equal and t within 2 ulp.
    A mismatch is
      * "tie":  both triangles are valid hits of the ray under the exact Woop test
                and their t lie within 4 ulp of each other (traversal order decides);
      * "edge": the oracle's triangle fails, or the GPU's passes, the Woop test once
                1/Dz moves by one ulp (v_rcp_f32's error bound): the outcome is
                decided by the reciprocal's rounding (a grazing ray on an edge);
      * "other": anything else (a real error; expected 0).
    Returns counts and up to 20 example rays per class."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    woop = np.ascontiguousarray(woop).view(np.int32)
    tri = np.ascontiguousarray(tri_index, np.int32)
    woop4 = woop.reshape(-1, 4)
    live = woop4[:, 0] != np.int32(-2147483648)
    g_id, w_id = gpu[:, 0], want[:, 0]
    g_t, w_t = gpu[:, 1].view(np.float32), want[:, 1].view(np.float32)
    # ulp distance of t, vectorised
    def ord_(x):
        i = x.view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    dt = np.abs(ord_(g_t) - ord_(w_t))
    bad = np.nonzero((g_id != w_id) | (dt > 2))[0]
    out = {"rays": int(len(rays)), "mismatch": int(len(bad)), "tie": 0, "edge": 0, "other": 0,
           "examples": {"tie": [], "edge": [], "other": []}}
    slots_of = {}

    def slots(tid):
        if tid not in slots_of:
            slots_of[tid] = np.nonzero((tri == tid) & live)[0]
        return slots_of[tid]
    for i in bad[:limit]:
        r = rays[i]
        tmax = float(r[7])
        cls = "other"
        if g_id[i] != -1 and w_id[i] != -1:
            exact_g = [t for s in slots(int(g_id[i])) for h, t in [woop_hit(r, woop, s, tmax)] if h]
            if exact_g and min(_ulps(t, w_t[i]) for t in exact_g) <= 4 and _ulps(g_t[i], w_t[i]) <= 4:
                cls = "tie"
        if cls == "other":
            flips = False
            for tid, wanted in ((int(w_id[i]), True), (int(g_id[i]), False)):
                if tid == -1:
                    continue
                for s in slots(tid):
                    res = [woop_hit_rcp(r, woop, s, tmax, k)[0] for k in (-1, 0, 1)]
                    if len(set(res)) > 1:
                        flips = True
            # the oracle's hit missed by the GPU, or a GPU hit the oracle did not take, decided by 1/Dz rounding
            if flips:
                cls = "edge"
        out[cls] += 1
        if len(out["examples"][cls]) < 20:
            out["examples"][cls].append([int(i), int(g_id[i]), float(g_t[i]), int(w_id[i]), float(w_t[i])])
    out["unclassified"] = int(max(0, len(bad) - limit))
    return out


def classify_any_hit_flips(rays, gpu, want, woop, tri_index):
    """Any-hit rays whose hit/miss outcome differs between the fast-reciprocal GPU mode
    and the oracle: an "edge" flip when the triangle that decided it (the GPU's hit, or
    the oracle's) changes acceptance once 1/Dz moves by one ulp (v_rcp_f32's bound),
    else "other". Returns {"flips", "edge", "other"}."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    woop = np.ascontiguousarray(woop).view(np.int32)
    tri = np.ascontiguousarray(tri_index, np.int32)
    live = woop.reshape(-1, 4)[:, 0] != np.int32(-2147483648)
    flips = np.nonzero((gpu[:, 0] == -1) != (want[:, 0] == -1))[0]
    out = {"flips": int(len(flips)), "edge": 0, "other": 0}
    for i in flips:
        tid = int(gpu[i, 0] if gpu[i, 0] != -1 else want[i, 0])
        edge = any(len({woop_hit_rcp(rays[i], woop, s, float(rays[i][7]), k)[0] for k in (-1, 0, 1)}) > 1
                   for s in np.nonzero((tri == tid) & live)[0])
        out["edge" if edge else "other"] += 1
    return out


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
