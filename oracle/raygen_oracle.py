"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

An independent numpy restatement of the reference's AO / diffuse ray generator
rayGenAOKernel (src/rt/ray/RayGenKernels.cu:117-227) and of its Jenkins hash
(RayGenKernels.cu:36-47), written from the reference source without reusing the
product's raygen_common.hpp, so the device generator (csrc/raygen_kernel.hip) is
checked against something other than its own header.

Per input ray i of a batch (task index i, input slot first + i):
  origin  = o + d * max(t - 1e-4, 0)                         (:138-139, float32 mul then add)
  normal  = normals[id] (or (1,0,0) for a miss), flipped to face the viewer  (:143-147)
  perp    = the normal's perpendicular on its largest axis, normalised; biperp = n x perp  (:151-158)
  angle   = 2 pi * jenkins(seed + i) * 2^-32                   (:162-167)
  sample s: Halton(2,3) point (s + 1) warped onto the cosine hemisphere,
            dir = normalize(x t0 + y t1 + z n), tmin = 0, tmax = maxDist (or -1 for a miss)

Returned in float64 next to the float32 fields that are exact restatements
(origin, tmin, tmax, the normal and the hash angle); the directions involve
cosf/sinf, which differ between the device and libm, so tests compare them with a
tolerance.
"""
from __future__ import annotations

import numpy as np

PI_F32 = np.float32(3.14159265358979323846)


def jenkins_mix(a, b, c):
    """RayGenKernels.cu:36-47 on uint32 arrays (wrapping)."""
    def step(x, y, z, shift, left):
        x = (x - y - z) & 0xFFFFFFFF
        x ^= ((z << shift) & 0xFFFFFFFF) if left else (z >> shift)
        return x
    a = step(a, b, c, 13, False); b = step(b, c, a, 8, True); c = step(c, a, b, 13, False)
    a = step(a, b, c, 12, False); b = step(b, c, a, 16, True); c = step(c, a, b, 5, False)
    a = step(a, b, c, 3, False); b = step(b, c, a, 10, True); c = step(c, a, b, 15, False)
    return a, b, c


def hash_angle(seed: int, n: int) -> np.ndarray:
    """float32 rotation angle of tasks 0..n-1 (RayGenKernels.cu:162-167)."""
    a = (np.uint64(seed) + np.arange(n, dtype=np.uint64)) & np.uint64(0xFFFFFFFF)
    b = np.full(n, 0x9E3779B9, np.uint64)
    c = np.full(n, 0x9E3779B9, np.uint64)
    a, b, c = jenkins_mix(a, b, c)
    a, b, c = jenkins_mix(a, b, c)
    two_pi = np.float32(2.0) * PI_F32
    return (two_pi * c.astype(np.float32)) * np.float32(2.0 ** -32)


def halton23(i: int):
    """Base-2 / base-3 radical inverses of i + 1 in the kernel's float32 accumulation order."""
    x, xadd, h = np.float32(0), np.float32(1), i + 1
    while h:
        xadd = np.float32(xadd * np.float32(0.5))
        if h & 1:
            x = np.float32(x + xadd)
        h >>= 1
    y, yadd, h = np.float32(0), np.float32(1), i + 1
    third = np.float32(1.0) / np.float32(3.0)
    while h:
        yadd = np.float32(yadd * third)
        y = np.float32(y + np.float32(h % 3) * yadd)
        h //= 3
    return x, y


def ao_rays(in_rays: np.ndarray, in_results: np.ndarray, normals: np.ndarray, num_samples: int, max_dist: float,
            seed: int):
    """Restated rayGenAOKernel over one batch. in_rays float32 [n, 8], in_results int32 [n, 4],
    normals float32 [tris, 3]. Returns a dict of arrays (per output ray unless noted)."""
    rays = np.ascontiguousarray(in_rays, np.float32).reshape(-1, 8)
    res = np.ascontiguousarray(in_results).view(np.int32).reshape(-1, 4)
    n = len(rays)
    o, d = rays[:, 0:3], rays[:, 4:7]
    t = res[:, 1].view(np.float32)
    ids = res[:, 0]
    back = np.maximum(t - np.float32(1e-4), np.float32(0.0)).astype(np.float32)
    origin = (o + (d * back[:, None]).astype(np.float32)).astype(np.float32)
    miss = ids == -1
    nrm = np.tile(np.array([1, 0, 0], np.float32), (n, 1))
    nrm[~miss] = normals[ids[~miss]]
    facing = (((nrm[:, 0] * d[:, 0]).astype(np.float32) + (nrm[:, 1] * d[:, 1]).astype(np.float32))
              .astype(np.float32) + (nrm[:, 2] * d[:, 2]).astype(np.float32)).astype(np.float32)
    nrm = np.where((facing > 0)[:, None], -nrm, nrm).astype(np.float32)
    na = np.abs(nrm)
    nm = np.maximum(np.maximum(na[:, 0], na[:, 1]), na[:, 2])
    perp = np.stack([nrm[:, 1], -nrm[:, 0], np.zeros(n, np.float32)], 1)
    z_axis = nm == na[:, 2]
    x_axis = ~z_axis & (nm == na[:, 0])
    perp[z_axis] = np.stack([np.zeros(z_axis.sum(), np.float32), nrm[z_axis, 2], -nrm[z_axis, 1]], 1)
    perp[x_axis] = np.stack([-nrm[x_axis, 2], np.zeros(x_axis.sum(), np.float32), nrm[x_axis, 0]], 1)
    perp64 = perp.astype(np.float64)
    perp64 /= np.linalg.norm(perp64, axis=1, keepdims=True)
    n64 = nrm.astype(np.float64)
    biperp = np.cross(n64, perp64)
    angle = hash_angle(seed, n).astype(np.float64)
    t0 = perp64 * np.cos(angle)[:, None] + biperp * np.sin(angle)[:, None]
    t1 = perp64 * -np.sin(angle)[:, None] + biperp * np.cos(angle)[:, None]
    dirs = np.empty((n, num_samples, 3))
    for s in range(num_samples):
        hx, hy = halton23(s)
        a2 = 2.0 * np.pi * float(hy)
        r = np.sqrt(float(hx))
        x, y = r * np.cos(a2), r * np.sin(a2)
        z = np.sqrt(max(0.0, 1.0 - x * x - y * y))
        v = x * t0 + y * t1 + z * n64
        dirs[:, s] = v / np.linalg.norm(v, axis=1, keepdims=True)
    out = {
        "origin": np.repeat(origin, num_samples, axis=0),
        "tmin": np.zeros(n * num_samples, np.float32),
        "tmax": np.repeat(np.where(miss, np.float32(-1.0), np.float32(max_dist)), num_samples),
        "normal": np.repeat(nrm, num_samples, axis=0),
        "dir": dirs.reshape(-1, 3),
        "angle": np.repeat(hash_angle(seed, n), num_samples),
    }
    return out
