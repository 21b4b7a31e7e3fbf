"""Offline analysis (CPU): at which BVH depths do a workload's node visits fall?
Decides how much a treetop node cache (the top levels held in LDS) could serve.

Replays the per-lane traversal order (near child first, far child pushed, leaves
tested in pop order; float64 slab and Woop tests — counts, not bit-exact results)
for a sample of rays of a bench workload built with the host ray generator, and
prints the cumulative share of node visits at depth <= d next to the number of
nodes (and LDS bytes) the top d levels hold.

  python tools/visit_depth.py hairball-diffuse-640x480 [n_rays] [cache_dir]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def node_depths(nodes):
    ni = nodes.reshape(-1, 16)
    depth = np.full(len(ni), -1, np.int32)
    depth[0] = 0
    frontier = [0]
    while frontier:
        nxt = []
        for n in frontier:
            for c in ni[n, 12:14]:
                if c >= 0:
                    depth[c // 4] = depth[n] + 1
                    nxt.append(c // 4)
        frontier = nxt
    return depth


def main():
    import bench
    import mrt
    import oracle_lib as O
    name = sys.argv[1]
    n_sample = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    cache = sys.argv[3] if len(sys.argv) > 3 else "/tmp/mrt_bvhcache"
    sname, w, h, kind, _ = bench.workload_spec(name)
    scene = mrt.Scene.synthetic(sname, 0, 1)
    import hashlib
    from mrt import _lib
    key = hashlib.sha1(open(_lib.HOST_LIB_PATH, "rb").read()).hexdigest()[:12]
    path = os.path.join(cache, f"{sname}-{key}.dat")
    bvh = mrt.Bvh.load(path) if os.path.exists(path) else mrt.Bvh.build(scene)
    nodes, woop, tri = bvh.buffers()
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, w, h)
    if kind != "primary":
        res, _, _ = O.trace(rays, nodes, woop, tri, threads=8)
        rays = mrt.ao_rays(rays, res, scene, ao if kind == "ao" else cam.far)
        rays = rays[rays[:, 7] > 0]
    rng = np.random.default_rng(0)
    rays = rays[rng.choice(len(rays), min(n_sample, len(rays)), replace=False)]
    depth = node_depths(nodes)
    nf = nodes.view(np.float32).reshape(-1, 16).astype(np.float64)
    ni = nodes.reshape(-1, 16)
    wf = woop.view(np.float32).reshape(-1, 4).astype(np.float64)
    wi = woop.reshape(-1, 4)
    visits = np.zeros(depth.max() + 1, np.int64)
    any_hit = kind == "ao"
    for r in rays.astype(np.float64):
        o, d, tmin, hit_t = r[0:3], r[4:7], r[3], r[7]
        idir = 1.0 / np.where(np.abs(d) > 2.0 ** -80, d, np.copysign(2.0 ** -80, d))
        ood = o * idir
        stack, node = [], 0
        done = False
        while not done:
            if node >= 0:
                n = node // 4
                visits[depth[n]] += 1
                b = nf[n]
                lo0 = np.array([b[0], b[2], b[8]]); hi0 = np.array([b[1], b[3], b[9]])
                lo1 = np.array([b[4], b[6], b[10]]); hi1 = np.array([b[5], b[7], b[11]])
                c0a, c0b = lo0 * idir - ood, hi0 * idir - ood
                c1a, c1b = lo1 * idir - ood, hi1 * idir - ood
                c0min = max(np.minimum(c0a, c0b).max(), tmin); c0max = min(np.maximum(c0a, c0b).min(), hit_t)
                c1min = max(np.minimum(c1a, c1b).max(), tmin); c1max = min(np.maximum(c1a, c1b).min(), hit_t)
                t0, t1 = c0max >= c0min, c1max >= c1min
                ch0, ch1 = int(ni[n, 12]), int(ni[n, 13])
                if t0 and t1:
                    near, far = (ch1, ch0) if c1min < c0min else (ch0, ch1)
                    stack.append(far)
                    node = near
                elif t0 or t1:
                    node = ch0 if t0 else ch1
                else:
                    if not stack:
                        break
                    node = stack.pop()
            else:
                a = ~node
                while wi[a, 0] != np.int32(-2147483648):
                    z, u, v = wf[a], wf[a + 1], wf[a + 2]
                    Oz = z[3] - o @ z[:3]
                    Dz = d @ z[:3]
                    t = Oz / Dz if Dz != 0 else np.inf
                    if tmin < t < hit_t:
                        uu = u[3] + o @ u[:3] + t * (d @ u[:3])
                        vv = v[3] + o @ v[:3] + t * (d @ v[:3])
                        if uu >= 0 and vv >= 0 and uu + vv <= 1:
                            hit_t = t
                            if any_hit:
                                done = True
                                break
                    a += 3
                if done or not stack:
                    break
                node = stack.pop()
    counts = np.bincount(depth[depth >= 0])
    cum_v = np.cumsum(visits) / visits.sum()
    cum_n = np.cumsum(counts)
    print(f"{name}: {len(rays)} rays, {visits.sum() / len(rays):.1f} node visits per ray, max depth {depth.max()}")
    print(" depth  visits<=d  nodes<=d  LDS KB")
    for dd in range(min(16, len(cum_v))):
        print(f"  {dd:4d}  {cum_v[dd]:8.3f}  {cum_n[dd]:8d}  {cum_n[dd] * 64 / 1024:7.1f}")


if __name__ == "__main__":
    main()
