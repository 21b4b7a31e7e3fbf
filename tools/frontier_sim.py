"""Offline estimate (CPU): dependent memory round trips per ray when a ray's
traversal processes up to F pending entries per step (a frontier of the ray's
own stack: the current entry and the F-1 entries below it, all fetched in one
round trip, children pushed back in depth-first order), against F = 1 (one
4-wide node or one chunk of four leaf triangles per round trip, the cooperative
tail's step). Runs over the rays the oracle counts as most expensive.

  python tools/frontier_sim.py bunny-primary-640x480 [n_longest] [F ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from wide_sim import Tree, slab, TERM  # noqa: E402


def leaf_tris(tree, ref):
    a = ~ref
    out = []
    while tree.wi[a, 0] != TERM:
        out.append(a)
        a += 3
    return out


def tri_t(tree, a, o, d, tmin, hit_t):
    z, u, v = tree.wf[a], tree.wf[a + 1], tree.wf[a + 2]
    Dz = d @ z[:3]
    t = (z[3] - o @ z[:3]) / Dz if Dz != 0 else np.inf
    if tmin < t < hit_t:
        uu = u[3] + o @ u[:3] + t * (d @ u[:3])
        vv = v[3] + o @ v[:3] + t * (d @ v[:3])
        if uu >= 0 and vv >= 0 and uu + vv <= 1:
            return t
    return None


def frontier(tree, r, F, cache):
    """Round trips of the frontier traversal with width F (F = 1: depth first)."""
    o, d, tmin, hit_t = r[0:3], r[4:7], r[3], r[7]
    idir = 1.0 / np.where(np.abs(d) > 2.0 ** -80, d, np.copysign(2.0 ** -80, d))
    ood = o * idir
    # pending entries in depth-first order, next first: ("n", ref) or ("l", [tri addrs])
    pend = [("n", 0)]
    steps = nodes = tris = 0
    maxlen = 1
    while pend:
        steps += 1
        work, pend = pend[:F], pend[F:]
        out = []
        best = hit_t
        for kind, x in work:
            if kind == "n":
                nodes += 1
                n = x // 4
                if n not in cache:
                    cache[n] = tree.wide(n, 4)
                hits = []
                for c, lo, hi in cache[n]:
                    ok, t = slab(lo, hi, idir, ood, tmin, hit_t)
                    if ok:
                        hits.append((t, c))
                hits.sort(key=lambda h: h[0])
                for _, c in hits:
                    out.append(("n", c) if c >= 0 else ("l", leaf_tris(tree, c)))
            else:
                chunk, rest = x[:4], x[4:]
                tris += len(chunk)
                for a in chunk:
                    t = tri_t(tree, a, o, d, tmin, hit_t)
                    if t is not None and t < best:
                        best = t
                if rest:
                    out.append(("l", rest))
        hit_t = best
        pend = [e for e in out if not (e[0] == "l" and not e[1])] + pend
        maxlen = max(maxlen, len(pend))
    return steps, nodes, tris, maxlen, hit_t


def main():
    import bench
    import mrt
    import oracle_lib as O
    name = sys.argv[1]
    n_long = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    widths = [int(x) for x in sys.argv[3:]] or [1, 2, 4, 8, 16]
    sname, w, h, kind, _ = bench.workload_spec(name)
    scene = mrt.Scene.synthetic(sname, 0, 1)
    bvh = mrt.Bvh.build(scene)
    nodes, woop, tri = bvh.buffers()
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, w, h)
    if kind != "primary":
        res, _, _ = O.trace(rays, nodes, woop, tri, threads=8)
        rays = mrt.ao_rays(rays, res, scene, ao if kind == "ao" else cam.far)
    rays = rays[rays[:, 7] > 0]
    _, cnt, _ = O.trace(rays, nodes, woop, tri, threads=8, stats=True)
    cost = cnt[:, 0] + cnt[:, 1] + cnt[:, 2]
    order = np.argsort(cost)[::-1]
    print(f"{name}: {len(rays)} rays; binary steps (nodes+tris+leaves) mean {cost.mean():.1f}, "
          f"p99 {np.percentile(cost, 99):.0f}, p99.99 {np.percentile(cost, 99.99):.0f}, max {cost.max()}", flush=True)
    sample = rays[order[:n_long]].astype(np.float64)
    tree = Tree(nodes, woop)
    cache = {}
    base = None
    for F in widths:
        st, nd, tr, ml, ts = [], [], [], [], []
        for r in sample:
            s, n_, t_, m, hit = frontier(tree, r, F, cache)
            st.append(s); nd.append(n_); tr.append(t_); ml.append(m); ts.append(hit)
        st = np.array(st)
        if base is None:
            base = st
        print(f"  F={F:2d}: round trips mean {st.mean():6.1f} max {st.max():4d} (x{np.mean(base / st):.2f} of F=1, "
              f"max ratio {base.max() / st.max():.2f}); nodes {np.mean(nd):6.1f} tris {np.mean(tr):6.1f}; "
              f"pending max {max(ml)}; t checksum {np.sum(np.minimum(ts, 1e30)):.6f}", flush=True)


if __name__ == "__main__":
    main()
