"""Offline estimate (CPU): how many dependent node fetches would a 4-wide BVH
collapsed from the bound Compact2 tree take per ray, against the binary tree?

Collapse: each wide node starts from a binary inner node's two children and
repeatedly replaces its inner child of largest surface area by that child's two
children until it holds 4 (leaves stay leaves). Traversal replay (float64, counts
only): binary = near first / far pushed / leaves tested in pop order; wide = the
hit children sorted by entry distance, nearest taken, the rest pushed farthest
first, leaves tested as they come.

  python tools/wide_sim.py sponza-diffuse-640x480 [n_rays]
"""
import glob
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

TERM = np.int32(-2147483648)


class Tree:
    def __init__(self, nodes, woop):
        self.nf = nodes.view(np.float32).reshape(-1, 16).astype(np.float64)
        self.ni = nodes.reshape(-1, 16)
        self.wf = woop.view(np.float32).reshape(-1, 4).astype(np.float64)
        self.wi = woop.reshape(-1, 4)

    def children(self, n):
        """[(child ref, lo[3], hi[3])] of binary node n (float4 index // 4)."""
        b = self.nf[n]
        return [(int(self.ni[n, 12]), np.array([b[0], b[2], b[8]]), np.array([b[1], b[3], b[9]])),
                (int(self.ni[n, 13]), np.array([b[4], b[6], b[10]]), np.array([b[5], b[7], b[11]]))]

    def wide(self, n, width):
        ch = self.children(n)
        while len(ch) < width:
            inner = [i for i, c in enumerate(ch) if c[0] >= 0]
            if not inner:
                break
            area = [np.prod(np.maximum(ch[i][2] - ch[i][1], 0)[[0, 1, 2]]) for i in inner]
            ext = [ch[i][2] - ch[i][1] for i in inner]
            sa = [e[0] * e[1] + e[1] * e[2] + e[2] * e[0] for e in ext]
            k = inner[int(np.argmax(sa))]
            ref = ch[k][0]
            ch = ch[:k] + self.children(ref // 4) + ch[k + 1:]
        return ch

    def leaf(self, ref, o, d, tmin, hit_t, counts):
        a = ~ref
        counts["leaves"] += 1
        while self.wi[a, 0] != TERM:
            counts["tris"] += 1
            z, u, v = self.wf[a], self.wf[a + 1], self.wf[a + 2]
            Dz = d @ z[:3]
            t = (z[3] - o @ z[:3]) / Dz if Dz != 0 else np.inf
            if tmin < t < hit_t:
                uu = u[3] + o @ u[:3] + t * (d @ u[:3])
                vv = v[3] + o @ v[:3] + t * (d @ v[:3])
                if uu >= 0 and vv >= 0 and uu + vv <= 1:
                    hit_t = t
            a += 3
        return hit_t


def slab(lo, hi, idir, ood, tmin, hit_t):
    a, b = lo * idir - ood, hi * idir - ood
    cmin = max(np.minimum(a, b).max(), tmin)
    cmax = min(np.maximum(a, b).min(), hit_t)
    return cmax >= cmin, cmin


def trace(tree, r, width):
    o, d, tmin, hit_t = r[0:3], r[4:7], r[3], r[7]
    idir = 1.0 / np.where(np.abs(d) > 2.0 ** -80, d, np.copysign(2.0 ** -80, d))
    ood = o * idir
    counts = {"nodes": 0, "tris": 0, "leaves": 0}
    stack = [0]
    cache = {}
    while stack:
        ref = stack.pop()
        while ref >= 0:
            counts["nodes"] += 1
            n = ref // 4
            if width == 2:
                ch = tree.children(n)
            else:
                if n not in cache:
                    cache[n] = tree.wide(n, width)
                ch = cache[n]
            hits = []
            for c, lo, hi in ch:
                ok, t = slab(lo, hi, idir, ood, tmin, hit_t)
                if ok:
                    hits.append((t, c))
            hits.sort(key=lambda x: x[0])
            if not hits:
                ref = None
                break
            for t, c in reversed(hits[1:]):
                stack.append(c)
            ref = hits[0][1]
        if ref is not None and ref < 0:
            hit_t = tree.leaf(ref, o, d, tmin, hit_t, counts)
    return counts, hit_t


def main():
    import bench
    import mrt
    import oracle_lib as O
    name = sys.argv[1]
    n_sample = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    sname, w, h, kind, _ = bench.workload_spec(name)
    scene = mrt.Scene.synthetic(sname, 0, 1)
    dats = glob.glob(f"/tmp/mrt_bvhcache/{sname}-*.dat")
    bvh = mrt.Bvh.load(dats[0]) if dats else mrt.Bvh.build(scene)
    nodes, woop, tri = bvh.buffers()
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, w, h)
    if kind != "primary":
        res, _, _ = O.trace(rays, nodes, woop, tri, threads=8)
        rays = mrt.ao_rays(rays, res, scene, ao if kind == "ao" else cam.far)
    rays = rays[rays[:, 7] > 0]
    rng = np.random.default_rng(0)
    rays = rays[rng.choice(len(rays), min(n_sample, len(rays)), replace=False)].astype(np.float64)
    tree = Tree(nodes, woop)
    for width in (2, 4, 8):
        tot = {"nodes": 0, "tris": 0, "leaves": 0}
        ts = []
        for r in rays:
            c, t = trace(tree, r, width)
            ts.append(t)
            for k in tot:
                tot[k] += c[k]
        n = len(rays)
        print(f"{name} width {width}: nodes/ray {tot['nodes'] / n:6.2f}  tris/ray {tot['tris'] / n:6.2f}  "
              f"leaves/ray {tot['leaves'] / n:5.2f}  (closest-t checksum {np.sum(np.minimum(ts, 1e30)):.6f})",
              flush=True)


if __name__ == "__main__":
    main()
