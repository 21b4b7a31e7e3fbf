"""Wave-level (SIMT) model of the while-while traversal, for choosing the
node/leaf scheduling policy offline.

For one wave of 64 rays it replays the kernel's control flow with numpy masks
and counts wave iterations: node-loop iterations (every lane in the node loop
pays one when any lane visits a node) and triangle-loop iterations (one per
triangle slot of the longest leaf among the lanes in the leaf loop, plus the
terminator check). Arithmetic is plain float32 (not the kernel's FMA chains):
counts, not results, are the output.

Policies:
  K      leaves a lane may postpone before it stops visiting nodes (reference: 1,
         plus one more that ends its node walk)
  frac   the node loop breaks when at least this fraction of the lanes still in
         it hold a postponed leaf (reference: 1.0 = all of them)
  stream a lane walks all its postponed leaves in one triangle stream instead of
         one leaf per pass

Usage: python tools/simt_sim.py [workload] [n_waves]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

SENT = 0x76543210
TERM = np.int32(-2147483648)


class Wave:
    def __init__(self, nodes, woop, rays):
        self.nf = nodes.view(np.float32).reshape(-1, 16)
        self.ni = nodes.reshape(-1, 16)
        self.wf = woop.view(np.float32).reshape(-1, 4)
        self.wi = woop.reshape(-1, 4)
        n = len(rays)
        self.n = n
        o, d = rays[:, 0:3].astype(np.float32), rays[:, 4:7].astype(np.float32)
        self.o, self.d = o, d
        self.tmin = rays[:, 3].astype(np.float32)
        self.hitT = rays[:, 7].astype(np.float32).copy()
        eps = np.float32(2.0 ** -80)
        dd = np.where(np.abs(d) > eps, d, np.copysign(eps, d)).astype(np.float32)
        self.idir = (np.float32(1) / dd).astype(np.float32)
        self.ood = (o * self.idir).astype(np.float32)
        self.hit = np.full(n, -1, np.int64)

    def boxes(self, lanes, addr):
        nd = self.nf[addr // 4]
        idir, ood = self.idir[lanes], self.ood[lanes]

        def span(lo_x, hi_x, lo_y, hi_y, lo_z, hi_z):
            ax = lo_x * idir[:, 0] - ood[:, 0]
            bx = hi_x * idir[:, 0] - ood[:, 0]
            ay = lo_y * idir[:, 1] - ood[:, 1]
            by = hi_y * idir[:, 1] - ood[:, 1]
            az = lo_z * idir[:, 2] - ood[:, 2]
            bz = hi_z * idir[:, 2] - ood[:, 2]
            tmn = np.maximum.reduce([np.minimum(ax, bx), np.minimum(ay, by), np.minimum(az, bz), self.tmin[lanes]])
            tmx = np.minimum.reduce([np.maximum(ax, bx), np.maximum(ay, by), np.maximum(az, bz), self.hitT[lanes]])
            return tmn, tmx
        c0min, c0max = span(nd[:, 0], nd[:, 1], nd[:, 2], nd[:, 3], nd[:, 8], nd[:, 9])
        c1min, c1max = span(nd[:, 4], nd[:, 5], nd[:, 6], nd[:, 7], nd[:, 10], nd[:, 11])
        ci = self.ni[addr // 4]
        return c0max >= c0min, c1max >= c1min, c1min < c0min, ci[:, 12].astype(np.int64), ci[:, 13].astype(np.int64)

    def leaf_tris(self, lane, leaf):
        """Triangles of a leaf tested in order (updates hitT); returns slots walked."""
        a = ~leaf
        k = 0
        while self.wi[a, 0] != TERM:
            v0, v1, v2 = self.wf[a], self.wf[a + 1], self.wf[a + 2]
            o, d = self.o[lane], self.d[lane]
            Oz = v0[3] - o @ v0[:3]
            Dz = d @ v0[:3]
            t = Oz / Dz if Dz != 0 else np.inf
            if self.tmin[lane] < t < self.hitT[lane]:
                u = (v1[3] + o @ v1[:3]) + t * (d @ v1[:3])
                if u >= 0:
                    v = (v2[3] + o @ v2[:3]) + t * (d @ v2[:3])
                    if v >= 0 and u + v <= 1:
                        self.hitT[lane] = t
                        self.hit[lane] = a
            a += 3
            k += 1
        return k + 1   # + the terminator check


def simulate(nodes, woop, rays, K=1, frac=1.0, stream=False):
    w = Wave(nodes, woop, rays)
    n = w.n
    node = np.zeros(n, np.int64)
    stack = [[SENT] for _ in range(n)]
    queue = [[] for _ in range(n)]
    it_node = it_tri = passes = 0

    def inner(x):
        return (x >= 0) & (x != SENT)

    while (node != SENT).any() or any(queue):
        # ---- node phase
        while True:
            act = np.nonzero(inner(node))[0]
            if len(act) == 0:
                break
            it_node += 1
            t0, t1, swp, c0, c1 = w.boxes(act, node[act])
            for j, L in enumerate(act):
                if not t0[j] and not t1[j]:
                    node[L] = stack[L].pop()
                else:
                    nx = c0[j] if t0[j] else c1[j]
                    far = c1[j]
                    if t0[j] and t1[j]:
                        if swp[j]:
                            nx, far = far, nx
                        stack[L].append(far)
                    node[L] = nx
                if node[L] < 0 and len(queue[L]) < K:
                    queue[L].append(node[L])
                    node[L] = stack[L].pop()
            have = np.array([len(queue[L]) > 0 for L in act])
            if have.mean() >= frac:
                break
        # ---- leaf phase
        while True:
            lanes = [L for L in range(n) if queue[L]]
            if not lanes:
                break
            passes += 1
            cost = []
            for L in lanes:
                c = 0
                todo = queue[L] if stream else queue[L][:1]
                for leaf in todo:
                    c += w.leaf_tris(L, leaf)
                queue[L] = [] if stream else queue[L][1:]
                cost.append(c)
            it_tri += max(cost)
            # reference: a leaf popped meanwhile (node < 0) is processed too
            for L in lanes:
                if not queue[L] and node[L] < 0:
                    queue[L].append(node[L])
                    node[L] = stack[L].pop()
    return it_node, it_tri, passes, w.hit, w.hitT


def simulate_ifif(nodes, woop, rays):
    """'if-if' scheduling: every iteration each lane does one node visit or one
    triangle slot; the wave pays a node pass and/or a triangle pass."""
    w = Wave(nodes, woop, rays)
    n = w.n
    node = np.zeros(n, np.int64)
    stack = [[SENT] for _ in range(n)]
    leafpos = np.full(n, -1, np.int64)   # current woop slot when in a leaf
    it_node = it_tri = 0

    def inner(x):
        return (x >= 0) & (x != SENT)
    while True:
        in_leaf = leafpos >= 0
        act = np.nonzero(inner(node) & ~in_leaf)[0]
        tri_l = np.nonzero(in_leaf)[0]
        if len(act) == 0 and len(tri_l) == 0:
            break
        if len(act):
            it_node += 1
            t0, t1, swp, c0, c1 = w.boxes(act, node[act])
            for j, L in enumerate(act):
                if not t0[j] and not t1[j]:
                    node[L] = stack[L].pop()
                else:
                    nx = c0[j] if t0[j] else c1[j]
                    far = c1[j]
                    if t0[j] and t1[j]:
                        if swp[j]:
                            nx, far = far, nx
                        stack[L].append(far)
                    node[L] = nx
                if node[L] < 0:
                    leafpos[L] = ~node[L]
                    node[L] = stack[L].pop()
        if len(tri_l):
            it_tri += 1
            for L in tri_l:
                a = leafpos[L]
                if w.wi[a, 0] == TERM:
                    leafpos[L] = -1
                else:
                    # one triangle (reuse leaf_tris on a one-triangle view is awkward: inline)
                    v0, v1, v2 = w.wf[a], w.wf[a + 1], w.wf[a + 2]
                    o, d = w.o[L], w.d[L]
                    Dz = d @ v0[:3]
                    t = (v0[3] - o @ v0[:3]) / Dz if Dz != 0 else np.inf
                    if w.tmin[L] < t < w.hitT[L]:
                        u = (v1[3] + o @ v1[:3]) + t * (d @ v1[:3])
                        v = (v2[3] + o @ v2[:3]) + t * (d @ v2[:3])
                        if u >= 0 and v >= 0 and u + v <= 1:
                            w.hitT[L] = t
                            w.hit[L] = a
                    leafpos[L] = a + 3
    return it_node, it_tri


def main():
    import bench
    import oracle_lib as O
    wl = sys.argv[1] if len(sys.argv) > 1 else "bunny-primary-1024x768"
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    scene_name = bench.workload_spec(wl)[0]
    scene, bufs, _, _ = bench.bvh_for(scene_name, 1, 0)
    import mrt
    _, wdt, hgt = bench.workload_spec(wl)[:3]
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, wdt, hgt)
    nodes, woop, tri = bufs
    res, st, _ = O.trace(rays, nodes, woop, tri, stats=True, threads=8)
    steps = st[:, 0] + st[:, 1] + st[:, 2]
    waves = steps[: len(steps) // 64 * 64].reshape(-1, 64)
    order = np.argsort(-waves.max(1))
    pick = list(order[:nw]) + list(np.random.default_rng(0).choice(len(waves), nw, replace=False))
    policies = [dict(K=1), dict(K=2), dict(K=2, stream=True), dict(K=4, stream=True), dict(K=1, frac=0.75),
                dict(K=2, stream=True, frac=0.75), dict(K=8, stream=True)]
    print(f"{wl}: {len(pick)} waves ({nw} slowest by max steps, {nw} random); per wave: node iters / tri iters / passes")
    tot = {i: np.zeros(3) for i in range(len(policies))}
    for wi in pick:
        r = rays[wi * 64:(wi + 1) * 64]
        line = f"  wave {wi:6d} max {waves[wi].max():3d} mean {waves[wi].mean():6.1f} |"
        for i, p in enumerate(policies):
            a, b, c, hit, _ = simulate(nodes, woop, r, **p)
            tot[i] += (a, b, c)
            line += f" {a:4d}/{b:4d}/{c:3d}"
        print(line, flush=True)
    ifif = np.zeros(2)
    for wi in pick:
        a, b = simulate_ifif(nodes, woop, rays[wi * 64:(wi + 1) * 64])
        ifif += (a, b)
        print(f"  if-if wave {wi:6d}: node passes {a:4d} tri passes {b:4d}", flush=True)
    print(f"  if-if total: node {ifif[0]:.0f} tri {ifif[1]:.0f}")
    for i, p in enumerate(policies):
        print(f"  {str(p):45s} node {tot[i][0]:8.0f} tri {tot[i][1]:8.0f} passes {tot[i][2]:6.0f} "
              f"sum {tot[i][0] + tot[i][1]:8.0f}")


if __name__ == "__main__":
    main()
