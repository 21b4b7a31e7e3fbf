"""Hand-built Compact2 BVHs with known answers (shared by the CPU oracle tests
and the GPU parity tests).

Every triangle here is an axis-aligned right triangle with power-of-two
extents, so its Woop rows (the inverse of [v0-v2, v1-v2, n, v2],
reference CudaBVH.cc:361-380) are exact in float32 and every expected t below
is exactly representable: the answers are computed by hand, not by the code
under test.
"""
from __future__ import annotations

import numpy as np

SENTINEL = 0x76543210
NEG_ZERO = np.int32(-2147483648)   # 0x80000000: the -0.0 terminator


def f2i(x: float) -> int:
    return int(np.float32(x).view(np.int32))


def woop_rows(v0, v1, v2):
    """Exact Woop rows (Z, U, V) via float64 inverse (exact for these triangles)."""
    v0, v1, v2 = (np.asarray(v, np.float64) for v in (v0, v1, v2))
    e0, e1 = v0 - v2, v1 - v2
    n = np.cross(e0, e1)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = e0, e1, n, v2
    inv = np.linalg.inv(m)
    z = np.array([inv[2, 0], inv[2, 1], inv[2, 2], -inv[2, 3]])
    rows = np.stack([z, inv[0], inv[1]]).astype(np.float32)
    assert np.all(rows.astype(np.float64) == np.stack([z, inv[0], inv[1]])), "triangle is not exactly representable"
    rows[0, 0] = rows[0, 0] + np.float32(0.0)   # -0.0 -> +0.0 in Z.x (CudaBVH.cc:316-317)
    return rows


class Compact2Builder:
    """Tiny explicit Compact2 writer: inner nodes are (box0, box1, child0, child1)."""

    def __init__(self):
        self.nodes = []      # list of 16-int records
        self.woop = []       # list of 4-float rows
        self.tri_index = []

    def leaf(self, tris):
        """tris: list of (id, v0, v1, v2). Returns the ~offset child reference."""
        ref = ~len(self.woop)
        for tid, v0, v1, v2 in tris:
            for r in woop_rows(v0, v1, v2):
                self.woop.append(r.view(np.int32))
            self.tri_index += [tid, 0, 0]
        self.woop.append(np.full(4, NEG_ZERO, np.int32))
        self.tri_index.append(0)
        return ref

    def reserve_inner(self):
        idx = len(self.nodes)
        self.nodes.append(None)
        return idx

    def set_inner(self, idx, box0, box1, c0, c1):
        (l0, h0), (l1, h1) = box0, box1
        f = np.array([l0[0], h0[0], l0[1], h0[1], l1[0], h1[0], l1[1], h1[1], l0[2], h0[2], l1[2], h1[2]],
                     np.float32).view(np.int32)
        self.nodes[idx] = np.concatenate([f, np.array([c0, c1, 0, 0], np.int32)])
        return idx * 4   # float4 index

    def buffers(self):
        nodes = np.concatenate(self.nodes).astype(np.int32)
        woop = np.concatenate(self.woop).astype(np.int32)
        return nodes, woop, np.array(self.tri_index, np.int32)


def ray(o, d, tmin=0.0, tmax=100.0):
    return np.array([o[0], o[1], o[2], tmin, d[0], d[1], d[2], tmax], np.float32)


def scene_two_floors():
    """Root with two leaves.
    leaf A (child 0): tri 7 = unit right triangle in the plane z = 0,
                      tri 3 = the same footprint at z = -2.
    leaf B (child 1): tri 5 = right triangle of leg 2 in the plane z = -1, shifted to x in [2, 4].
    """
    b = Compact2Builder()
    root = b.reserve_inner()
    A = b.leaf([(7, (0, 0, 0), (1, 0, 0), (0, 1, 0)),
                (3, (0, 0, -2), (1, 0, -2), (0, 1, -2))])
    B = b.leaf([(5, (2, 0, -1), (4, 0, -1), (2, 2, -1))])
    b.set_inner(root, ((0, 0, -2), (1, 1, 0)), ((2, 0, -1), (4, 2, -1)), A, B)
    return b.buffers()


def scene_deep():
    """Inner root -> inner child -> two leaves, plus a leaf sibling:
    exercises push/pop ordering. Triangles are stacked along -z at x,y in [0,1]."""
    b = Compact2Builder()
    root = b.reserve_inner()
    inner = b.reserve_inner()
    near = b.leaf([(10, (0, 0, -1), (1, 0, -1), (0, 1, -1))])
    far = b.leaf([(11, (0, 0, -3), (1, 0, -3), (0, 1, -3))])
    side = b.leaf([(12, (0, 0, -2), (1, 0, -2), (0, 1, -2))])
    cinner = b.set_inner(inner, ((0, 0, -1), (1, 1, -1)), ((0, 0, -3), (1, 1, -3)), near, far)
    b.set_inner(root, ((0, 0, -3), (1, 1, -1)), ((0, 0, -2), (1, 1, -2)), cinner, side)
    return b.buffers()


# (name, scene builder, rays, any_hit, expected [(id, t)]) — hand-derived.
def cases():
    out = []
    two = scene_two_floors
    down = (0, 0, -1)
    out.append(("closest: near floor", two, [ray((0.25, 0.25, 1), down)], False, [(7, 1.0)]))
    out.append(("closest: far leaf only", two, [ray((2.5, 0.5, 1), down)], False, [(5, 2.0)]))
    out.append(("miss keeps tmax", two, [ray((8, 8, 1), down, tmax=50.0)], False, [(-1, 50.0)]))
    out.append(("tmin skips the near floor", two, [ray((0.25, 0.25, 1), down, tmin=1.5)], False, [(3, 3.0)]))
    out.append(("tmax cuts before the far floor", two, [ray((0.25, 0.25, 1), down, tmin=1.5, tmax=2.5)], False,
                [(-1, 2.5)]))
    out.append(("tmin == tmax never hits", two, [ray((0.25, 0.25, 1), down, tmin=1.0, tmax=1.0)], False,
                [(-1, 1.0)]))
    out.append(("degenerate AO ray tmax=-1", two, [ray((0.25, 0.25, 1), down, tmin=0.0, tmax=-1.0)], True,
                [(-1, -1.0)]))
    out.append(("upward ray from below", two, [ray((0.25, 0.25, -4), (0, 0, 1))], False, [(3, 2.0)]))
    out.append(("any-hit stops at the first tested (tri 7 before 3)", two, [ray((0.25, 0.25, 1), down)], True,
                [(7, 1.0)]))
    out.append(("any-hit from below: first tested in the leaf is still 7", two,
                [ray((0.25, 0.25, -4), (0, 0, 1))], True, [(7, 4.0)]))
    out.append(("outside the triangle (u+v>1)", two, [ray((0.75, 0.75, 1), down)], False, [(-1, 100.0)]))
    out.append(("parallel ray misses (2^-80 clamp)", two, [ray((-1, 0.25, 0.0 + 0.5), (1, 0, 0))], False,
                [(-1, 100.0)]))
    deep = scene_deep
    out.append(("deep: nearest of three stacked", deep, [ray((0.25, 0.25, 0), down)], False, [(10, 1.0)]))
    out.append(("deep: tmin=1.5 -> middle (other subtree)", deep, [ray((0.25, 0.25, 0), down, tmin=1.5)], False,
                [(12, 2.0)]))
    out.append(("deep: tmin=2.5 -> farthest", deep, [ray((0.25, 0.25, 0), down, tmin=2.5)], False, [(11, 3.0)]))
    out.append(("deep: from below, nearest is 11", deep, [ray((0.25, 0.25, -5), (0, 0, 1))], False, [(11, 2.0)]))
    return out


def scene_comb(depth):
    """A comb of `depth` inner nodes for a stack-depth test (reference STACK_SIZE 64,
    kepler_dynamic_fetch.cu:47). Inner node k (k < depth-1) has child 0 = inner
    node k+1 (its box entered at t = k + 1.5) and child 1 = leaf k (entered at
    t = k + 2), so a ray down -z through (0.25, 0.25) goes near and pushes one
    leaf per level: `depth` pushes before the first pop. Leaf k holds triangle k
    in the plane z = -(k+1) (t = k + 2); the last inner node holds leaves
    depth-1 and depth. Closest hit: triangle 0 at t = 2 (hand answer).
    Returns (buffers, ray, (id, t))."""
    b = Compact2Builder()
    inner = [b.reserve_inner() for _ in range(depth)]
    bottom = -(depth + 2.0)

    def tri_leaf(k):
        z = -(k + 1.0)
        return b.leaf([(k, (0, 0, z), (1, 0, z), (0, 1, z))])

    def leaf_box(k):
        return ((0, 0, -(k + 1.0)), (1, 1, -(k + 1.0)))

    for k in range(depth - 1, -1, -1):
        if k == depth - 1:
            b.set_inner(inner[k], leaf_box(k), leaf_box(k + 1), tri_leaf(k), tri_leaf(k + 1))
        else:
            child_box = ((0, 0, bottom), (1, 1, -(k + 1.0) + 0.5))
            b.set_inner(inner[k], child_box, leaf_box(k), inner[k + 1] * 4, tri_leaf(k))
    return b.buffers(), ray((0.25, 0.25, 1), (0, 0, -1), tmax=1000.0), (0, 2.0)


def scene_complete(depth, hit_last=False):
    """A complete binary tree of `depth` inner levels whose nested boxes
    ([0,2]^2 x [0, 1 - level/64], so a level's boxes are larger than the next
    level's) all hold (0.5, 0.5), one triangle per leaf (2^depth leaves): the
    4-wide derivation collapses it level pair by level pair into a complete 4-ary
    tree of depth/2 levels, every child of every node hit by a ray down -z through
    (0.5, 0.5). Each leaf's
    triangle is a small one in the corner (missed), except, with hit_last, the
    last leaf's: a leg-2 triangle in the plane z = 0.5 (t = 1.5 from z = 2).
    ADVICE r3: a frontier that expands many entries per step must still fit such a
    ray's list in the stack. Returns (buffers, ray, (id, t))."""
    b = Compact2Builder()
    leaves = 1 << depth
    counter = [0]

    def leaf():
        k = counter[0]
        counter[0] += 1
        z = 0.25 + 0.5 * (k % 2)
        if hit_last and k == leaves - 1:
            return b.leaf([(k, (0, 0, 0.5), (2, 0, 0.5), (0, 2, 0.5))])
        return b.leaf([(k, (0, 0, z), (0.125, 0, z), (0, 0.125, z))])

    def build(level):
        idx = b.reserve_inner()
        c = [build(level + 1) if level + 1 < depth else leaf() for _ in range(2)]
        box = ((0, 0, 0), (2, 2, 1.0 - (level + 1) / 64.0))
        return b.set_inner(idx, box, box, c[0], c[1])

    build(0)
    expect = (leaves - 1, 1.5) if hit_last else (-1, 1000.0)
    return b.buffers(), ray((0.5, 0.5, 2), (0, 0, -1), tmax=1000.0), expect
