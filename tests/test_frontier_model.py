"""The frontier tail's traversal order (trace_kernel.hip frontier_tail), modelled on the
CPU by tools/frontier_sim.py: expanding up to F pending entries of a ray's list per step
(children back in depth-first order, each step's triangles tested against the hitT at the
start of the step) finds the same closest hit as the depth-first walk (F = 1), in fewer
steps. The GPU kernel's own parity against the oracle is tests/test_gpu_parity.py
(test_frontier_tail_group_widths and every speculative-mode test); this pins the model
the design was derived from."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import mrt  # noqa: E402
import oracle_lib as O  # noqa: E402
from frontier_sim import frontier  # noqa: E402
from wide_sim import Tree  # noqa: E402


def test_frontier_widths_keep_the_closest_hit():
    scene = mrt.Scene.synthetic("mori", 0, 1)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    base, _ = mrt.primary_rays(cam, 48, 36)
    prim, _, _ = O.trace(base, nodes, woop, tri)
    hits = np.nonzero(prim[:, 0] >= 0)[0]
    rng = np.random.default_rng(3)
    n = 120
    pick = rng.choice(hits, n)
    t = prim[pick, 1].view(np.float32)
    p = base[pick, 0:3] + base[pick, 4:7] * t[:, None]
    extent = float(np.ptp(p, axis=0).max())
    rays = np.zeros((n, 8), np.float64)
    rays[:, 0:3] = p + rng.normal(0.0, 0.05 * extent, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = np.where(rng.random(n) < 0.3, np.inf, rng.uniform(0.05, 2.0, n) * extent)
    tree = Tree(nodes, woop)
    cache = {}
    steps = {}
    for F in (1, 2, 4, 16):
        out = [frontier(tree, r, F, cache) for r in rays]
        steps[F] = np.array([o[0] for o in out])
        ts = np.array([o[4] for o in out])
        if F == 1:
            t1 = ts
        else:
            assert np.array_equal(ts, t1), f"F={F}: closest t differs on {(ts != t1).sum()} rays"
    # wider frontiers never need more steps than the depth-first walk, and fewer overall
    assert (steps[16] <= steps[1]).all()
    assert steps[16].sum() < steps[4].sum() < steps[1].sum()


def _tail_list_peak(children, G, stack_cap, bound):
    """The frontier tail's list bookkeeping (trace_kernel.hip frontier_tail) for one ray
    whose every child box is hit and no triangle: window m <= G, home stack h; per step
    nproc = min(m, F, max(1, (cap - bound - L) // 3)) entries expanded (a node becomes its
    children, a leaf of <= 4 triangles ends), entries past the window pushed home, the
    window refilled to F from home. Returns the largest list L = m + h reached."""
    F = G // 4
    cap = stack_cap - 1 + G
    window, home = [0], []
    peak = 1
    while window or home:
        L = len(window) + len(home)
        nproc = min(len(window), F, max(1, (cap - bound - L) // 3))
        out = []
        for e in window[:nproc]:
            out += children.get(e, [])
        window = out + window[nproc:]
        if len(window) > G:
            home += reversed(window[G:])   # deepest first: home[-1] is the next entry after the window
            window = window[:G]
        peak = max(peak, len(window) + len(home))
        while len(window) < F and home:
            window.append(home.pop())
    return peak


def test_frontier_tail_list_fits_the_stack():
    """a frontier expanding up to F entries per step grows a ray's list by
    three per node, past the depth-first walk's worst case. On a complete 4-ary tree whose
    every box a ray hits (kat.scene_complete), the old rule (headroom only for the step
    itself) overflows the 64-entry stack at F = 16; the kernel's rule (wide steps only while
    the tree's depth-first bound still fits behind them) never passes the capacity."""
    import ctypes as C
    import kat
    from mrt import _lib
    (nodes, woop, _), _, _ = kat.scene_complete(12)
    lib = _lib.trace_lib()
    size = C.c_int64(0)
    assert lib.mrt_derive_wide_nodes(nodes.ctypes.data, nodes.nbytes, woop.ctypes.data, woop.nbytes, 1, None, 0,
                                     C.byref(size)) == 0
    wide = np.zeros(size.value // 4, np.uint32)
    assert lib.mrt_derive_wide_nodes(nodes.ctypes.data, nodes.nbytes, woop.ctypes.data, woop.nbytes, 1,
                                     wide.ctypes.data, wide.nbytes, C.byref(size)) == 0
    refs = wide.reshape(-1, 32)[:, 24:28].view(np.int32)
    children = {i: [int(r) // 8 if r >= 0 else -1 - len(refs) for r in row if r != kat.SENTINEL]
                for i, row in enumerate(refs)}
    # the tree's depth-first bound (wide_bvh.cpp wide_stack_bound): ancestors' pushes plus its own
    def dfs_bound(i, depth):
        below = depth + len(children[i]) - 1
        return max([below] + [dfs_bound(c, below) for c in children[i] if c in children])
    bound = dfs_bound(0, 0)
    # a complete 4-ary tree of six levels, three pushes per level
    assert len(refs) == (4 ** 6 - 1) // 3 and bound == 18
    for G in (4, 8, 16, 32, 64):
        assert _tail_list_peak(children, G, 64, bound) <= 64 - 1 + G
    assert _tail_list_peak(children, 64, 64, 0) > 64 - 1 + 64   # the old rule overflows
