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
