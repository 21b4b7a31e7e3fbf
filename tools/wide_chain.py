"""CPU model: dependent steps per ray (node visits + leaves) of the 4-wide traversal
against an 8-wide tree collapsed the same way (tools/wide_sim.py's collapse and replay, float64,
closest-hit order — an upper bound for any-hit rays), with the distribution's tail (p90/p99/max:
a short any-hit frame is its slowest rays' chains) and the 16-B lane loads per ray the node fetches
cost (7 per 4-wide node, 14 per 8-wide node: two 128-B lines).
  python tools/wide_chain.py mori-ao-640x480 [n_rays]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tools", "", "gpu-ray-tracing_amd", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import wide_sim as W  # noqa: E402


def main():
    import bench
    import mrt
    import oracle_lib as O
    name = sys.argv[1]
    n_sample = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    sname, w, h, kind, _ = bench.workload_spec(name)
    scene = mrt.Scene.synthetic(sname, 0, 1)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, w, h)
    if kind != "primary":
        res, _, _ = O.trace(rays, nodes, woop, tri, threads=8)
        rays = mrt.ao_rays(rays, res, scene, ao if kind == "ao" else cam.far)
    rays = rays[rays[:, 7] > 0]
    rng = np.random.default_rng(0)
    rays = rays[rng.choice(len(rays), min(n_sample, len(rays)), replace=False)].astype(np.float64)
    tree = W.Tree(nodes, woop)
    for width, loads in ((4, 7), (8, 14)):
        steps, nload = [], []
        for r in rays:
            c, _ = W.trace(tree, r, width)
            steps.append(c["nodes"] + c["leaves"])
            nload.append(c["nodes"] * loads + c["tris"] * 3)
        s, ld = np.array(steps), np.array(nload)
        print(f"{name} width {width}: dependent steps/ray mean {s.mean():.2f} p90 {np.percentile(s, 90):.1f} "
              f"p99 {np.percentile(s, 99):.1f} max {s.max()}; 16-B lane loads/ray {ld.mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
