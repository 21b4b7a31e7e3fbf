"""Regenerates the golden fixtures in this directory (run from the repo root:
`python tests/golden/make_golden.py`). Each .npz holds one Compact2 BVH built
by this repo's SBVH builder, a ray batch from this repo's ray generators, and
the CPU oracle's results + per-ray counters. They pin the oracle and the
builder against regressions and give the GPU tests fixed inputs; they are NOT
reference-executed outputs (the reference cannot run here, see oracle/)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import mrt  # noqa: E402
import oracle_lib as O  # noqa: E402

CASES = [
    # file, scene, param, seed, width, height, ray type
    ("golden_mori_primary_64x48.npz", "mori", 0, 1, 64, 48, "primary"),
    ("golden_random1500_ao_48x32.npz", "random", 1500, 7, 48, 32, "ao"),
    ("golden_random2500_diffuse_48x32.npz", "random", 2500, 9, 48, 32, "diffuse"),
]


def make(fname, scene_name, param, seed, w, h, kind):
    scene = mrt.Scene.synthetic(scene_name, param, seed)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, ao = scene.camera()
    rays, _ = mrt.primary_rays(cam, w, h)
    any_hit = False
    if kind != "primary":
        prim, _, _ = O.trace(rays, nodes, woop, tri)
        rays = mrt.ao_rays(rays, prim, scene, ao if kind == "ao" else cam.far)
        any_hit = kind == "ao"
    res, stats, _ = O.trace(rays, nodes, woop, tri, any_hit=any_hit, stats=True)
    np.savez_compressed(os.path.join(HERE, fname), scene=scene_name, param=param, seed=seed, rays=rays,
                        nodes=nodes, woop=woop, tri_index=tri, any_hit=any_hit, results=res, stats=stats)
    print(fname, len(rays), "rays,", int((res[:, 0] != -1).sum()), "hits")


if __name__ == "__main__":
    for c in CASES:
        make(*c)
