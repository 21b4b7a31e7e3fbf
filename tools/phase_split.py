"""Diagnostic: how a workload's trace time splits between the node loop and the
leaf (triangle) loop. Needs libmrt.so built with -DMRT_PHASE_TIMING
(tools/build_variant.sh phase "-DMRT_PHASE_TIMING"), selected with MRT_LIB_DIR:
the STATS variant then stores, per ray, the 10-ns ticks its wave spent in each
phase while the ray was live. Production mode (speculative, exact rcp) for the
given node width.

  MRT_LIB_DIR=.../variants/phase python tools/phase_split.py hairball-diffuse-1920x1080 [wide]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))


def main():
    import torch
    import bench
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    tr = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    for wl in sys.argv[1].split(","):
        e = scenes.get(bench.workload_spec(wl)[0])
        for wide in (0, 1):
            tr.set_config(wide=wide)
            b = bench.Batches(wl, e["scene"], e["gbvh"], tr)
            rb = b.batches[-1][0]
            for _ in range(3):
                tr.trace_batch(rb, exact_rcp=True)
            plain = np.median([tr.trace_batch(rb, exact_rcp=True) for _ in range(5)])
            ms = tr.trace_batch(rb, exact_rcp=True, stats=True)
            st = rb.stats.cpu().numpy().astype(np.int64)
            live = rb.rays.cpu().numpy()[:, 7] > 0
            node, leaf = st[live, 2].sum() * 1e-2, st[live, 3].sum() * 1e-2
            print(f"{wl:28s} wide={wide}: kernel {plain:.4f} ms ({ms:.4f} with timing); per live ray: "
                  f"{st[live, 0].mean():5.1f} nodes {st[live, 1].mean():5.1f} tris; wave time node loop "
                  f"{node / live.sum():7.1f} us, leaf loop {leaf / live.sum():7.1f} us "
                  f"({100 * leaf / (node + leaf):.0f} % leaf)", flush=True)


if __name__ == "__main__":
    main()
