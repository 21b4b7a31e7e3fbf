"""Experiment: how much does ray order (coherence inside a wave) move the trace
time of incoherent batches? Rays of a bench workload are reordered on the host by
several keys, uploaded, and traced; median kernel time per ordering (HIP events,
20 launches after warmup). Results are checked to be the same rays' results.

  python tools/sort_probe.py hairball-diffuse-1920x1080 sponza-diffuse-640x480
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))


def part1by2(x):
    x = x.astype(np.uint64) & 0x3FF
    x = (x | (x << 16)) & 0x030000FF
    x = (x | (x << 8)) & 0x0300F00F
    x = (x | (x << 4)) & 0x030C30C3
    x = (x | (x << 2)) & 0x09249249
    return x


def morton3(q):   # q: [n, 3] ints in [0, 1024)
    return (part1by2(q[:, 0]) << 2) | (part1by2(q[:, 1]) << 1) | part1by2(q[:, 2])


def quant(v, bits):
    lo, hi = v.min(0), v.max(0)
    return np.clip(((v - lo) / np.maximum(hi - lo, 1e-30) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)


def keys(rays):
    o, d = rays[:, 0:3], rays[:, 4:7]
    live = rays[:, 7] > 0
    octant = ((d[:, 0] < 0).astype(np.uint64) << 2) | ((d[:, 1] < 0).astype(np.uint64) << 1) | (d[:, 2] < 0)
    mo = morton3(quant(o, 10))
    md = morton3(quant(d, 10))
    out = {
        "octant+origin": (octant << 30) | mo,
        "origin": mo,
        "dir(5)+origin(5)": (morton3(quant(d, 5)) << 15) | morton3(quant(o, 5)),
        "origin(5)+dir(5)": (morton3(quant(o, 5)) << 15) | morton3(quant(d, 5)),
        "dir": md,
        "octant+origin(4)+dir(6)": (octant << 30) | (morton3(quant(o, 4)) << 18) | morton3(quant(d, 6)),
    }
    # dead rays (tmax < 0, missed primaries) first: they cost nothing either way
    return {k: np.where(live, v + (np.uint64(1) << np.uint64(40)), v) for k, v in out.items()}


def main():
    import torch
    import bench
    from mrt.tracer import RayBuffer, Tracer
    torch.cuda.set_device(0)
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    for name in sys.argv[1:]:
        e = scenes.get(bench.workload_spec(name)[0])
        b = bench.Batches(name, e["scene"], e["gbvh"], tracer)
        rb0 = b.batches[0][0]
        rays = rb0.rays.cpu().numpy()
        tracer.trace_batch(rb0, exact_rcp=True)
        ref = rb0.results_numpy()
        orders = {"as generated": np.arange(len(rays))}
        for k, v in keys(rays).items():
            orders[k] = np.argsort(v, kind="stable")
        for k, perm in orders.items():
            rb = RayBuffer(rays[perm], need_closest_hit=rb0.need_closest_hit)
            go = tracer.launcher(rb, exact_rcp=True)
            for _ in range(30):
                go()
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                go()
                z.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(z))
            same = np.array_equal(rb.results_numpy()[:, :2], ref[perm, :2]) if rb0.need_closest_hit else None
            print(f"{name:32s} {k:28s} {np.median(ts):8.4f} ms  results equal: {same}", flush=True)


if __name__ == "__main__":
    main()
