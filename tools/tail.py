"""Tail experiment: how much of the frame time is the slowest rays' critical path?
Traces subsets of the bunny 1024x768 batch ordered by per-ray step count (STATS)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import bench  # noqa
import torch
from mrt.tracer import Tracer, RayBuffer

def timeit(tr, rb, reps=10):
    ms = []
    for i in range(reps + 2):
        m = tr.trace_batch(rb, exact_rcp=True)
        if i >= 2:
            ms.append(m)
    return float(np.median(ms))

def main():
    torch.cuda.set_device(0)
    tr = Tracer(0)
    wl = sys.argv[1] if len(sys.argv) > 1 else "bunny-primary-1024x768"
    scene, bufs, _, _ = bench.bvh_for(bench.workload_spec(wl)[0], 1, 0)
    b = bench.Batches(wl, scene, bufs, tr)
    rb = b.batches[0][0]
    tr.trace_batch(rb, exact_rcp=True, speculative=False, stats=True)
    st = rb.stats.cpu().numpy().astype(np.int64)
    steps = st[:, 0] + st[:, 1] + st[:, 2]
    rays = rb.rays.cpu().numpy()
    order = np.argsort(steps)
    n = len(rays)
    print(f"{wl}: all {n} rays: {timeit(tr, rb):.4f} ms; steps max {steps.max()} p99 {np.percentile(steps, 99)}", flush=True)
    for name, idx in [("slowest ray alone", order[-1:]), ("slowest 64", order[-64:]), ("slowest 1%", order[-n // 100:]),
                      ("fastest 99%", np.sort(order[: n - n // 100])), ("fastest 90%", np.sort(order[: n - n // 10]))]:
        sub = RayBuffer(rays[idx], need_closest_hit=rb.need_closest_hit)
        for w in (0, 4, 32):
            tr.set_config(waves_per_cu=w)
            print(f"  {name:18s} ({len(idx)} rays, max steps {steps[idx].max()}) waves={w}: {timeit(tr, sub):.4f} ms", flush=True)
        tr.set_config(waves_per_cu=0)

if __name__ == "__main__":
    main()
