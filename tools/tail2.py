"""Where does a slow wave's time go? Times one wave of the 64 slowest bunny
rays against the same rays one per wave, and the slowest ray x64 (no divergence)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import bench  # noqa
import torch
from mrt.tracer import Tracer, RayBuffer


def timeit(tr, rb, spec=True, reps=10):
    ms = []
    for i in range(reps + 2):
        m = tr.trace_batch(rb, exact_rcp=True, speculative=spec)
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
    dead = np.array([0, 0, 0, 1, 0, 0, 1, -1], np.float32)   # tmax < tmin: finishes at the root
    slow64 = rays[order[-64:]]
    cases = {
        "slowest x1": rays[order[-1:]],
        "slowest x64 (identical lanes)": np.repeat(rays[order[-1:]], 64, axis=0),
        "slowest 64 in one wave": slow64,
        "slowest 64 one per wave": np.concatenate([np.vstack([r[None], np.repeat(dead[None], 63, 0)]) for r in slow64]),
        "slowest 64 sorted by steps": rays[order[-64:]][np.argsort(steps[order[-64:]])],
        "8 lanes of the slowest 64": slow64[-8:],
    }
    print(f"{wl}: slowest 64 steps {steps[order[-64:]].min()}..{steps[order[-64:]].max()} "
          f"(nodes {st[order[-64:], 0].mean():.1f} tris {st[order[-64:], 1].mean():.1f} leaves {st[order[-64:], 2].mean():.1f})")
    for name, r in cases.items():
        sub = RayBuffer(np.ascontiguousarray(r), need_closest_hit=True)
        print(f"  {name:32s} {len(r):5d} rays: spec {timeit(tr, sub):.4f} ms  lockstep-off {timeit(tr, sub, False):.4f} ms",
              flush=True)


if __name__ == "__main__":
    main()
