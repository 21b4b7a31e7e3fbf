"""Per-ray latency census (STATS kernel variant records s_memrealtime deltas):
how long the slowest rays take, and the time per traversal step."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import bench  # noqa
import torch
from mrt.tracer import Tracer

def main():
    torch.cuda.set_device(0)
    tr = Tracer(0)
    base = tr.config()
    for wl in sys.argv[1].split(","):
        scene, bufs, _, _ = bench.bvh_for(bench.workload_spec(wl)[0], 1, 0)
        b = bench.Batches(wl, scene, bufs, tr)
        for cfg in [{}, {"waves_per_cu": 8}]:
            tr.set_config(**{**base, **cfg})
            for spec in (True, False):
                rb = b.batches[0][0]
                ms = [tr.trace_batch(rb, exact_rcp=True, speculative=spec, stats=True) for _ in range(3)][-1]
                st = rb.stats.cpu().numpy().astype(np.int64)
                steps = st[:, 0] + st[:, 1] + st[:, 2]
                lat = st[:, 3] * 0.01   # us
                i = np.argmax(lat)
                print(f"{wl} {cfg} spec={spec}: kernel {ms*1e3:.1f} us; ray latency p50 {np.percentile(lat,50):.2f} "
                      f"p99 {np.percentile(lat,99):.2f} max {lat.max():.2f} us (steps {steps[i]}); "
                      f"us/step mean {np.sum(lat)/np.sum(steps):.3f}; max steps {steps.max()} "
                      f"(lat {lat[np.argmax(steps)]:.2f} us)", flush=True)
        tr.set_config(**base)

if __name__ == "__main__":
    main()
