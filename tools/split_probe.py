"""Does a large batch trace faster as k concurrent sub-launches on two streams?
For each workload: the batch as one launch vs cut into k balanced sub-launches
alternating over two streams (the strong-scaling shards' form); wall time per
step over interleaved rounds, results checked equal to the one-launch trace.
--overlap lets consecutive steps overlap (no per-step join): that measures a
pipeline of frames, not one frame (profiles/round2_tuning.md).

  python tools/split_probe.py hairball-diffuse-1920x1080 sponza-diffuse-1920x1080
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))


def main():
    import torch
    import bench
    from mrt.dist import shard_launches
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    overlap = "--overlap" in sys.argv
    for wl in [a for a in sys.argv[1:] if not a.startswith("--")]:
        e = scenes.get(bench.workload_spec(wl)[0])
        b = bench.Batches(wl, e["scene"], e["gbvh"], tracer)
        rb = b.batches[-1][0]
        variants = {}
        for k in (1, 2, 4):
            variants[k] = [tracer.launcher(rb.view(lo, hi), exact_rcp=True, stream=streams[i % 2])
                           for i, (lo, hi) in enumerate(shard_launches(0, rb.size, 1 << 30, k))]
        times = {k: [] for k in variants}
        ref = None
        for rnd in range(6):
            for k, ls in variants.items():
                bench.warm(ls, 5, 0.05)
                torch.cuda.synchronize()
                step = (lambda ls=ls: [go() for go in ls]) if overlap else bench.joined(ls)
                t0 = time.perf_counter()
                for _ in range(20):
                    step()
                torch.cuda.synchronize()
                if rnd > 0:
                    times[k].append((time.perf_counter() - t0) / 20 * 1e3)
                out = rb.results[:, :2].cpu().numpy()
                if ref is None:
                    ref = out
                elif rb.need_closest_hit and not np.array_equal(out, ref):
                    print(f"  WARNING: k={k} results differ", flush=True)
        base = np.median(times[1])
        print(f"{wl} ({rb.size} rays):", "  ".join(f"k={k} {np.median(v):.4f} ms (x{base / np.median(v):.3f})"
                                                   for k, v in times.items()), flush=True)


if __name__ == "__main__":
    main()
