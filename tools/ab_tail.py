"""Interleaved A/B of launch configs on the bench's own workloads (one process, same
inputs, same clocks): median per-launch kernel ms over rounds of back-to-back launches
timed with HIP events on the launch stream. Default: the cooperative tail off/on.

  python tools/ab_tail.py [--workload W ...] [--config '{"tail_lanes": 0}' ...]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))

DEFAULT_WL = ["bunny-primary-640x480", "bunny-primary-1024x768", "conference-ao-640x480", "mori-ao-640x480",
              "sponza-diffuse-640x480", "hairball-diffuse-640x480", "hairball-diffuse-1920x1080"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", action="append")
    ap.add_argument("--config", action="append", help="JSON launch config (repeatable)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--fast-rcp", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    cfgs = [json.loads(c) for c in (args.config or ['{"tail_lanes": 0, "autotune": 0}',
                                                     '{"tail_lanes": 16, "autotune": 0}'])]
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    base = tracer.config()
    for wl in args.workload or DEFAULT_WL:
        e = scenes.get(bench.workload_spec(wl)[0])
        batches = bench.Batches(wl, e["scene"], e["gbvh"], tracer)
        times = {i: [] for i in range(len(cfgs))}
        for r in range(args.rounds + 1):
            for i, c in enumerate(cfgs):
                tracer.set_config(**{**base, **c})
                launches = [tracer.launcher(rb, exact_rcp=not args.fast_rcp) for rb, _ in batches.batches]
                for go in launches * 3:   # settle
                    go()
                # one event pair around back-to-back launches (an event between launches
                # fences the caches)
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record()
                for _ in range(args.launches):
                    for go in launches:
                        go()
                b_.record()
                torch.cuda.synchronize()
                if r:   # round 0 is a warmup
                    times[i].append(a_.elapsed_time(b_) / args.launches)
        tracer.set_config(**base)
        line = [f"{wl:28s}"]
        for i, c in enumerate(cfgs):
            med = float(np.median(times[i]))
            line.append(f"{json.dumps(c)} {med:.4f} ms ({batches.rays_counted / med / 1e3:.0f} Mrays/s)")
        print("  |  ".join(line), flush=True)


if __name__ == "__main__":
    main()
