"""Would a live-first ray order pay on a single frame? (diagnostic, one GPU)

Times one bench workload's batch in the caller's (frame) order and reordered with
its block_weights-sorted blocks first (mrt.dist.shard_spans priority, world = 1),
under a fixed schedule, with HIP events around back-to-back launches.

  python tools/order_probe.py hairball-diffuse-1920x1080 '{"autotune": 0, ...}' [block ...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from mrt.dist import block_weights, local_rays, shard_spans  # noqa: E402
from mrt.tracer import RayBuffer, Tracer  # noqa: E402


def timed(tracer, rb, launches=30, rounds=7):
    go = tracer.launcher(rb, exact_rcp=True)
    out = []
    for r in range(rounds + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(launches):
            go()
        b.record()
        torch.cuda.synchronize()
        if r:
            out.append(a.elapsed_time(b) / launches)
    return sorted(out)[len(out) // 2]


def main():
    wl, cfg = sys.argv[1], json.loads(sys.argv[2])
    blocks = [int(x) for x in sys.argv[3:]] or [1024]
    torch.cuda.set_device(0)
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    e = scenes.get(bench.workload_spec(wl)[0])
    rb = bench.Batches(wl, e["scene"], e["gbvh"], tracer).batches[0][0]
    tracer.set_config(**cfg)
    live = int((rb.rays[:, 7] >= 0).sum())
    print(f"{wl}: {rb.size} rays, {live} live; {cfg}", flush=True)
    print(f"  frame order: {timed(tracer, rb):.4f} ms", flush=True)
    for blk in blocks:
        w = block_weights(rb.rays, blk)
        ordered = RayBuffer(local_rays(rb.rays, shard_spans(rb.size, 1, 0, blk, None, w)).contiguous(),
                            rb.need_closest_hit)
        print(f"  live blocks first ({blk}-ray blocks): {timed(tracer, ordered):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
