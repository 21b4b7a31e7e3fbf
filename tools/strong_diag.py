"""Strong-scaling shard diagnosis (one GPU): every 8-rank shard of the hairball
1920x1080x8spp buffer traced alone, one launch per step on one stream, under
fixed schedules (no autotuning) and in both shard orders, so that a slow shard
can be told apart from a slow schedule or a timing position. Prints one line per
(schedule, order, shard): rays, live rays, median launch ms (HIP events)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from mrt.dist import balance_blocks, block_weights, local_rays, shard_spans  # noqa: E402
from mrt.raygen import RAY_DIFFUSE  # noqa: E402
from mrt.renderer import Renderer  # noqa: E402
from mrt.tracer import RayBuffer, Tracer  # noqa: E402

SCHEDULES = {
    "rule": {"autotune": 0},
    "xcd4096": {"autotune": 0, "num_queues": 8, "fetch_threshold": 48, "queue_shared": 5, "queue_block": 4096,
                "waves_per_cu": 20},
    "strided20": {"autotune": 0, "num_queues": 0, "waves_per_cu": 20},
}


def main():
    world = int(os.environ.get("WORLD", "8"))
    block = int(os.environ.get("BLOCK", "16384"))
    balance = int(os.environ.get("BALANCE", "0"))
    reps = int(os.environ.get("REPS", "10"))
    torch.cuda.set_device(0)
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, None)
    e = scenes.get("hairball")
    tracer.set_bvh(e["gbvh"])
    cam, _ = e["scene"].camera()
    r = Renderer(tracer, e["scene"], max_batch=1 << 21, exact_rcp=True)
    r.set_params(RAY_DIFFUSE, 8)
    r.begin_frame(cam, 1920, 1080)
    big = torch.cat([b.rays for b, _ in r.batches()])
    n = big.shape[0]
    weights = block_weights(big, block)
    owners = balance_blocks(weights, world) if balance else None
    if os.environ.get("DEAL") == "rot":   # block-cyclic with the deal rotated by one rank per round
        import numpy as np
        nb = len(weights)
        owners = ((np.arange(nb) + np.arange(nb) // world) % world).astype(np.int32)
    prio = weights if int(os.environ.get("ORDER", "0")) else None   # costly (live) blocks first in each shard
    shards = []
    for k in range(world):
        rb = RayBuffer(local_rays(big, shard_spans(n, world, k, block, owners, prio)).contiguous(),
                       need_closest_hit=True, secondary=True)
        shards.append((k, rb, int((rb.rays[:, 7] >= 0).sum())))
    torch.cuda.synchronize()
    if os.environ.get("TIMELINE"):
        # per-ray {start, end, tail entry, iterations} of shard 0 (needs MRT_LIB_DIR = a -DMRT_TAIL_TIMELINE build)
        import numpy as np
        name = os.environ.get("SCHEDS", "x8192").split(",")[0]
        for item in filter(None, os.environ.get("EXTRA_SCHEDS", "").split(";")):
            nm, cfg = item.split("=", 1)
            SCHEDULES[nm] = __import__("json").loads(cfg)
        tracer.set_config(**SCHEDULES[name])
        k, rb, live = shards[0]
        for _ in range(3):
            tracer.trace_batch(rb, exact_rcp=True)
        st = None
        for _ in range(3):
            tracer.trace_batch(rb, exact_rcp=True, stats=True)
            st = rb.stats.cpu().numpy().astype(np.int64)
        t0 = st[:, 0].min()
        start, end = (st[:, 0] - t0) * 0.01, (st[:, 1] - t0) * 0.01
        dry = start.max()
        liv = rb.rays[:, 7].cpu().numpy() >= 0
        print(f"timeline shard {k} ({name}): last ray ends {end.max():.1f} us; first-round starts by "
              f"{np.percentile(start, 1):.1f}..{np.percentile(start[:327680], 99):.1f} us; "
              + " ".join(f"{q}%:{np.percentile(end, q):.1f}" for q in (50, 90, 99, 99.9)), flush=True)
        print(f"   last fetch {dry:.1f} us; live rays in flight then {int(((start <= dry) & (end > dry) & liv).sum())}; "
              f"in flight at +10/+25/+50 us: " + " ".join(str(int(((start <= dry + d) & (end > dry + d)).sum()))
                                                       for d in (10, 25, 50)), flush=True)
        last_live_start = start[liv].max()
        print(f"   last live ray fetched at {last_live_start:.1f} us; live rays done by then "
              f"{100.0 * (end[liv] <= last_live_start).mean():.1f} %", flush=True)
        return
    if os.environ.get("STATS"):
        # the shards' traversal work: node visits and triangle tests per shard (STATS variant)
        for k, rb, live in shards:
            tracer.trace_batch(rb, exact_rcp=True, stats=True)
            st = rb.stats.to(torch.int64).sum(0).tolist()
            print(f"work shard {k}: rays {rb.size} live {live} nodes {st[0]} tris {st[1]} leaves {st[2]} "
                  f"nodes/live {st[0] / max(1, live):.2f}", flush=True)
    import time
    from mrt.dist import shard_launches
    whole = RayBuffer(local_rays(big, shard_spans(n, 1, 0, block, None, prio)).contiguous(), need_closest_hit=True,
                      secondary=True)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    import json
    for item in filter(None, os.environ.get("EXTRA_SCHEDS", "").split(";")):
        name, cfg = item.split("=", 1)
        SCHEDULES[name] = json.loads(cfg)
    only = os.environ.get("SCHEDS")
    for name, cfg in SCHEDULES.items():
        if only and name not in only.split(","):
            continue
        base = tracer.config()
        tracer.set_config(**cfg)
        for ns in (2, 1):
            # T1: the whole buffer in <= 2^21-ray launches alternating over ns streams
            gos = [tracer.launcher(whole.view(a, b), exact_rcp=True, stream=streams[i % ns])
                   for i, (a, b) in enumerate(shard_launches(0, whole.size, 1 << 21))]

            def step():
                for go in gos:
                    with torch.cuda.stream(go.stream):
                        go()
                if ns > 1:
                    streams[0].wait_stream(streams[1])
                    streams[1].wait_stream(streams[0])
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                step()
            torch.cuda.synchronize()
            print(f"{name:10s} T1 {ns} stream(s): {(time.perf_counter() - t0) / reps * 1e3:.4f} ms", flush=True)
        split = int(os.environ.get("SPLIT", "1"))
        if split > 1:
            # each shard as `split` launches alternating over the two streams, joined per step
            for k, rb, live in shards:
                gos = [tracer.launcher(rb.view(a, b), exact_rcp=True, stream=streams[i % 2])
                       for i, (a, b) in enumerate(shard_launches(0, rb.size, 1 << 21, split))]

                def sstep():
                    streams[1].wait_stream(streams[0])
                    for go in gos:
                        with torch.cuda.stream(go.stream):
                            go()
                    streams[0].wait_stream(streams[1])
                for _ in range(3):
                    sstep()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    sstep()
                torch.cuda.synchronize()
                print(f"{name:10s} fwd shard {k}: rays {rb.size} live {live} median "
                      f"{(time.perf_counter() - t0) / reps * 1e3:.4f} ms (split {split})", flush=True)
            tracer.set_config(**{kk: base[kk] for kk in cfg})
            continue
        for order in os.environ.get("ORDERS", "fwd,rev").split(","):
            seq = shards if order == "fwd" else shards[::-1]
            for k, rb, live in seq:
                for _ in range(2):
                    tracer.trace_batch(rb, exact_rcp=True)
                ms = sorted(tracer.trace_batch(rb, exact_rcp=True) for _ in range(reps))
                print(f"{name:10s} {order} shard {k}: rays {rb.size} live {live} median {ms[reps // 2]:.4f} ms "
                      f"min {ms[0]:.4f}", flush=True)
        tracer.set_config(**{k: base[k] for k in cfg})


if __name__ == "__main__":
    main()
