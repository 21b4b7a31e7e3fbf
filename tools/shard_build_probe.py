"""Where the strong-scaling shard build goes: device time (HIP events on the
current stream) and host wall time of its parts — the live count per block from the primary
results, the device order of the rank's blocks, the rays generated in that order — for the
N = 1 frame and one 8-rank shard of the hairball 1920x1080x8spp frame.
  python tools/shard_build_probe.py [reps]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from mrt.dist import live_block_weights, shard_blocks_device  # noqa: E402
from mrt.raygen import RAY_DIFFUSE  # noqa: E402
from mrt.renderer import GlibcRand, Renderer  # noqa: E402
from mrt.tracer import Tracer  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg = bench.STRONG
    scenes = bench.SceneCache(1, 0, "/tmp/mrt_bvhcache")
    e = scenes.get(cfg["scene"])
    tr = Tracer(0)
    bench.bind(tr, e["gbvh"])
    cam, _ = e["scene"].camera()
    r = Renderer(tr, e["scene"], max_batch=cfg["max_batch"], rand=GlibcRand())
    r.set_params(RAY_DIFFUSE, cfg["spp"])
    r.begin_frame(cam, cfg["w"], cfg["h"])
    r.batch_seeds()
    n, B = r.primary.size * cfg["spp"], cfg["block"]
    for world, rank in ((1, 0), (8, 0), (8, 7)):
        parts = {"weights": [], "order": [], "raygen": [], "all_device": [], "all_host": []}
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev[0].record()
            w = live_block_weights(r.primary.results, cfg["spp"], B)
            ev[1].record()
            blocks, m = shard_blocks_device(n, world, rank, B, priority=w, device=w.device)
            ev[2].record()
            rb = r.secondary_blocks(blocks, m, B)
            ev[3].record()
            torch.cuda.synchronize()
            parts["all_host"].append(1e3 * (time.perf_counter() - t0))
            parts["weights"].append(ev[0].elapsed_time(ev[1]))
            parts["order"].append(ev[1].elapsed_time(ev[2]))
            parts["raygen"].append(ev[2].elapsed_time(ev[3]))
            parts["all_device"].append(ev[0].elapsed_time(ev[3]))
            del rb
        med = {k: round(sorted(v)[len(v) // 2], 4) for k, v in parts.items()}
        print(f"world {world} rank {rank}: {m} rays, {blocks.numel()} blocks  torch order, median ms {med}", flush=True)
        lib = {"order": [], "raygen": [], "all_device": [], "all_host": []}
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev[0].record()
            blocks, m = r.gen.shard_blocks(r.primary, cfg["spp"], B, world, rank, 1)
            ev[1].record()
            rb = r.secondary_blocks(blocks, m, B)
            ev[2].record()
            torch.cuda.synchronize()
            lib["all_host"].append(1e3 * (time.perf_counter() - t0))
            lib["order"].append(ev[0].elapsed_time(ev[1]))
            lib["raygen"].append(ev[1].elapsed_time(ev[2]))
            lib["all_device"].append(ev[0].elapsed_time(ev[2]))
            del rb
        med = {k: round(sorted(v)[len(v) // 2], 4) for k, v in lib.items()}
        print(f"world {world} rank {rank}: library order (mrt_shard_blocks), median ms {med}", flush=True)


if __name__ == "__main__":
    main()
