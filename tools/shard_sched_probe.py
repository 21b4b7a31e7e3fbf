"""Schedules for one 8-rank strong-scaling shard (round 6): the shard is one 2.07 M-ray launch whose
rays are ordered live blocks first, while the saved schedule of its size was tuned on the frame-order
1 spp batch. Times the shard (joined steps, like bench.py's projection) under the saved schedule, the
schedule a fresh autotune settles on the shard itself, and fixed configurations.
  python tools/shard_sched_probe.py [rank] ['{"num_queues": 8, ...}' ...]"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from mrt.raygen import RAY_DIFFUSE  # noqa: E402
from mrt.renderer import GlibcRand, Renderer  # noqa: E402
from mrt.schedules import DEFAULT_PATH, ScheduleStore  # noqa: E402
from mrt.tracer import Tracer  # noqa: E402


def main():
    rank = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    cfgs = [json.loads(a) for a in sys.argv[2:]]
    cfg = bench.STRONG
    bench.STORE = ScheduleStore(DEFAULT_PATH)
    scenes = bench.SceneCache(1, 0, "/tmp/mrt_bvhcache")
    e = scenes.get(cfg["scene"])
    tr = Tracer(0)
    bench.bind(tr, e["gbvh"])
    cam, _ = e["scene"].camera()
    r = Renderer(tr, e["scene"], max_batch=cfg["max_batch"], rand=GlibcRand())
    r.set_params(RAY_DIFFUSE, cfg["spp"])
    r.begin_frame(cam, cfg["w"], cfg["h"])
    sb = r.shard(8, rank, cfg["block"])
    print(f"shard rank {rank}/8: {sb.size} rays", flush=True)

    def timed(label, reps=3, steps=50):
        go = tr.launcher(sb, exact_rcp=True)
        out = []
        for _ in range(reps):
            w, _, _ = bench.time_steps([go], steps, 3, 1)
            out.append(w / steps * 1e3)
        print(f"  {label:70s} {np.median(out):.4f} ms (runs {', '.join(f'{x:.4f}' for x in out)}) "
              f"{bench.schedule_of(tr, sb, True)['name']}", flush=True)

    timed("saved schedule")
    tr.set_bvh(e["gbvh"])   # fresh: the autotuner explores on the shard itself
    go = tr.launcher(sb, exact_rcp=True)
    n = 0
    while n < 1200 and not [c for k, _, c, _ in tr.schedules() if k == sb.size]:
        for _ in range(8):
            go()
        n += 8
        torch.cuda.synchronize()
    timed(f"autotuned on the shard ({n} launches)")
    base = tr.config()
    for c in cfgs:
        tr.set_config(**c, autotune=0)
        timed(json.dumps(c))
        tr.set_config(**base)


if __name__ == "__main__":
    main()
