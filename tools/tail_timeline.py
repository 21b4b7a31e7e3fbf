"""Where a frame's time goes with the cooperative tail (diagnostic). Needs a libmrt.so
built with -DMRT_TAIL_TIMELINE (tools/build_variant.sh tailtl "-DMRT_TAIL_TIMELINE"),
selected with MRT_LIB_DIR: the STATS variant stores per ray {start, end, tail entry,
tail iterations} (10-ns s_memrealtime ticks; tail entry 0 = finished in the main
loop, then the last field is its step count). Prints the frame's last-ray time, when
the main loop hands its stragglers to the tail, and the tail's time per iteration.
  python tools/tail_timeline.py WORKLOAD '{"tail_lanes": 16, "autotune": 0}' ..."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import bench  # noqa: E402
import torch  # noqa: E402
from mrt.tracer import Tracer  # noqa: E402


def main():
    torch.cuda.set_device(0)
    tr = Tracer(0)
    wl = sys.argv[1]
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    e = scenes.get(bench.workload_spec(wl)[0])
    b = bench.Batches(wl, e["scene"], e["gbvh"], tr)
    rb = b.batches[0][0]
    base = tr.config()
    for cfg in sys.argv[2:]:
        tr.set_config(**{**base, **json.loads(cfg)})
        for _ in range(5):
            tr.trace_batch(rb, exact_rcp=True)
        plain = np.median([tr.trace_batch(rb, exact_rcp=True) for _ in range(10)])
        runs = []
        for _ in range(5):
            tr.trace_batch(rb, exact_rcp=True, stats=True)
            runs.append(rb.stats.cpu().numpy().astype(np.int64))
        # the run with the median last end
        ends = [r[:, 1].max() - r[:, 0].min() for r in runs]
        if os.environ.get("TL2"):
            # MRT_TAIL_TIMELINE=2 build: field 0 holds the ticks spent popping the home stack
            st = runs[0]
            tail = st[:, 2] != 0
            iters = np.maximum(1, st[:, 3] & 0xFFFF)
            per_it = (st[:, 1] - st[:, 2]) * 0.01 / iters
            pop = st[:, 0] * 0.01 / iters
            mem = ((st[:, 3] >> 16) & 0xFFFF) * 0.01 / iters
            print(f"{wl} {cfg}: kernel {plain:.4f} ms; {tail.sum()} tail rays; us per tail iteration median "
                  f"{np.median(per_it[tail]):.3f} (node/leaf loads {np.median(mem[tail]):.3f}, pop "
                  f"{np.median(pop[tail]):.3f}); p90 {np.percentile(per_it[tail], 90):.3f} (loads "
                  f"{np.percentile(mem[tail], 90):.3f}, pop {np.percentile(pop[tail], 90):.3f})", flush=True)
            continue
        st = runs[int(np.argsort(ends)[len(ends) // 2])]
        t0 = st[:, 0].min()
        start, end = (st[:, 0] - t0) * 0.01, (st[:, 1] - t0) * 0.01
        tail = st[:, 2] != 0
        entry = np.where(tail, (st[:, 2] - t0) * 0.01, np.nan)
        iters = np.where(tail, st[:, 3] & 0xFFFF, 0)
        mem = np.where(tail, (st[:, 3] >> 16) & 0xFFFF, 0) * 0.01   # us waiting for the step's loads
        print(f"{wl} {cfg}: kernel {plain:.4f} ms; last ray ends {end.max():.1f} us; "
              f"{tail.sum()} of {len(end)} rays finished in the tail", flush=True)
        for q in (50, 90, 99, 99.9, 100):
            print(f"   {q:5}% of rays done by {np.percentile(end, q):7.1f} us")
        print("   ray starts (with a -DMRT_TAIL_TIMELINE=3 build: a lane's first ray = its wave's start): "
              + " ".join(f"p{q}:{np.percentile(start, q):.1f}" for q in (1, 10, 50, 90, 99, 100)) + " us")
        # the last fetch: the queue (or the strided rounds) ran dry here; what was in flight then
        dry = start.max()
        fl = (start <= dry) & (end > dry)
        print(f"   last ray fetched at {dry:.1f} us ({100.0 * (end <= dry).mean():.1f} % done by then, {fl.sum()} in "
              f"flight); drain {end.max() - dry:.1f} us; in flight at +10/+25/+50/+100 us: "
              + " ".join(str(int(((start <= dry + d) & (end > dry + d)).sum())) for d in (10, 25, 50, 100)))
        if tail.any():
            print(f"   tail entries after the last fetch: {int((entry[tail] > dry).sum())} of {tail.sum()}; "
                  f"rays in flight at the last fetch that end in the tail: {int((fl & tail).sum())}")
        if tail.any():
            per = (end[tail] - entry[tail]) / np.maximum(1, iters[tail])
            print(f"   tail entries: median {np.nanmedian(entry):.1f} us, 90% by {np.nanpercentile(entry, 90):.1f}, "
                  f"last {np.nanmax(entry):.1f}; iterations per ray median {np.median(iters[tail]):.0f} "
                  f"max {iters[tail].max()}; us per iteration median {np.median(per):.3f} p90 {np.percentile(per, 90):.3f}; "
                  f"of which waiting for loads median {np.median(mem[tail] / np.maximum(1, iters[tail])):.3f}")
            last = np.argsort(end)[::-1][:8]
            print("   last rays (start, tail entry, end, tail iters):",
                  [(round(start[i], 1), round(entry[i], 1) if tail[i] else None, round(end[i], 1), int(iters[i]))
                   for i in last])
        else:
            last = np.argsort(end)[::-1][:8]
            print("   last rays (start, end, steps):", [(round(start[i], 1), round(end[i], 1), int(st[i, 3])) for i in last])


if __name__ == "__main__":
    main()
