"""Frame timeline of one trace launch (diagnostic). Needs a libmrt.so built with
-DMRT_STATS_TIMELINE (tools/build_variant.sh timeline "-DMRT_STATS_TIMELINE"),
selected with MRT_LIB_DIR: the STATS variant then stores per ray {start, end,
wave, steps} in 10-ns s_memrealtime ticks. Runs the production mode
(speculative, exact rcp) and prints when rays start/finish, how many are in
flight, and which waves finish last; saves the raw arrays to gpurun_out/."""
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
    wl = sys.argv[1] if len(sys.argv) > 1 else "bunny-primary-1024x768"
    if len(sys.argv) > 2:
        import json
        tr.set_config(**json.loads(sys.argv[2]))
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    e = scenes.get(bench.workload_spec(wl)[0])
    b = bench.Batches(wl, e["scene"], e["gbvh"], tr)
    rb = b.batches[0][0]
    for _ in range(3):
        tr.trace_batch(rb, exact_rcp=True)
    plain = np.median([tr.trace_batch(rb, exact_rcp=True) for _ in range(10)])
    ms = [tr.trace_batch(rb, exact_rcp=True, stats=True) for _ in range(3)]
    print(f"  trace info: {tr.last_info}", flush=True)
    st = rb.stats.cpu().numpy().astype(np.int64)
    start, end, wave, steps = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    t0 = start.min()
    start, end = (start - t0) * 0.01, (end - t0) * 0.01     # microseconds
    dur = end - start
    n = len(start)
    print(f"{wl}: {n} rays; kernel {plain:.4f} ms plain, {np.median(ms):.4f} ms with timeline stats; "
          f"last end {end.max():.1f} us", flush=True)
    for q in (50, 90, 99, 99.9, 100):
        print(f"  {q:5}% of rays done by {np.percentile(end, q):7.1f} us", flush=True)
    span = end.max()
    edges = np.linspace(0, span * 1.0001, 11)
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (end >= lo) & (end < hi)
        if sel.any():
            print(f"  ending in [{lo:.0f},{hi:.0f}) us: {sel.sum():7d} rays, start median {np.median(start[sel]):6.1f} "
                  f"dur median {np.median(dur[sel]):6.1f} max {dur[sel].max():6.1f} steps median {np.median(steps[sel]):5.0f} "
                  f"max {steps[sel].max()}", flush=True)
    order = np.argsort(end)[::-1]
    print("  last 10 rays: (start, dur, steps, wave)", [(round(start[i], 1), round(dur[i], 1), int(steps[i]), int(wave[i]))
                                                         for i in order[:10]])
    wend = {}
    for w in np.unique(wave[order[:2000]]):
        sel = wave == w
        wend[w] = (end[sel].max(), sel.sum(), np.sort(start[sel]).round(1)[:6].tolist())
    print("  last-finishing waves (end us, rays, first starts):")
    for w, v in sorted(wend.items(), key=lambda kv: -kv[1][0])[:10]:
        print(f"    wave {w}: end {v[0]:.1f} rays {v[1]} starts {v[2]}")
    bins = np.linspace(0, end.max(), 41)
    inflight = [(int(((start <= t) & (end > t)).sum())) for t in bins]
    waves_live = [len(np.unique(wave[(start <= t) & (end > t)])) for t in bins]
    print("  t(us) rays-in-flight waves-live:")
    for t, a, w in zip(bins, inflight, waves_live):
        print(f"    {t:6.0f} {a:7d} {w:6d}")
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "gpurun_out", f"timeline_{wl}{os.environ.get('TL_TAG', '')}.npz"), start=start.astype(np.float32),
                        end=end.astype(np.float32), wave=wave.astype(np.int32), steps=steps.astype(np.int32))


if __name__ == "__main__":
    main()
