"""Builds gpu-ray-tracing_amd/mrt/tuned_schedules.json, the saved autotuner choices the
bench locks at bind (the same schedule every run).

The in-library autotuner ranks candidates from ~100 launches interleaved with each
other, early in a process while clocks still ramp; here every candidate is timed in
steady state instead: the GPU is warmed first, each candidate is locked in turn
(mrt_tracer_tune_import) and timed over interleaved rounds of back-to-back launches
(HIP events): the eight ray-distribution schedules, each also with every stage-2
modifier (spec_slack 4 / 6, the frontier tail toggled, 16 lane groups), then the two fastest against the
fixed rule again; a challenger replaces the rule only when its median is 3 % faster
(mrt_api.cpp kTuneMargin).

  python tools/tune_db.py [--workload W ...] [--rounds 5] [--launches 20] [--out PATH]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))

MARGIN = 0.03
N_SCHEDULES, STAGE2 = 8, 5


def variant_key(any_hit, exact, lds_stack=16, nodes=1, tail=False, secondary=False):
    """mrt_api.cpp's tuning key of a speculative, stats-free launch: variant_key() | 512 for a
    MRT_TRACE_SECONDARY batch."""
    return (int(any_hit) | 2 | (4 if exact else 0) | ({8: 0, 16: 1, 32: 2}[lds_stack] << 4) | (nodes << 6)
            | (256 if tail else 0) | (512 if secondary else 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", action="append")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--fast-rcp", action="store_true", help="tune the v_rcp_f32 variant too")
    ap.add_argument("--out", default=None)
    ap.add_argument("--out-cells", default=None,
                    help="also write each workload's own choice (JSON: workload -> keys, candidate): two ray types of "
                         "one BVH and batch size share a key in --out, the last tuned wins there")
    ap.add_argument("--margin", type=float, default=MARGIN,
                    help="how much faster (median) a candidate must be to replace the rule (the library's 3 %%)")
    args = ap.parse_args()
    import torch
    import bench
    from mrt import _lib
    from mrt.schedules import DEFAULT_PATH, ScheduleStore
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    out = args.out or DEFAULT_PATH
    store = ScheduleStore(out if os.path.exists(out) else "")
    store.path = out
    tracer = Tracer(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    wls = args.workload or [bench.HEADLINE] + bench.EXTRA_N1
    bench.STORE = None
    cells = {}
    for wl in wls:
        e = scenes.get(bench.workload_spec(wl)[0])
        b = bench.Batches(wl, e["scene"], e["gbvh"], tracer)
        for exact in ([True, False] if args.fast_rcp else [True]):
            launches = [tracer.launcher(rb, exact_rcp=exact) for rb, _ in b.batches]
            cfg = tracer.config()
            tail = cfg["tail_lanes"] > 0 and cfg["wide"] == 1   # the library's with_tail()
            keys = sorted({(rb.size, variant_key(not rb.need_closest_hit, exact, tail=tail, secondary=rb.secondary))
                           for rb, _ in b.batches})

            def lock(code):
                tracer.load_schedules([(n, v, code, _lib.MRT_TUNE_VERSION) for n, v in keys])

            def timed(codes):
                t = {c: [] for c in codes}
                for r in range(args.rounds + 1):
                    for c in codes:
                        lock(c)
                        for go in launches * 3:
                            go()
                        # one event pair around back-to-back launches (an event between
                        # launches fences the caches)
                        a_, z_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a_.record()
                        for _ in range(args.launches):
                            for go in launches:
                                go()
                        z_.record()
                        torch.cuda.synchronize()
                        if r:
                            t[c].append(a_.elapsed_time(z_) / args.launches)
                return {c: float(np.median(v)) for c, v in t.items()}

            # warm the clocks on the rule
            lock(0)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.5:
                for go in launches:
                    go()
                torch.cuda.synchronize()
            # the candidate equal to the fixed rule (mrt_api.cpp effective_cfg): the global queue for a
            # BVH above the Infinity Cache, 12 waves/CU up to 3 rays per lane of a 16-wave grid, else 16
            g = e["gbvh"]
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            big = g.node_bytes + g.woop_bytes > bench.MALL_BYTES
            rule_c = 0 if not big else (4 if b.batches[0][0].size <= 3 * cus * 16 * 64 else 3)
            # every schedule, and every schedule with each stage-2 modifier (spec_slack 4, 6, the
            # frontier tail toggled): the in-library tuner only modifies its stage-1 winner, which
            # misses e.g. per-XCD queues without the tail on bunny primary 1024x768
            codes = list(range(N_SCHEDULES)) + [(N_SCHEDULES + k) | (c << 8) for c in range(N_SCHEDULES)
                                                for k in range(STAGE2)]
            s1 = timed(codes)
            best = min(s1, key=s1.get)
            # the two best against each other again (the sweep's medians are one sample each)
            top2 = sorted(s1, key=s1.get)[:2]
            s2 = timed(sorted(set([rule_c] + top2)))
            best2 = min(s2, key=s2.get)
            chosen = best2 if s2[best2] < (1 - args.margin) * s2[rule_c] else rule_c
            lock(chosen)
            store.update(e["gbvh"].fingerprint, tracer.schedules())
            cells[f"{wl}{'' if exact else ':fast'}"] = {"fingerprint": e["gbvh"].fingerprint,
                                                       "keys": [list(k) for k in keys], "candidate": chosen}
            print(f"{wl} exact={exact}: rule {rule_c} {s1[rule_c]:.4f} ms; sweep "
                  + " ".join(f"{c & 0xff}/{c >> 8}:{v:.4f}" for c, v in sorted(s1.items(), key=lambda kv: kv[1])[:6])
                  + "; final " + " ".join(f"{c & 0xff}/{c >> 8}:{v:.4f}" for c, v in s2.items())
                  + f" -> {chosen & 0xff}/{chosen >> 8} ({bench.schedule_name(chosen)})", flush=True)
    store.save(out)
    print(f"wrote {out}")
    if args.out_cells:
        import json
        with open(args.out_cells, "w") as f:
            json.dump({"version": _lib.MRT_TUNE_VERSION, "cells": cells}, f, indent=1)
        print(f"wrote {args.out_cells}")


if __name__ == "__main__":
    main()
