#!/usr/bin/env python3
"""Benchmark of the MI355X BVH traversal hot path (the reference's `trace`
kernel behind CudaTracer::traceBatch, reference App.cc:137-210).

One "step" = one pass of the hot path over one batch: the persistent trace
launch(es) over every ray of the workload, rays and BVH already resident in
HBM. The headline workload (BASELINE.json configs[1]) is Bunny primary rays at
1024x768 on one MI355X; its metric is the reference's Mrays/s
(rays counted / kernel time, App.cc:204). Scenes are deterministic synthetic
stand-ins with the published triangle counts (the OBJ assets are absent).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--extra/--no-extra]

For N>1 launch with torch.distributed.run (one rank per GPU, RCCL): rank 0
builds the SBVH and broadcasts the Compact2 buffers (the BVH is replicated).
The job is N samples per pixel of the workload's view, sharded by sample:
rank r traces the rays of sample r (rank 0's are the reference's pixel-centre
rays; rank r > 0 samples each pixel at the r-th Halton (2,3) point), so every
rank traces a distinct, equally sized and equally coherent batch (weak
scaling, no collective in the timed region); time = max over ranks, value =
rays counted on all ranks / time. After the timed steps the hit results are
gathered to rank 0 over RCCL point-to-point (timed separately). Rank 0 prints
one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))

METRIC = "Mrays/s (primary/AO/diffuse) at 1/2/4/8 GPUs; achieved HBM GB/s % of peak"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# README numbers (Kepler-class sm_35 build, hardware unstated) — README.md:46-81.
REFERENCE_MRAYS = {
    "bunny-primary-640x480": 825.11,
    "conference-ao-640x480": 1478.43,
    "sponza-diffuse-640x480": 325.33,
    "mori-primary-640x480": 1271.61,
    "mori-ao-640x480": 2763.01,
    "mori-diffuse-640x480": 1466.05,
    "sponza-primary-640x480": 597.51,
    "sponza-ao-640x480": 1022.61,
    "conference-diffuse-640x480": 831.28,
    "hairball-primary-640x480": 280.49,
    "dragon-primary-640x480": 575.43,
    "fairy-ao-640x480": 1280.77,
    "fairy-diffuse-640x480": 678.77,
    "sibenik-ao-640x480": 1499.86,
    "sibenik-diffuse-640x480": 286.97,
    "san-ao-640x480": 556.89,
    "san-diffuse-640x480": 132.28,
}

WORKLOADS = {
    # name: (scene, width, height, ray type, bounces)
    "bunny-primary-1024x768": ("bunny", 1024, 768, "primary", 1),
    "bunny-primary-640x480": ("bunny", 640, 480, "primary", 1),
    "conference-ao-640x480": ("conference", 640, 480, "ao", 1),
    "conference-diffuse-640x480": ("conference", 640, 480, "diffuse", 1),
    "sponza-diffuse-640x480": ("sponza", 640, 480, "diffuse", 1),
    "sponza-diffuse2-640x480": ("sponza", 640, 480, "diffuse", 2),
    "sponza-primary-640x480": ("sponza", 640, 480, "primary", 1),
    "sponza-ao-640x480": ("sponza", 640, 480, "ao", 1),
    "mori-primary-640x480": ("mori", 640, 480, "primary", 1),
    "mori-ao-640x480": ("mori", 640, 480, "ao", 1),
    "mori-diffuse-640x480": ("mori", 640, 480, "diffuse", 1),
    "hairball-primary-640x480": ("hairball", 640, 480, "primary", 1),
    "hairball-diffuse-640x480": ("hairball", 640, 480, "diffuse", 1),
    "hairball-diffuse-1920x1080": ("hairball", 1920, 1080, "diffuse", 1),
}
HEADLINE = "bunny-primary-1024x768"


def workload_spec(name):
    """WORKLOADS entry, or a parsed '<scene>-<primary|ao|diffuse|diffuseN>-<W>x<H>' name."""
    if name in WORKLOADS:
        return WORKLOADS[name]
    scene, kind, res = name.split("-")
    w, h = (int(v) for v in res.split("x"))
    bounces = int(kind[7:]) if kind.startswith("diffuse") and len(kind) > 7 else 1
    return (scene, w, h, kind.rstrip("0123456789"), bounces)
EXTRA_N1 = ["bunny-primary-640x480", "conference-ao-640x480", "sponza-diffuse-640x480", "sponza-diffuse2-640x480"]


# PMC-measured HBM traffic per launch (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in
# separate passes, tools/profile_round.sh + tools/summarize_prof.py); counters
# cannot be read inside this timed process, so the committed profile is cited.
PMC_PROFILES = {w: f"profiles/round1_{w}_pmc_summary.json" for w in
                ("bunny-primary-1024x768", "bunny-primary-640x480", "conference-ao-640x480", "sponza-diffuse-640x480",
                 "sponza-diffuse2-640x480", "hairball-diffuse-640x480")}


def pmc_traffic(name):
    path = os.path.join(REPO, PMC_PROFILES.get(name, "-"))
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        s = json.load(f)
    hbm = s.get("hbm_bytes_per_launch")
    return (int(hbm["total_corrected"]) if hbm else None), PMC_PROFILES[name]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- setup
DIST_BACKEND = "nccl"


def dist_setup(n_gpus, backend="nccl"):
    """One process per GPU. backend "nccl" is RCCL; "gloo" (CPU collectives) is
    only for rehearsing the N>1 flow with several ranks on one GPU."""
    global DIST_BACKEND
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    device = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        DIST_BACKEND = backend
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    return rank, world, device


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def bvh_for(scene_name, world, rank, cache_dir=None):
    """Rank 0 builds the SBVH (or loads it from cache_dir/<scene>.dat, the
    reference's bvhcache idea, Renderer.cc:157-217); the Compact2 buffers are
    broadcast over RCCL."""
    import mrt
    scene = mrt.Scene.synthetic(scene_name, 0, 1)
    t0 = time.perf_counter()
    if rank == 0:
        path = os.path.join(cache_dir, f"{scene_name}.dat") if cache_dir else None
        if path and os.path.exists(path):
            bvh = mrt.Bvh.load(path)
        else:
            bvh = mrt.Bvh.build(scene)
            if path:
                os.makedirs(cache_dir, exist_ok=True)
                bvh.save(path)
        bufs = bvh.buffers()
        stats = bvh.stats()
    else:
        bufs, stats = None, None
    build_s = time.perf_counter() - t0
    if world > 1:
        from mrt.dist import replicate_buffers
        bufs = tuple(replicate_buffers(bufs, src=0))
    return scene, bufs, stats, build_s


def halton(i, base):
    f, r = 1.0, 0.0
    while i > 0:
        f /= base
        r += f * (i % base)
        i //= base
    return r


def subpixel_sample(rank):
    """Sample position inside the pixel for the shard of `rank`: the centre (the
    reference's primary rays) for rank 0, the rank-th Halton (2,3) point otherwise."""
    return (0.5, 0.5) if rank == 0 else (halton(rank, 2), halton(rank, 3))


class Batches:
    """Ray batches of one workload, generated on the device like the reference
    Renderer (Renderer.cc:112-152,242-291; RayGen.cc:50-120): primary rays in
    Morton order; AO/diffuse rays from the traced primary hits (degenerate
    tmax=-1 rays for misses are traced too; only primary hits are counted)."""

    def __init__(self, name, scene, bufs, tracer, rank=0):
        from mrt.raygen import DeviceRayGen
        from mrt.tracer import GpuBvh
        sname, w, h, kind, bounces = workload_spec(name)
        self.name, self.kind, self.w, self.h = name, kind, w, h
        self.gbvh = GpuBvh(bufs)
        tracer.set_bvh(self.gbvh)
        cam, ao_radius = scene.camera()
        gen = DeviceRayGen(scene)   # RayGen on the device (mrt_raygen_*), like the reference's RayGenKernels
        prim, _ = gen.primary(cam, w, h, subpixel=subpixel_sample(rank))
        self.batches = []   # (RayBuffer, rays counted)
        if kind == "primary":
            self.batches.append((prim, w * h))
        else:
            tracer.trace_batch(prim, exact_rcp=True)
            prev = prim
            for b in range(bounces):
                hits = gen.count_hits(prev)
                max_dist = ao_radius if kind == "ao" else cam.far
                rb = gen.ao(prev, 1, max_dist, mrt_seed(b) + 7919 * rank, closest_hit=(kind == "diffuse"))
                self.batches.append((rb, hits))
                if b + 1 < bounces:
                    tracer.trace_batch(rb, exact_rcp=True)
                    prev = rb
        self.rays_counted = sum(c for _, c in self.batches)
        self.rays_traced = sum(rb.size for rb, _ in self.batches)


def mrt_seed(bounce):
    import mrt
    return mrt.AO_SEED + bounce


def algorithmic_bytes(tracer, batches):
    """B_ray = 32 + 8 + 64 N_node + 48 N_tri + 16 N_leaf + 4 [hit],
    with the per-ray counts of the single-ray traversal order (the kernel's
    per-lane mode, which reproduces the CPU restatement's counters exactly)."""
    import torch
    total, nodes, tris, leaves = 0, 0, 0, 0
    for rb, _ in batches.batches:
        saved = rb.results.clone()
        tracer.trace_batch(rb, exact_rcp=True, speculative=False, stats=True)
        s = rb.stats.to(torch.int64)
        hits = (rb.results[:, 0] != -1).to(torch.int64).sum().item()
        n, t, l = (s[:, 0].sum().item(), s[:, 1].sum().item(), s[:, 2].sum().item())
        nodes, tris, leaves = nodes + n, tris + t, leaves + l
        total += 40 * rb.size + 64 * n + 48 * t + 16 * l + 4 * hits
        rb.results.copy_(saved)
    return total, nodes, tris, leaves


def time_steps(tracer, batches, steps, warmup, world, exact):
    """Warmup, then exactly `steps` steps bracketed by barrier + synchronize.
    One HIP event pair on the launch stream around the K steps gives the GPU
    time per launch (kernel duration plus the inter-launch gap, an upper bound on
    the kernel's own average); no per-launch host work besides the launch."""
    import torch
    stream = torch.cuda.current_stream()
    launches = [tracer.launcher(rb, exact_rcp=exact, stream=stream) for rb, _ in batches.batches]
    for _ in range(warmup):
        for go in launches:
            go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        for go in launches:
            go()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    launch_ms = e0.elapsed_time(e1) / (steps * len(launches))
    return wall, launch_ms


def reduce_over_ranks(x, world, op="max"):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if DIST_BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def max_over_ranks(x, world):
    return reduce_over_ranks(x, world, "max")


def gather_to_root(batches, world):
    """The hit-result gather that follows a sharded trace: every
    rank's RayResult {id, t} of each batch to rank 0, RCCL point-to-point
    (mrt/dist.py). Returns (ms, bytes received by rank 0)."""
    import torch
    from mrt.dist import gather_results
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    nbytes = 0
    for rb, _ in batches.batches:
        res = rb.results if DIST_BACKEND == "nccl" else rb.results.cpu()
        full = gather_results(res, world * rb.size)
        if full is not None:
            nbytes += full.numel() * 4
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0)
    return max_over_ranks(ms, world), nbytes


def cpu_baseline(batches, bufs, threads):
    """The oracle (oracle/, a scalar C restatement of the same traversal) on the
    host cores: the first batch of the workload, best of 3 after 1 warmup. Also
    checks the GPU results of that batch against it (parity on the bench input)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    rb, counted = batches.batches[0]
    rays = rb.rays.cpu().numpy()
    any_hit = not rb.need_closest_hit
    nodes, woop, tri = bufs
    res, _, _ = O.trace(rays, nodes, woop, tri, any_hit=any_hit, threads=threads)
    best = min(O.trace(rays, nodes, woop, tri, any_hit=any_hit, threads=threads)[2] for _ in range(3))
    gpu = rb.results_numpy()
    exact = float(((gpu[:, 0] == res[:, 0]) & (gpu[:, 1] == res[:, 1])).mean())
    return {"value": round(counted / best / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{batches.name} batch 0: {rb.size} rays ({counted} counted), best of 3 after 1 warmup, "
                      f"{threads} threads, oracle/trace_oracle.c",
            "parity_exact_fraction": exact}


def run_workload(name, tracer, world, rank, steps, warmup, exact, want_cpu, cache_dir=None):
    scene_name = workload_spec(name)[0]
    scene, bufs, bstats, build_s = bvh_for(scene_name, world, rank, cache_dir)
    batches = Batches(name, scene, bufs, tracer, rank)
    alg_bytes, n_nodes, n_tris, n_leaves = algorithmic_bytes(tracer, batches)
    wall, launch_ms = time_steps(tracer, batches, steps, warmup, world, exact)
    wall = max_over_ranks(wall, world)
    launch_ms = max_over_ranks(launch_ms, world)
    counted = int(reduce_over_ranks(batches.rays_counted, world, "sum"))
    traced = int(reduce_over_ranks(batches.rays_traced, world, "sum"))
    alg_bytes = reduce_over_ranks(alg_bytes, world, "sum") / world   # per-GPU launch bytes (mean over ranks)
    ms_per_step = 1e3 * wall / steps
    value = counted * steps / wall / 1e6
    gather = gather_to_root(batches, world) if world > 1 else None
    kernel_ms_per_step = launch_ms * len(batches.batches)
    achieved = alg_bytes / (kernel_ms_per_step * 1e-3) / 1e9
    out = {
        "workload": name,
        "value": round(value, 2),
        "ms_per_step": round(ms_per_step, 4),
        "kernel_ms_per_launch": round(launch_ms, 4),
        "rays_counted": batches.rays_counted,
        "rays_traced": batches.rays_traced,
        "mrays_traced_per_s": round(traced * steps / wall / 1e6, 2),
        "rays_counted_all_ranks": counted,
        "gather": ({"ms": round(gather[0], 3), "bytes_to_root": gather[1],
                    "value_incl_gather": round(counted * steps / (wall + steps * gather[0] / 1e3) / 1e6, 2)}
                   if gather else None),
        "scene_tris": scene.num_triangles,
        "bvh": {"inner_nodes": len(bufs[0]) // 16, "woop_slots": len(bufs[1]) // 4,
                "bytes": 4 * (len(bufs[0]) + len(bufs[1]) + len(bufs[2])), "build_s": round(build_s, 2),
                **({"max_depth": bstats["max_depth"], "sah": round(bstats["sah_cost"], 2)} if bstats else {})},
        "per_ray": {"nodes": round(n_nodes / batches.rays_traced, 2), "tris": round(n_tris / batches.rays_traced, 2),
                    "leaves": round(n_leaves / batches.rays_traced, 2),
                    "bytes": round(alg_bytes / batches.rays_traced, 1)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(name)[0],
                     "traffic_source": pmc_traffic(name)[1],
                     "algorithmic_bytes_per_launch": int(alg_bytes / len(batches.batches))},
        "reference_mrays": REFERENCE_MRAYS.get(name),
    }
    if want_cpu:
        out["cpu_baseline"] = cpu_baseline(batches, bufs, threads=min(16, os.cpu_count() or 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # 0.15 ms steps: 20 left clocks ramping (4.8-5.3 G vs 5.35 G stable)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default=HEADLINE, help="a WORKLOADS key or <scene>-<ray>-<W>x<H>")
    ap.add_argument("--rcp", default="exact", choices=["exact", "fast"],
                    help="exact = correctly rounded 1/x (bit-identical to the oracle); fast = v_rcp_f32")
    ap.add_argument("--extra", dest="extra", action="store_true", default=None,
                    help="also measure the AO/diffuse configs (default on at N=1)")
    ap.add_argument("--no-extra", dest="extra", action="store_false")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--fetch-threshold", type=int, default=-1)
    ap.add_argument("--lds-stack", type=int, default=0)
    ap.add_argument("--queues", type=int, default=0)
    ap.add_argument("--schedule", type=int, default=0, help="1 while-while, 2 if-if (0: library default)")
    ap.add_argument("--bvh-cache", default=None, help="directory of <scene>.dat Compact2 caches (built if missing)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL) for real runs; gloo only to rehearse N>1 ranks on one GPU")
    ap.add_argument("--lane-groups", type=int, default=0)
    args = ap.parse_args()

    import torch
    from mrt.tracer import Tracer

    rank, world, local = dist_setup(args.gpus, args.dist_backend)
    tracer = Tracer(local)
    cfg = {}
    if args.waves_per_cu:
        cfg["waves_per_cu"] = args.waves_per_cu
    if args.fetch_threshold >= 0:
        cfg["fetch_threshold"] = args.fetch_threshold
    if args.lds_stack:
        cfg["lds_stack"] = args.lds_stack
    if args.queues:
        cfg["num_queues"] = args.queues
    if args.schedule:
        cfg["schedule"] = args.schedule
    if args.lane_groups:
        cfg["lane_groups"] = args.lane_groups
    if cfg:
        tracer.set_config(**cfg)
    exact = args.rcp == "exact"
    want_cpu = (rank == 0 and world == 1 and not args.no_cpu)

    head = run_workload(args.workload, tracer, world, rank, args.steps, args.warmup, exact, want_cpu, args.bvh_cache)
    extras = []
    do_extra = args.extra if args.extra is not None else (world == 1)
    if do_extra:
        for name in EXTRA_N1:
            if name != args.workload:
                r = run_workload(name, tracer, world, rank, args.steps, args.warmup, exact, False, args.bvh_cache)
                extras.append(r)
                log(f"[extra] {name}: {r['value']} Mrays/s (reference {r['reference_mrays']})")

    if rank == 0:
        ref = REFERENCE_MRAYS.get(args.workload)
        line = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(head["value"] / ref, 3) if ref else None,
            "dtype": "f32",
            "data": "synthetic (deterministic stand-in scene with the README triangle count; rays generated on the device)",
            "config": {"workload": args.workload, "scene": workload_spec(args.workload)[0],
                       "scene_tris": head["scene_tris"], "width": workload_spec(args.workload)[1],
                       "height": workload_spec(args.workload)[2], "ray_type": workload_spec(args.workload)[3],
                       "rays_per_gpu": head["rays_counted"], "rcp": args.rcp,
                       "parallelism": (f"rays sharded by pixel sample x{world}, BVH replicated "
                                       f"(weak: one {workload_spec(args.workload)[1]}x{workload_spec(args.workload)[2]} "
                                       f"sample per GPU, no collective in the step)"),
                       "tracer": tracer.config()},
            "roofline": head["roofline"],
            "cpu_baseline": head.get("cpu_baseline"),
            "detail": {k: head[k] for k in ("kernel_ms_per_launch", "rays_traced", "mrays_traced_per_s", "bvh",
                                            "per_ray", "reference_mrays", "rays_counted_all_ranks", "gather")},
            "extra_workloads": [{k: r[k] for k in ("workload", "value", "reference_mrays", "kernel_ms_per_launch",
                                                   "rays_counted", "rays_traced", "per_ray", "roofline", "bvh")}
                                for r in extras],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
