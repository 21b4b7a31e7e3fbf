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
                  [--readme-cells default|all|none] [--scaling weak|strong]

Multi-GPU (one rank per GPU, RCCL): under torch.distributed.run (WORLD_SIZE set)
every process is one rank; `python bench.py --gpus N` without a launcher starts
its N ranks itself as child processes before any GPU call (launch_ranks), relays
rank 0's line and exits non-zero if any rank failed. Rank 0 builds the
SBVH and broadcasts the Compact2 buffers, which stay in HBM (the BVH is
replicated). Two scalings are measured in every run:

  * strong (BASELINE configs[4]; the line's value at N > 1): ONE
    fixed RayBuffer — hairball diffuse 1920x1080 x 8 spp = 16.6 M rays, generated
    as the reference's Renderer does in <= 2^21-ray batches (Renderer.cc:46,
    RayGen.cc:124-142) — cut into block-cyclic shards (1 024-ray blocks dealt
    round-robin to the ranks; --strong-balance 1 deals them by live-ray count, 2 by the
    next frame's traversal cost),
    each shard's blocks ordered live rays first (--strong-order; T_1's buffer
    too), each traced in <= 2^21-ray launches with no collective; T_n = max over
    ranks. T_1 is measured in the same run (rank 0
    traces the whole buffer alone), eta(n) = T_1 / (n T_n), with and without the
    RCCL gather of the {id, t} results to rank 0.
  * weak (the line's value at N = 1, BASELINE configs[1]; a sub-block at N > 1):
    the N-GPU job is N samples per pixel of the workload's view, rank r tracing
    sample r (rank 0's are the reference's pixel-centre rays, rank r > 0 the r-th
    Halton (2,3) point in each pixel).

Rank 0 prints one JSON line (kept under 10 kB: the headline, its roofline and CPU
baseline, strong scaling, a few numbers per extra workload and, at N = 1, the other
README cells with their ratio to the README and the oracle's agreement); the full
per-workload detail goes to --detail-out.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))

METRIC = "Mrays/s (primary/AO/diffuse) at 1/2/4/8 GPUs; achieved HBM GB/s % of peak"
# Ceilings of the cache levels the trace's bytes are served from (MI355X_MICROARCH.md):
HBM_PEAK_GBS = 8000.0    # HBM3E peak (chip-level parameters, §HBM)
MALL_PEAK_GBS = 8600.0   # Infinity Cache, uniformly random rows (§Indexed rows, 38 MB table)
L2_PEAK_GBS = 34500.0    # the eight XCD L2s together (§L2)
LINE_BYTES = 128         # gfx950 L1 and L2 line: one TCP_TCC_READ_REQ / TCC_EA0_RDREQ per line
                         # (tools/ubench_levels.hip, profiles/round3_counter_calibration.md)
MALL_BYTES = 256 << 20   # Infinity Cache: a BVH above this streams from HBM
PROFILE_TAGS = ("round6", "round5", "round4")   # committed rocprofv3 summaries the line may cite, newest first
                                      # (profiles/<tag>_<workload>_*): only one of the timed schedule is cited
PROFILE_RATIO = (0.9, 1.1)   # a cited profile's mean kernel time / this run's event time must lie in here
LATENCY_BOUND = 0.25         # every memory level served below this fraction of its ceiling: bound = "latency"
LINE_MAX_BYTES = 10_000  # the driver parses one stdout line; round 3's 21.7 kB line was not parsed
STORE = None             # mrt.schedules.ScheduleStore the tracer's schedules are locked from (main())
LEARNED = None           # ScheduleStore collecting the schedules this run settled (--save-schedules)

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
    "fairy-ao-640x480": ("fairy", 640, 480, "ao", 1),
    "fairy-diffuse-640x480": ("fairy", 640, 480, "diffuse", 1),
    "dragon-primary-640x480": ("dragon", 640, 480, "primary", 1),
    "sibenik-diffuse-640x480": ("sibenik", 640, 480, "diffuse", 1),
    "sibenik-ao-640x480": ("sibenik", 640, 480, "ao", 1),
    "san-diffuse-640x480": ("san", 640, 480, "diffuse", 1),
    "san-ao-640x480": ("san", 640, 480, "ao", 1),
    "hairball-primary-640x480": ("hairball", 640, 480, "primary", 1),
    "hairball-diffuse-640x480": ("hairball", 640, 480, "diffuse", 1),
    "hairball-diffuse-1920x1080": ("hairball", 1920, 1080, "diffuse", 1),
}
HEADLINE = "bunny-primary-1024x768"
# (Mori AO and Fairy AO: the two README cells furthest from their targets, VERDICT r4 #7, measured by every bench run)
EXTRA_N1 = ["bunny-primary-640x480", "conference-ao-640x480", "sponza-diffuse-640x480", "sponza-diffuse2-640x480",
            "hairball-diffuse-640x480", "hairball-diffuse-1920x1080", "mori-ao-640x480", "fairy-ao-640x480"]
# The other README cells (README.md:61-81) a default N = 1 run measures too, so that the driver's own run checks
# them (14 of 17 cells were measured only by tools/readme_table.py): timed steps with the schedule
# saved for the BVH or settled by the autotuner in the warmup, and the oracle's agreement. Since round 6 (VERDICT
# r5 #5) San Miguel's two cells too: its 10.5 M-triangle SBVH is built once per run on the host (about a minute
# on the box's 16 threads), like the hairball's, so all 17 README cells are in the driver's own run.
README_N1 = ["sponza-primary-640x480", "sponza-ao-640x480", "mori-primary-640x480", "mori-diffuse-640x480",
             "hairball-primary-640x480", "dragon-primary-640x480", "conference-diffuse-640x480",
             "fairy-diffuse-640x480", "sibenik-diffuse-640x480", "sibenik-ao-640x480",
             "san-diffuse-640x480", "san-ao-640x480"]
README_ALL = README_N1
# Strong-scaling config: scene, frame, samples per pixel, rays per launch.
# min_launches: a shard is cut into at least this many launches (alternating over two streams).
STRONG = {"name": "hairball-diffuse-1920x1080x8spp", "scene": "hairball", "w": 1920, "h": 1080, "spp": 8,
          "max_batch": 1 << 21, "min_launches": 1, "block": 1 << 10, "streams": 2, "balance": 0,
          "order": 1}
STRONG_PROJECT = (2, 4, 8)   # N=1 only: rank counts whose per-rank shards are timed on the one GPU


def workload_spec(name):
    """WORKLOADS entry, or a parsed '<scene>-<primary|ao|diffuse|diffuseN>-<W>x<H>' name."""
    if name in WORKLOADS:
        return WORKLOADS[name]
    scene, kind, res = name.split("-")
    w, h = (int(v) for v in res.split("x"))
    bounces = int(kind[7:]) if kind.startswith("diffuse") and len(kind) > 7 else 1
    return (scene, w, h, kind.rstrip("0123456789"), bounces)


def pmc_profile(name, rcp="exact"):
    """rocprofv3 PMC summary of a workload (one counter group per pass,
    tools/profile_round.sh + tools/summarize_prof.py): counters cannot be read
    inside this timed process, so the committed profile of the same command is
    cited. Per launch: bytes the L1s requested from L2 (TCP_TCC_READ_REQ lines),
    bytes L2 read over the fabric (TCC_EA0_RDREQ lines: Infinity Cache or HBM) and
    wrote (WRITE_SIZE), the mean kernel duration and the schedule it ran."""
    tag = "" if rcp == "exact" else "_rcpfast"
    found = []
    for ptag in PROFILE_TAGS:
        path = os.path.join("profiles", f"{ptag}_{name}{tag}_pmc_summary.json")
        if os.path.exists(os.path.join(REPO, path)):
            with open(os.path.join(REPO, path)) as f:
                s = json.load(f)
            s["path"] = path
            found.append(s)
    return found


def log(*a):
    print(*a, file=sys.stderr, flush=True)


LINE_OUT = None   # the stream the one JSON line goes to (reserve_line_stdout)


def reserve_line_stdout():
    """Keep the process's stdout for the one JSON line: the original fd 1 is kept for
    it and fd 1 itself becomes stderr, so whatever libraries print there (gloo's
    "[Gloo] Rank r is connected to ..." lines, runtime banners) cannot end up next to
    the line the driver parses."""
    global LINE_OUT
    if LINE_OUT is None:
        sys.stdout.flush()
        keep = os.dup(1)
        os.dup2(2, 1)
        LINE_OUT = os.fdopen(keep, "w")
    return LINE_OUT


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Host threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS is set
    to it on the GPU boxes; os.cpu_count() reports the whole machine there)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", "16"))))


# ----------------------------------------------------------------------------- setup
DIST_BACKEND = "nccl"


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, script=None, poll_s=0.2, grace_s=30.0):
    """`--gpus N` (N > 1) without a launcher (no WORLD_SIZE in the environment): start
    N ranks of `script` (this file) as child processes with the torch.distributed.run
    environment — RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a
    free port — one per GPU. The parent never touches the GPU (it is called before
    anything imports the tracer) and never execs: it waits for its children, which
    inherit its stdout, so rank 0's line is the parent's line. When a rank fails the
    others are terminated (SIGTERM, then SIGKILL after grace_s: a rank blocked in a
    collective on a dead peer would wait forever) and its exit code is returned;
    0 when every rank succeeded. SIGTERM/SIGINT to the parent are passed on."""
    import signal
    import subprocess
    script = os.path.abspath(script or __file__)
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_signal(signum, _frame):
        stop_all(signum)
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                log(f"[launch] rank {procs.index(bad[0])} exited with {rc}: stopping the other ranks")
                stop_all()
                t0 = time.time()
                while any(p.poll() is None for p in procs) and time.time() - t0 < grace_s:
                    time.sleep(poll_s)
                stop_all(signal.SIGKILL)
                break
            time.sleep(poll_s)
        for p in procs:
            p.wait()
        if rc == 0:   # every rank ended within one poll: report the first failure here
            failed = [r for r, p in enumerate(procs) if p.returncode != 0]
            if failed:
                rc = procs[failed[0]].returncode
                log(f"[launch] rank {failed[0]} exited with {rc}" + (f" (ranks {failed} failed)" if len(failed) > 1 else ""))
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc if rc > 0 else (1 if rc else 0)


def dist_setup(n_gpus, backend="nccl"):
    """One process per GPU. backend "nccl" is RCCL; "gloo" (CPU collectives) is
    only for rehearsing the N>1 flow with several ranks on one GPU."""
    global DIST_BACKEND
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world} (a launcher started this process for another "
                         f"world size)")
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


def reduce_over_ranks(x, world, op="max"):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if DIST_BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "sum": dist.ReduceOp.SUM}[op])
    return float(t.item())


def gather_floats(x, world):
    """x from every rank, in rank order (on every rank)."""
    if world == 1:
        return [x]
    import torch
    import torch.distributed as dist
    dev = "cuda" if DIST_BACKEND == "nccl" else "cpu"
    out = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(out, torch.tensor([x], dtype=torch.float64, device=dev))
    return [float(t.item()) for t in out]


class SceneCache:
    """Scenes and their Compact2 BVHs, built once per process. Rank 0 builds the
    SBVH (or loads it from cache_dir: the reference's bvhcache idea,
    Renderer.cc:157-217, keyed here by the scene and the builder library's bytes
    so a rebuilt builder never reads a stale file); the buffers are broadcast
    over RCCL and stay in HBM on every rank."""

    def __init__(self, world, rank, cache_dir=None):
        self.world, self.rank, self.cache_dir = world, rank, cache_dir
        self.entries = {}
        self._builder_key = None

    def builder_key(self):
        if self._builder_key is None:
            from mrt import _lib
            with open(_lib.HOST_LIB_PATH, "rb") as f:
                self._builder_key = hashlib.sha1(f.read()).hexdigest()[:12]
        return self._builder_key

    def get(self, scene_name):
        if scene_name in self.entries:
            return self.entries[scene_name]
        import mrt
        from mrt.schedules import bvh_fingerprint
        from mrt.tracer import GpuBvh
        scene = mrt.Scene.synthetic(scene_name, 0, 1)
        t0 = time.perf_counter()
        bufs, stats, cached = None, None, False
        if self.rank == 0:
            path = (os.path.join(self.cache_dir, f"{scene_name}-{self.builder_key()}.dat")
                    if self.cache_dir else None)
            if path and os.path.exists(path):
                bvh, cached = mrt.Bvh.load(path), True
            else:
                bvh = mrt.Bvh.build(scene)
                if path:
                    os.makedirs(self.cache_dir, exist_ok=True)
                    tmp = f"{path}.{os.getpid()}.tmp"
                    bvh.save(tmp)
                    os.replace(tmp, path)
            bufs, stats = bvh.buffers(), bvh.stats()
            del bvh
        build_s = time.perf_counter() - t0
        if self.world > 1:
            from mrt.dist import replicate_buffers
            bufs = tuple(replicate_buffers(bufs, src=0))
        gbvh = GpuBvh(bufs)   # device tensors from RCCL are bound in place; gloo/numpy are uploaded
        gbvh.fingerprint = bvh_fingerprint(*bufs)   # the key of the BVH's saved schedules (mrt/schedules.py)
        entry = {"scene": scene, "gbvh": gbvh, "stats": stats, "build_s": build_s, "cached": cached,
                 "host_bufs": bufs if self.rank == 0 and self.world == 1 else None}
        self.entries[scene_name] = entry
        return entry

    def host_buffers(self, scene_name):
        """(nodes, woop, triIndex) as numpy on this rank (for the CPU baseline)."""
        e = self.get(scene_name)
        if e["host_bufs"] is not None:
            return e["host_bufs"]
        g = e["gbvh"]
        return g.nodes.cpu().numpy(), g.woop.cpu().numpy(), g.tri_index.cpu().numpy()


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


def mrt_seed(bounce):
    import mrt
    return mrt.AO_SEED + bounce


def bind(tracer, gbvh):
    """set_bvh, then lock the BVH's saved schedules (bind forgets them). Returns the
    bind's wall ms (wide-node derivation included) and how many schedules were locked."""
    tracer.set_bvh(gbvh)
    ms = tracer.bind_info()["bind_ms"]
    n = STORE.apply(tracer, gbvh.fingerprint) if STORE is not None else 0
    return ms, n


class Batches:
    """Ray batches of one workload, generated on the device like the reference
    Renderer (Renderer.cc:112-152,242-291; RayGen.cc:50-120): primary rays in
    Morton order; AO/diffuse rays from the traced primary hits (degenerate
    tmax=-1 rays for misses are traced too; only primary hits are counted).
    "diffuseN" chains N bounces, each generated from the previous bounce's hits."""

    def __init__(self, name, scene, gbvh, tracer, rank=0):
        from mrt.raygen import DeviceRayGen
        sname, w, h, kind, bounces = workload_spec(name)
        self.name, self.kind, self.w, self.h = name, kind, w, h
        self.bind_ms, self.locked_from_store = bind(tracer, gbvh)
        cam, ao_radius = scene.camera()
        gen = DeviceRayGen(scene)   # RayGen on the device (mrt_raygen_*), like the reference's RayGenKernels
        prim, _ = gen.primary(cam, w, h, subpixel=subpixel_sample(rank))
        self.primary = prim
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


def algorithmic_bytes(tracer, batches):
    """B_ray = 32 + 8 + 64 N_node + 48 N_tri + 16 N_leaf + 4 [hit],
    with the per-ray counts of the single-ray traversal order (the kernel's
    per-lane mode, which reproduces the CPU restatement's counters exactly)."""
    import torch
    total, nodes, tris, leaves = 0, 0, 0, 0
    for rb, _ in batches:
        saved = rb.results.clone()
        tracer.trace_batch(rb, exact_rcp=True, speculative=False, stats=True)
        s = rb.stats.to(torch.int64)
        hits = (rb.results[:, 0] != -1).to(torch.int64).sum().item()
        n, t, l = (s[:, 0].sum().item(), s[:, 1].sum().item(), s[:, 2].sum().item())
        nodes, tris, leaves = nodes + n, tris + t, leaves + l
        total += 40 * rb.size + 64 * n + 48 * t + 16 * l + 4 * hits
        rb.results.copy_(saved)
        rb.stats = None
    return total, nodes, tris, leaves


def kernel_bytes(tracer, batches):
    """The bytes the PRODUCTION traversal reads per launch, next to
    SURVEY §8(d)'s binary-order figure: the speculative kernel's STATS variant counts
    its own 4-wide node visits, triangle tests and leaf ends (bit-identical closest
    hits; the STATS launch runs the fixed-rule schedule, so the counts of other
    schedules differ by the frontier tail's few extra visits). Per ray:
    32 (ray) + 8 (result) + 128 N_wide + 48 N_tri + 4 [hit] — the wide leaf refs carry
    their triangle counts, so no terminator slot is read. Returns (bytes, nodes, tris)."""
    import torch
    total, nodes, tris = 0, 0, 0
    for rb, _ in batches:
        saved = rb.results.clone()
        tracer.trace_batch(rb, exact_rcp=True, speculative=True, stats=True)
        li = tracer.last_info   # node_bytes: 128 for the 4-wide lines, 64 for Compact2 (wide nodes off)
        s = rb.stats.to(torch.int64)
        hits = (rb.results[:, 0] != -1).to(torch.int64).sum().item()
        n, t, lv = s[:, 0].sum().item(), s[:, 1].sum().item(), s[:, 2].sum().item()
        nodes, tris = nodes + n, tris + t
        term = 16 * lv if li["wide"] != 4 else 0   # binary leaves end on a -0.0 terminator slot
        total += 40 * rb.size + li["node_bytes"] * n + 48 * t + term + 4 * hits
        rb.results.copy_(saved)
        rb.stats = None
    return total, nodes, tris


def joined(launches):
    """The launches of one step, as one callable. When they span several streams the
    step is a frame: its other streams wait for everything enqueued on the first
    before the step's launches, and the first waits for them after, so consecutive
    steps never overlap (a step's launches still overlap each other)."""
    import torch
    streams = []
    for go in launches:
        if all(go.stream != s for s in streams):
            streams.append(go.stream)
    if len(streams) < 2:
        def step():
            for go in launches:
                go()
        return step
    head, rest = streams[0], streams[1:]

    def step():
        ev = torch.cuda.Event()
        ev.record(head)
        for s_ in rest:
            s_.wait_event(ev)
        for go in launches:
            go()
        for s_ in rest:
            e_ = torch.cuda.Event()
            e_.record(s_)
            head.wait_event(e_)
    return step


def warm(launches, warmup, min_seconds=0.3):
    """At least `warmup` steps and at least min_seconds of back-to-back launches, so
    the timed steps never run on ramping clocks (a 20-step default on 0.15 ms steps
    measured 4.8-5.3 G rays/s against 5.35 G once the clocks settle)."""
    import torch
    step = joined(launches)
    t0, done = time.perf_counter(), 0
    while done < warmup or time.perf_counter() - t0 < min_seconds:
        step()
        done += 1
        if done % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return done


def time_steps(launches, steps, warmup, world):
    """Warmup, then exactly `steps` steps bracketed by barrier + synchronize; wall
    time of the K steps (a multi-stream step is joined: see joined()). Then a probe
    pass: the average launch duration, from one HIP event pair on the launch stream
    around back-to-back launches (several streams: every launch bracketed by its own
    pair, one at a time)."""
    import torch
    warmed = warm(launches, warmup)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    step = joined(launches)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    probe = max(3, min(steps, 50))
    one_stream = all(go.stream == launches[0].stream for go in launches)
    if one_stream:
        # one event pair around `probe` back-to-back steps on the launch stream: an event
        # recorded between launches fences the caches (a system-scope release), so
        # bracketing every launch would time each one from cold caches
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record(launches[0].stream)
        for _ in range(probe):
            for go in launches:
                go()
        b_.record(launches[0].stream)
        torch.cuda.synchronize()
        return wall, a_.elapsed_time(b_) / (probe * len(launches)), warmed
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(probe * len(launches))]
    k = 0
    for _ in range(probe):
        for go in launches:
            ev[k][0].record(go.stream)
            go()
            ev[k][1].record(go.stream)
            k += 1
            torch.cuda.synchronize()   # one launch at a time: its own duration, not an overlap
    torch.cuda.synchronize()
    per_launch = [a.elapsed_time(b) for a, b in ev]
    return wall, float(np.mean(per_launch)), warmed


def gather_to_root(batches, world):
    """The hit-result gather that follows a sharded trace: every
    rank's RayResult {id, t} of each batch to rank 0, RCCL point-to-point
    (mrt/dist.py). Returns (ms, bytes received by rank 0)."""
    import torch
    from mrt.dist import gather_results
    # one untimed pass first: RCCL creates its point-to-point communicators on first use
    for rb, _ in batches.batches:
        gather_results(rb.results if DIST_BACKEND == "nccl" else rb.results.cpu(), world * rb.size)
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
    return reduce_over_ranks(ms, world), nbytes


def cpu_baseline(batches, bufs, counted, threads, label, fast_results=None):
    """The oracle (oracle/, a scalar C restatement of the same traversal, one ray at a
    time, std::thread-style dynamic chunks) on the host cores over every batch of the
    workload: best of 5 after 1 warmup. Also checks the GPU results against it
    (parity on the bench input: closest hit bit-identical, any hit hit/miss-identical)
    and, given the fast-reciprocal mode's results, classifies their mismatches
    (SURVEY §8(a) Note 3: tie / edge / other, tests/oracle_lib.classify_fast_rcp). An
    any-hit ray agrees when its hit/miss is the oracle's and, where its {id, t} differs,
    the reported triangle passes the oracle's Woop test with exactly that t
    (oracle_lib.invalid_hits: "valid hits", the reference's own any-hit contract)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    nodes, woop, tri = bufs
    host = [(rb.rays.cpu().numpy(), not rb.need_closest_hit, rb.results_numpy()) for rb, _ in batches]
    secs, agree, n, any_checked, ties = [], 0, 0, 0, 0
    fast = {"rays": 0, "mismatch": 0, "tie": 0, "edge": 0, "other": 0, "any_hit_outcome_flips": 0,
            "any_hit_invalid": 0} if fast_results is not None else None
    for rep in range(6):
        total = 0.0
        for b, (rays, any_hit, gpu) in enumerate(host):
            res, _, s = O.trace(rays, nodes, woop, tri, any_hit=any_hit, threads=threads)
            total += s
            if rep == 0:
                same = (gpu[:, 0] == res[:, 0]) & (gpu[:, 1] == res[:, 1])
                if any_hit:   # any valid hit is the reference's contract: re-verify every differing one
                    diff = np.nonzero(~same)[0]
                    bad = O.invalid_hits(rays, gpu, woop, tri, which=diff)
                    same = (gpu[:, 0] == -1) == (res[:, 0] == -1)
                    same[bad] = False
                    any_checked += len(diff)
                else:   # another triangle at exactly the oracle's t: a tie the traversal order breaks
                    t_eq = np.nonzero(~same & (gpu[:, 1] == res[:, 1]))[0]
                    ties += len(t_eq) - len(O.invalid_hits(rays, gpu, woop, tri, which=t_eq))
                agree += int(same.sum())
                n += len(rays)
                if fast is not None:
                    fr = fast_results[b]
                    fast["rays"] += len(rays)
                    if any_hit:   # hit/miss flips, classified edge / other like the closest-hit mismatches
                        c = O.classify_any_hit_flips(rays, fr, res, woop, tri)
                        fast["any_hit_outcome_flips"] += c["flips"]
                        fast["edge"] += c["edge"]
                        fast["other"] += c["other"]
                        fd = np.nonzero((fr[:, 0] != res[:, 0]) | (fr[:, 1] != res[:, 1]))[0]
                        fast["any_hit_invalid"] += len(O.invalid_hits(rays, fr, woop, tri, which=fd, rcp_ulps=1))
                    else:
                        c = O.classify_fast_rcp(rays, fr, res, woop, tri)
                        for k in ("mismatch", "tie", "edge", "other"):
                            fast[k] += c[k]
        if rep:
            secs.append(total)
    best = min(secs)
    rays = sum(len(r) for r, _, _ in host)
    out = {"value": round(counted / best / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "seconds_best": round(best, 4),
           "sample": f"{label}: all {len(host)} batch(es), {rays} rays ({counted} counted), best of 5 after 1 "
                     f"warmup, {threads} threads, oracle/trace_oracle.c (same Compact2 bytes, same rays)",
           "parity_exact_fraction": round(agree / max(1, n), 6), "parity_rays": n, "parity_same": agree,
           "closest_hit_exact_t_ties": ties, "any_hit_valid_hits_checked": any_checked}
    if fast is not None:
        fast["tie_fraction"] = round(fast["tie"] / max(1, fast["rays"]), 8)
        out["rcp_fast_parity"] = fast
    return out


def roofline(name, alg_bytes_per_launch, kernel_ms, bvh_bytes, schedule, rcp="exact", kernel_bytes_per_launch=None):
    """Roofline of the dominant kernel, as the bench contract defines it: achieved =
    the ALGORITHMIC bytes of SURVEY.md §8(d) per launch (every byte the rays read, from
    the per-ray node/triangle/leaf counts) / this run's HIP-event kernel time, against
    the 8 TB/s HBM peak; traffic = the bytes the L2s moved over the fabric per launch
    (rocprofv3 TCC_EA0_RDREQ x 128 B + WRITE_SIZE, calibrated on gfx950 in
    profiles/round3_counter_calibration.md; Infinity-Cache hits included, so an upper
    bound on HBM bytes), hbm_measured_frac = traffic / time / 8 TB/s. Cache-resident
    scenes read most algorithmic bytes from L1/L2, so `frac` can pass 1 there (stated,
    not clamped: SURVEY §8d). `served` prices what each level actually moved against its
    own ceiling (L1->L2 requests / 34.5 TB/s; fabric / 8.6 TB/s, the Infinity Cache's
    random-row rate) and names the larger as `binding_level`. The cited profile must
    have run the timed schedule (autotune candidate and its name, grid, queues) or none is cited,
    and its mean kernel time must lie within PROFILE_RATIO of this run's.

    kernel_bytes_per_launch (kernel_bytes(): what the production 4-wide traversal reads)
    gives `kernel_achieved` / `kernel_frac` beside the binary-order §8(d) figure. `bound` is
    read from the served fractions, not assumed: "latency" when every level serves under
    LATENCY_BOUND of its ceiling (dependent fetches of a few lanes per wave, not bandwidth),
    else "hbm" (the fabric) or "l2" as the binding level; "hbm" when no profile is cited."""
    t = kernel_ms * 1e-3
    alg = alg_bytes_per_launch / t / 1e9
    out = {"bound": "hbm", "achieved": round(alg, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(alg / HBM_PEAK_GBS, 4), "traffic": None,
           "basis": "SURVEY 8(d) algorithmic bytes per launch / HIP-event kernel time; traffic = PMC fabric bytes",
           "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": int(alg_bytes_per_launch),
           "bvh_bytes": int(bvh_bytes), "bvh_exceeds_mall": bvh_bytes > MALL_BYTES}
    if kernel_bytes_per_launch:
        kb = kernel_bytes_per_launch / t / 1e9
        out.update({"kernel_bytes_per_launch": int(kernel_bytes_per_launch), "kernel_achieved": round(kb, 1),
                    "kernel_frac": round(kb / HBM_PEAK_GBS, 4)})
    if alg > HBM_PEAK_GBS:
        out["note"] = "algorithmic rate above the HBM peak: the BVH is cache-resident (L1/L2 hits)"
    # the schedule's name too: it spells out what the candidate number means in this build (queue blocks, ...)
    want = {k: schedule.get(k) for k in ("autotune_candidate", "name", "grid_waves", "num_queues", "fetch_threshold")}
    profs = pmc_profile(name, rcp)
    prof = next((p for p in profs if {k: (p.get("schedule") or {}).get(k) for k in want} == want), None)
    if prof is None:
        out["profile"] = {"note": f"no committed PMC profile of the timed schedule {want}",
                          "seen": [p["path"] for p in profs]}
        return out
    ratio = prof["avg_ns"] / 1e6 / kernel_ms
    if not PROFILE_RATIO[0] <= ratio <= PROFILE_RATIO[1]:
        # same schedule, but the profiled launch ran at another speed (e.g. the gloo rehearsal's
        # ranks sharing one GPU): its bytes per launch would be priced against the wrong time
        out["profile"] = {"note": f"{prof['path']} not cited: its mean kernel time is {ratio:.3f}x this run's "
                                  f"(outside {PROFILE_RATIO})", "kernel_ms_ratio": round(ratio, 4)}
        return out
    lv = prof["levels"]
    levels = {"l2": (lv["l2_request_bytes"], L2_PEAK_GBS), "fabric": (lv["fabric_bytes"], MALL_PEAK_GBS)}
    fr = {k: b / t / 1e9 / peak for k, (b, peak) in levels.items()}
    out.update({"traffic": int(lv["fabric_bytes"]),
                "hbm_measured_GBps": round(lv["fabric_bytes"] / t / 1e9, 1),
                "hbm_measured_frac": round(lv["fabric_bytes"] / t / 1e9 / HBM_PEAK_GBS, 4),
                "served": {k: {"bytes_per_launch": int(levels[k][0]), "GBps": round(levels[k][0] / t / 1e9, 1),
                               "peak_GBps": levels[k][1], "frac": round(fr[k], 4)} for k in levels},
                "binding_level": max(fr, key=fr.get),
                "bound": ("latency" if max(fr.values()) < LATENCY_BOUND
                          else ("hbm" if max(fr, key=fr.get) == "fabric" else "l2")),
                "l1_hit_fraction_of_algorithmic": round(max(0.0, 1.0 - lv["l2_request_bytes"] / alg_bytes_per_launch), 4),
                "l2_hit_rate": prof.get("l2_hit_rate"),
                **({"vmem_frac": round(max(prof["vmem"]["ta_busy_frac"], prof["vmem"]["td_busy_frac"]), 4),
                    "vmem": {k: round(v, 4) for k, v in prof["vmem"].items() if k.endswith("frac")}}
                   if prof.get("vmem") else {}),
                "profile": {"path": prof["path"], "kernel_ms": round(prof["avg_ns"] / 1e6, 4),
                            "kernel_ms_ratio": round(prof["avg_ns"] / 1e6 / kernel_ms, 4)}})
    # the unit the traversal actually saturates, priced against its own ceiling: the
    # vector-memory path (TA address / TD data units busy per CU cycle), the L2 or the fabric
    units = {"l2": fr["l2"], "fabric": fr["fabric"]}
    if out.get("vmem_frac") is not None:
        units["vmem"] = out["vmem_frac"]
    out["binding_unit"] = max(units, key=units.get)
    out["binding_frac"] = round(units[out["binding_unit"]], 4)
    return out


def exploration_cost(tracer, gbvh, rb, exact, max_launches=1200):
    """What autotuning costs and finds for a caller without saved schedules (VERDICT r2 #5,
    r5 #4): a fresh bind, then back-to-back launches of one batch (as the timed steps run
    them, no blocking) until the library settles its schedule; then the settled and the
    saved schedule each timed by the headline's own probe (HIP events around back-to-back
    launches after a warmup), so `tuned_vs_saved` compares like with like. The saved
    schedules are locked again afterwards."""
    import torch
    tracer.set_bvh(gbvh)   # bind forgets every schedule: the autotuner starts from scratch
    go = tracer.launcher(rb, exact_rcp=exact)

    def settled():
        return [c for n, _, c, _ in tracer.schedules() if n == rb.size]

    t0 = time.perf_counter()
    n = 0
    while n < max_launches and not settled():
        for _ in range(8):
            go()
        n += 8
        torch.cuda.synchronize()   # lets the library read the candidates' event pairs
    explore_s = time.perf_counter() - t0

    def probe(reps=3, k=40):
        for _ in range(20):
            go()
        out = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(k):
                go()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / k)
        return float(np.median(out))

    cand = settled()
    tuned_ms = probe() if cand else None
    bind(tracer, gbvh)   # the saved schedules again
    saved = [c for n_, _, c, _ in tracer.schedules() if n_ == rb.size]
    saved_ms = probe() if saved else None
    if not cand:
        return {"locked": False, "launches": n}
    out = {"locked": True, "launches_to_lock": n, "exploring_s": round(explore_s, 3),
           "explored_candidate": cand[0], "explored_schedule": schedule_name(cand[0]),
           "settled_ms_each": round(tuned_ms, 4)}
    if saved_ms:
        out.update({"saved_candidate": saved[0], "saved_ms_each": round(saved_ms, 4),
                    "tuned_vs_saved": round(tuned_ms / saved_ms, 4)})
    return out


# cfg.autotune candidates (csrc/mrt_api.cpp tune_candidate)
SCHEDULES = {0: "static rounds, 20 waves/CU", 1: "static rounds, 8 waves/CU",
             2: "8 per-XCD queues of 8192-ray blocks, refill at 56, 20 waves/CU",
             3: "global queue, refill at 48, 16 waves/CU", 4: "global queue, refill at 48, 12 waves/CU",
             5: "static rounds, 16 waves/CU", 6: "static rounds, 12 waves/CU",
             7: "global queue, refill at 48, 20 waves/CU"}


def schedule_name(c):
    """mrt_trace_info.autotune_candidate: 0-7 a schedule, 8/9/10/11/12 (| stage-1 schedule << 8) that
    schedule with spec_slack 4/6, the frontier tail toggled, 16 lane groups, or 2 lane groups with spec_slack 6
    (the tail: off, since the library's default has it on, include/mrt.h tail_lanes); -1 the fixed rule
    (autotune off, distribution knobs set by the caller, or a batch size launched on several streams before a
    schedule settled for it — a settled, saved or inherited schedule runs on every stream, mrt_api.cpp)."""
    if c < 0:
        return "fixed rule"
    if (c & 0xff) >= 8:
        return f"{SCHEDULES[c >> 8]}, " + {8: "spec_slack 4", 9: "spec_slack 6", 10: "no frontier tail", 11: "16 lane groups",
                                            12: "2 lane groups, spec_slack 6"}[c & 0xff]
    return SCHEDULES[c & 0xff]   # (an exported stage-1 choice carries its own number in the stage-1 byte)


def schedule_of(tracer, rb, exact):
    """The schedule a batch's launches run on: one more blocking launch, outside the timed region."""
    tracer.trace_batch(rb, exact_rcp=exact)
    li = tracer.last_info
    return {"autotune_candidate": li["autotune_candidate"], "autotune_locked": li["autotune_locked"],
            "name": schedule_name(li["autotune_candidate"]), "num_queues": li["num_queues"],
            "fetch_threshold": li["fetch_threshold"], "grid_waves": li["grid_waves"]}


def readme_cell(name, tracer, scenes, steps, warmup, exact, want_cpu):
    """One README cell at N = 1 (README_N1): the workload's batches timed like a bench step,
    its schedule, and — in the cpu_baseline leg — the oracle's agreement on every ray."""
    scene_name = workload_spec(name)[0]
    e = scenes.get(scene_name)
    batches = Batches(name, e["scene"], e["gbvh"], tracer, 0)
    launches = [tracer.launcher(rb, exact_rcp=exact) for rb, _ in batches.batches]
    wall, launch_ms, _ = time_steps(launches, steps, warmup, 1)
    value = batches.rays_counted * steps / wall / 1e6
    sched = schedule_of(tracer, batches.batches[0][0], exact)
    ref = REFERENCE_MRAYS[name]
    out = {"cell": name, "value": round(value, 1), "x_readme": round(value / ref, 2), "kernel_ms": round(launch_ms, 4),
           "schedule": sched["name"], "saved": bool(batches.locked_from_store)}
    if want_cpu:
        cb = cpu_baseline(batches.batches, scenes.host_buffers(scene_name), batches.rays_counted, host_threads(),
                          name)
        out["agree"] = cb["parity_exact_fraction"]   # any hit: hit/miss identical and every differing hit valid
        if cb["closest_hit_exact_t_ties"]:
            out["ties"] = cb["closest_hit_exact_t_ties"]
        out["cpu"] = cb["value"]
    return out


def run_workload(name, tracer, scenes, world, rank, steps, warmup, exact, want_cpu, explore=False, fast=False):
    scene_name = workload_spec(name)[0]
    e = scenes.get(scene_name)
    batches = Batches(name, e["scene"], e["gbvh"], tracer, rank)
    alg_bytes, n_nodes, n_tris, n_leaves = algorithmic_bytes(tracer, batches.batches)
    k_bytes, k_nodes, k_tris = kernel_bytes(tracer, batches.batches)
    launches = [tracer.launcher(rb, exact_rcp=exact) for rb, _ in batches.batches]
    wall, launch_ms, warmed = time_steps(launches, steps, warmup, world)
    wall = reduce_over_ranks(wall, world)
    launch_ms = reduce_over_ranks(launch_ms, world)
    counted = int(reduce_over_ranks(batches.rays_counted, world, "sum"))
    traced = int(reduce_over_ranks(batches.rays_traced, world, "sum"))
    alg_bytes = reduce_over_ranks(alg_bytes, world, "sum") / world   # per-GPU bytes (mean over ranks)
    k_bytes = reduce_over_ranks(k_bytes, world, "sum") / world
    value = counted * steps / wall / 1e6
    gather = gather_to_root(batches, world) if world > 1 else None
    # the schedule the launches ran on: saved for this BVH (locked at bind), or settled
    # by the autotuner during the warmup
    schedule = schedule_of(tracer, batches.batches[0][0], exact)
    schedule["source"] = "saved (mrt/tuned_schedules.json)" if batches.locked_from_store else "autotuned in this run"
    if LEARNED is not None:
        LEARNED.update(e["gbvh"].fingerprint, tracer.schedules())
    g = e["gbvh"]
    # the drop-in's default arithmetic (v_rcp_f32, the reference's rcp.approx analogue)
    fast_block, fast_results = None, None
    if fast:
        fl = [tracer.launcher(rb, exact_rcp=False) for rb, _ in batches.batches]
        fsteps = max(10, min(steps, 100))
        fwall, fms, _ = time_steps(fl, fsteps, warmup, world)
        fsched = schedule_of(tracer, batches.batches[0][0], False)
        fast_results = []
        for rb, _ in batches.batches:
            tracer.trace_batch(rb, exact_rcp=False)
            fast_results.append(rb.results_numpy())
            tracer.trace_batch(rb, exact_rcp=exact)   # leave the exact results for the parity check
        fast_block = {"value": round(batches.rays_counted * fsteps / fwall / 1e6, 2), "steps": fsteps,
                      "kernel_ms_per_launch": round(fms, 4), "schedule": fsched,
                      "roofline": roofline(name, alg_bytes / len(batches.batches), fms, g.total_bytes, fsched,
                                           rcp="fast", kernel_bytes_per_launch=k_bytes / len(batches.batches))}
    explored = exploration_cost(tracer, g, batches.batches[0][0], exact) if explore else None
    out = {
        "workload": name,
        "value": round(value, 2),
        "ms_per_step": round(1e3 * wall / steps, 4),
        "kernel_ms_per_launch": round(launch_ms, 4),
        "warmup_steps_run": warmed,
        "rays_counted": batches.rays_counted,
        "rays_traced": batches.rays_traced,
        "mrays_traced_per_s": round(traced * steps / wall / 1e6, 2),
        "rays_counted_all_ranks": counted,
        "gather": ({"ms": round(gather[0], 3), "bytes_to_root": gather[1],
                    "value_incl_gather": round(counted * steps / (wall + steps * gather[0] / 1e3) / 1e6, 2)}
                   if gather else None),
        "scene_tris": e["scene"].num_triangles,
        "bvh": {"inner_nodes": g.nodes.numel() // 16, "woop_slots": g.woop.numel() // 4, "bytes": g.total_bytes,
                "build_s": round(e["build_s"], 2), "from_cache": e["cached"], "bind_ms": round(batches.bind_ms, 2),
                "stack_capacity": tracer.bind_info()["stack_capacity"],
                **({"max_depth": e["stats"]["max_depth"], "sah": round(e["stats"]["sah_cost"], 2)}
                   if e["stats"] and not e["cached"] else {})},
        "per_ray": {"nodes": round(n_nodes / batches.rays_traced, 2), "tris": round(n_tris / batches.rays_traced, 2),
                    "leaves": round(n_leaves / batches.rays_traced, 2),
                    "bytes": round(alg_bytes / batches.rays_traced, 1),
                    "wide_nodes": round(k_nodes / batches.rays_traced, 2),
                    "wide_tris": round(k_tris / batches.rays_traced, 2),
                    "kernel_bytes": round(k_bytes / batches.rays_traced, 1)},
        "schedule": schedule,
        "autotune_exploration": explored,
        "roofline": roofline(name, alg_bytes / len(batches.batches), launch_ms, g.total_bytes, schedule,
                             kernel_bytes_per_launch=k_bytes / len(batches.batches)),
        "reference_mrays": REFERENCE_MRAYS.get(name),
        "rcp_fast": fast_block,
    }
    if want_cpu:
        out["cpu_baseline"] = cpu_baseline(batches.batches, scenes.host_buffers(scene_name), batches.rays_counted,
                                           host_threads(), name, fast_results)
        if fast_block is not None:
            fast_block["parity"] = out["cpu_baseline"].pop("rcp_fast_parity")
    return out


def strong_scaling(tracer, scenes, world, rank, steps, warmup, exact, with_roofline=False):
    """one fixed RayBuffer (the hairball diffuse frame at 8 spp, the
    rays the Renderer's <= 2^21-ray batches hold with their glibc seeds), cut into
    shards — block-cyclic (STRONG["block"]-ray blocks dealt round-robin to the
    ranks) so that every shard samples the whole frame; each rank GENERATES its
    shard on its device in trace order (Renderer.secondary_blocks: the primary pass,
    then only its own blocks' rays, live blocks first — no frame-order buffer, no
    gather) and traces it in <= 2^21-ray launches. T_n = max over ranks; T_1 = rank 0
    tracing the whole frame alone, same run; then the {id, t} gather to rank 0,
    checked against the single-GPU results."""
    import torch
    from mrt.dist import (balance_blocks, block_sums, gather_results, live_block_weights, live_priority,
                          shard_blocks_device, shard_launches, shard_spans, spans_index)
    from mrt.raygen import RAY_DIFFUSE
    from mrt.renderer import GlibcRand, Renderer
    from mrt.tracer import RayBuffer
    cfg = STRONG
    e = scenes.get(cfg["scene"])
    bind(tracer, e["gbvh"])
    cam, _ = e["scene"].camera()
    rnd = GlibcRand()   # the reference's rand() sequence: this frame's batch seeds, then the next frame's
    B = cfg["block"]

    def begin(rand):
        r = Renderer(tracer, e["scene"], max_batch=cfg["max_batch"], exact_rcp=True, rand=rand)
        r.set_params(RAY_DIFFUSE, cfg["spp"])
        r.begin_frame(cam, cfg["w"], cfg["h"])   # the primary pass (traced, untimed: Renderer.cc:137-140)
        r.batch_seeds()                          # this frame's seeds, drawn in batch order
        return r

    def frame_batches(rand):
        # the frame's rays as the Renderer's batches hold them, in frame order (cost order 2's
        # next frame; the check that the generated shards are those rays)
        r = begin(rand)
        parts = [b for b, _ in r.batches()]
        return RayBuffer(torch.cat([b.rays for b in parts]), need_closest_hit=True, secondary=True)

    rend = begin(rnd)
    counted = rend.total_num_rays()
    n = rend.primary.size * cfg["spp"]

    # Blocks dealt by live-ray count (balance_blocks) or cyclically, and within a shard
    # in frame order (order 0), live blocks first (1) or costly blocks first (2). The live
    # count of every block follows from the primary pass (a sample is live iff its primary
    # hit: live_block_weights, one reduction on the device); a host copy serves the deal
    # and the gather's spans (brought over once, so no later shard_spans call syncs the device).
    # Order 2's cost is what a renderer knows from the frame before: the NEXT frame of the
    # same view (the following rand() seeds: the same pixels, other sample directions) is
    # traced once with per-ray counters, and each block's node + triangle visits rank it (the live-ray count ignores how long the live rays are).
    # Balance 2 deals the blocks by that cost instead of the live-ray count (equal work per rank).
    weights_dev = live_block_weights(rend.primary.results, cfg["spp"], B)
    weights = weights_dev.cpu().numpy() if (cfg["balance"] or cfg["order"]) and B > 0 else None
    cost = None
    if (cfg["order"] == 2 or cfg["balance"] == 2) and B > 0:
        other = frame_batches(rnd)
        for a_, b_ in shard_launches(0, other.size, cfg["max_batch"]):
            v = other.view(a_, b_)
            # the per-lane order's counters: deterministic (the oracle's), so every rank derives the same deal
            tracer.trace_batch(v, exact_rcp=exact, speculative=False, stats=True)
            other.stats = v.stats if a_ == 0 else torch.cat([other.stats, v.stats])
        cost = block_sums(other.stats[:, 0] + other.stats[:, 1], B).cpu().numpy()
        del other
    # the host's copy of the order (gather_results' spans): live_priority is mrt_shard_blocks' own key
    prio = {0: None, 1: None if weights is None else live_priority(weights, B), 2: cost}[int(cfg["order"])]
    deals = {}

    def owners_for(k):
        if weights is None or k == 1 or not cfg["balance"]:
            return None
        if k not in deals:
            deals[k] = balance_blocks(cost if cfg["balance"] == 2 else weights, k)
        return deals[k]

    def shard_order(k, rk):
        # rank rk's blocks of a k-rank job in its trace order: the library deals and orders
        # them (cyclic deal; frame order or live blocks first, from the primary results:
        # mrt_shard_blocks); the options it does not deal (balanced deals, the cost order)
        # order the blocks with torch on the device instead
        if cfg["order"] in (0, 1) and not cfg["balance"]:
            return rend.gen.shard_blocks(rend.primary, cfg["spp"], B, k, rk, int(cfg["order"]))
        pd = None if prio is None else torch.from_numpy(np.ascontiguousarray(prio)).to(weights_dev.device)
        return shard_blocks_device(n, k, rk, B, owners_for(k), pd, device=weights_dev.device)

    def shard_buffer(k, rk):
        # ... and those blocks' rays generated in that order (mrt_raygen_ao_blocks)
        blocks, m = shard_order(k, rk)
        return rend.secondary_blocks(blocks, m, B)

    # The shard build — what a rank does between its primary pass and its first trace
    # launch — is timed (max over ranks; device time by events, median of three) in its two
    # parts: the order of its blocks (the sharding's own work: the live count per block
    # from the primary results and a sort) and its rays generated in that order (the ray
    # generation every renderer does, one rank or eight — the reference's Mrays/s leaves it
    # out, and so do T_1 and T_n). VERDICT r5 #1: this replaces round 5's index_select of a
    # frame-order buffer (5.3 ms at N = 1); value_with_gather_and_shard adds the order,
    # value_with_raygen the generation too (and T_1's own generation to eta_with_raygen).
    def build_timed(k, rk):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        torch.cuda.synchronize()
        ts = time.perf_counter()
        ev[0].record()
        blocks, m = shard_order(k, rk)
        ev[1].record()
        buf = rend.secondary_blocks(blocks, m, B)
        ev[2].record()
        torch.cuda.synchronize()
        return buf, (1e3 * (time.perf_counter() - ts), ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]))

    def build_local():
        return build_timed(1, 0) if world == 1 else build_timed(world, rank)

    local, _ = build_local()   # (the first build also pays one-time kernel setup: timed on later ones)
    del local
    times = []
    for _ in range(3):
        barrier(world)
        local, tm = build_local()
        times.append(tm)
        if _ < 2:
            del local
    shard_build_ms, shard_order_ms, raygen_ms = (reduce_over_ranks(float(np.median([x[i] for x in times])), world)
                                                 for i in range(3))
    raygen_ms_n1 = raygen_ms
    if world > 1:   # T_1's generation of the whole frame (rank 0), for eta_with_raygen
        t1gen = []
        if rank == 0:
            for _ in range(3):
                b1, tm = build_timed(1, 0)
                t1gen.append(tm[2])
                del b1
        raygen_ms_n1 = reduce_over_ranks(float(np.median(t1gen)) if rank == 0 else 0.0, world)
    # The generated shard is the frame's rays: rank r's rays equal the Renderer's batches
    # (frame order) at its blocks' positions, bit for bit (checked on every rank).
    ref = torch.cat([b.rays for b, _ in rend.batches()])   # the same frame (primary pass, seeds) batch by batch
    idx = spans_index(shard_spans(n, 1 if world == 1 else world, 0 if world == 1 else rank, B,
                                  owners_for(world), prio), ref.device)
    shard_equal = bool(torch.equal(ref.index_select(0, idx), local.rays))
    del ref, idx
    shard_equal = reduce_over_ranks(1.0 if shard_equal else 0.0, world, op="min") > 0.5
    # The shard's <= 2^21-ray launches are independent batches: they alternate
    # between two streams (each stream has its own trace scratch), so one
    # launch's tail overlaps the next one's start.
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()][:cfg["streams"]]

    def shard_steps(buf, nstreams=len(streams)):
        return [tracer.launcher(buf.view(a, b), exact_rcp=exact, stream=streams[i % nstreams])
                for i, (a, b) in enumerate(shard_launches(0, buf.size, cfg["max_batch"], cfg["min_launches"]))]

    launches = shard_steps(local)
    wall, launch_ms, _ = time_steps(launches, steps, warmup, world)
    # The schedule each distinct launch size of the shard ran (a settled or
    # inherited schedule also runs on the second stream, so the label is read back from
    # the library, not assumed): one more blocking launch per size, after the timed steps.
    spans_l = shard_launches(0, local.size, cfg["max_batch"], cfg["min_launches"])
    scheds = {}
    for a_, b_ in spans_l:
        if b_ - a_ not in scheds:
            scheds[b_ - a_] = schedule_of(tracer, local.view(a_, b_), exact)
    one_stream_ms = None
    if world == 1 and len(streams) > 1:
        # the same launches on one stream: the autotuner's (or saved) schedule applies
        w1s, _, _ = time_steps(shard_steps(local, 1), steps, warmup, 1)
        one_stream_ms = w1s / steps * 1e3
    shard_roofline = None
    if with_roofline:   # the line's roofline at N > 1: this rank's launches (SURVEY §8(d) bytes, per launch)
        views = [(local.view(a, b), 0) for a, b in spans_l]
        alg, _, _, _ = algorithmic_bytes(tracer, views)
        kb, _, _ = kernel_bytes(tracer, views)
        sched = scheds[spans_l[0][1] - spans_l[0][0]]
        shard_roofline = roofline(f"{cfg['scene']}-diffuse-{cfg['w']}x{cfg['h']}", alg / len(views), launch_ms,
                                  e["gbvh"].total_bytes, sched, kernel_bytes_per_launch=kb / len(views))
        shard_roofline["note"] = (f"rank {rank}'s {len(views)} launches of <= {cfg['max_batch']} rays on "
                                  f"{len(streams)} streams; kernel_ms = one launch alone")
    per_rank = gather_floats(wall / steps * 1e3, world)
    tn = max(per_rank)
    # gather of this shard's {id, t} to rank 0 (RCCL point-to-point; gloo: via host),
    # after one untimed gather (RCCL creates its point-to-point communicators on first use)
    if world > 1:
        gather_results(local.results if DIST_BACKEND == "nccl" else local.results.cpu(), n, block=cfg["block"],
                       owners=owners_for(world), priority=prio)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    res = local.results if DIST_BACKEND == "nccl" else local.results.cpu()
    full = (gather_results(res, n, block=cfg["block"], owners=owners_for(world), priority=prio) if world > 1
            else None)
    torch.cuda.synchronize()
    gather_ms = reduce_over_ranks(1e3 * (time.perf_counter() - t0), world) if world > 1 else 0.0
    # T_1 in the same run: rank 0 alone over the whole buffer (the others wait)
    if world > 1:
        equal = None
        if rank == 0:
            t1buf = shard_buffer(1, 0)   # the whole frame, in the same block order as the N = 1 run
            w1, _, _ = time_steps(shard_steps(t1buf), steps, warmup, 1)
            t1 = w1 / steps * 1e3
            # T_1's results back in ray order
            idx1 = spans_index(shard_spans(n, 1, 0, B, None, prio), t1buf.results.device)
            single = torch.empty((n, 2), dtype=torch.int32, device=t1buf.results.device)
            single[idx1] = t1buf.results[:, :2]
            equal = bool(torch.equal(full.to(single.device), single))
            del t1buf, single
        barrier(world)
        t1 = reduce_over_ranks(t1 if rank == 0 else 0.0, world)
    else:
        t1, equal = tn, True
    # One GPU, N=1: every shard the 2/4/8-rank runs would give a rank, traced alone
    # the same way (its launches on two streams; the median of three timed runs), so T_n
    # is projected as the slowest shard and eta(n) = T_1 / (n T_n) is known before the
    # driver's multi-GPU runs (which measure the real thing: same code, own GPU per rank).
    projected = None
    if world == 1:
        projected = {}
        for k in STRONG_PROJECT:
            shard_ms = []
            for r_ in range(k):
                sb = shard_buffer(k, r_)
                # three timed runs of the shard, the median kept: one run of a round-5 bench saw a lone
                # 2x-slow shard (0.845 ms against 0.416-0.425 for the other seven, never reproduced in 10 runs)
                # — a projection from one GPU should not turn one transient into the rank's time
                reps = []
                for _ in range(3):
                    w, _, _ = time_steps(shard_steps(sb), steps, 3, 1)
                    reps.append(w / steps * 1e3)
                shard_ms.append(float(np.median(reps)))
                del sb
            projected[str(k)] = {"tn_ms": round(max(shard_ms), 4), "eta": round(t1 / (k * max(shard_ms)), 4),
                                 "shard_ms": [round(x, 4) for x in shard_ms]}
    return {
        "workload": cfg["name"], "rays_traced": n, "rays_counted": counted, "launch_rays_max": cfg["max_batch"],
        "shard_rays": local.size, "n_gpus": world, "t1_ms": round(t1, 4), "tn_ms": round(tn, 4),
        "per_rank_ms": [round(x, 4) for x in per_rank], "kernel_ms_per_launch": round(launch_ms, 4),
        "one_stream_ms": None if one_stream_ms is None else round(one_stream_ms, 4),
        "eta": round(t1 / (world * tn), 4), "gather_ms": round(gather_ms, 3),
        "eta_with_gather": round(t1 / (world * (tn + gather_ms)), 4),
        "value": round(counted / (tn * 1e-3) / 1e6, 2), "value_with_gather": round(counted / ((tn + gather_ms) * 1e-3) / 1e6, 2),
        "shard_build_ms": round(shard_build_ms, 3), "shard_order_ms": round(shard_order_ms, 4),
        "raygen_ms": round(raygen_ms, 4), "raygen_ms_n1": round(raygen_ms_n1, 4), "shard_generated_on_device": True,
        "shard_rays_equal_frame_batches": shard_equal,
        "value_with_gather_and_shard": round(counted / ((tn + gather_ms + shard_order_ms) * 1e-3) / 1e6, 2),
        "value_with_raygen": round(counted / ((tn + gather_ms + shard_order_ms + raygen_ms) * 1e-3) / 1e6, 2),
        "eta_with_raygen": round((t1 + raygen_ms_n1) / (world * (tn + gather_ms + shard_order_ms + raygen_ms)), 4),
        "schedule": {str(k): v for k, v in scheds.items()},
        "schedule_name": "; ".join(sorted({v["name"] for v in scheds.values()})),
        "gathered_equals_single_gpu": equal, "streams": len(streams), "min_launches": cfg["min_launches"],
        "shards": (((f"{cfg['block']}-ray blocks dealt by " + ("the next frame's cost" if cfg["balance"] == 2
                                                                else "live-ray count") if cfg["balance"]
                     else f"block-cyclic, {cfg['block']}-ray blocks")
                    + {0: "", 1: ", live blocks first", 2: ", costly blocks first (next frame's counters)"}[int(cfg["order"])])
                   if cfg["block"] > 0 else "contiguous"),
        "projected_from_one_gpu": projected,
        "roofline": shard_roofline,
        "collective": f"{DIST_BACKEND} point-to-point gather of {n * 8} B to rank 0" if world > 1 else None,
    }


def compact_roofline(rf):
    """The roofline fields the line keeps (the rest is in the detail file)."""
    if rf is None:
        return None
    keep = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms",
                                   "kernel_achieved", "kernel_frac", "kernel_bytes_per_launch",
                                   "hbm_measured_GBps", "hbm_measured_frac", "binding_level", "l2_hit_rate",
                                   "l1_hit_fraction_of_algorithmic", "alg_bytes_per_launch", "vmem_frac",
                                   "binding_unit", "binding_frac", "note")
            if rf.get(k) is not None}
    if rf.get("served"):
        keep["served_frac"] = {k: v["frac"] for k, v in rf["served"].items()}
    prof = rf.get("profile") or {}
    keep["profile"] = prof.get("path") or prof.get("note")
    if prof.get("kernel_ms_ratio") is not None:
        keep["profile_kernel_ms_ratio"] = prof["kernel_ms_ratio"]
    return keep


def compact_parity(cb, fast):
    out = {"exact_fraction": cb.get("parity_exact_fraction")} if cb else {}
    if cb and cb.get("any_hit_valid_hits_checked"):
        out["any_hit_valid_hits_checked"] = cb["any_hit_valid_hits_checked"]
    if cb and cb.get("closest_hit_exact_t_ties"):
        out["closest_hit_exact_t_ties"] = cb["closest_hit_exact_t_ties"]
    if fast and fast.get("parity"):
        fp = fast["parity"]
        out["rcp_fast"] = {k: fp[k] for k in ("rays", "mismatch", "tie", "edge", "other", "any_hit_outcome_flips",
                                              "any_hit_invalid") if k in fp}
    return out


def compact_workload(r):
    """One extra workload in the line: value, kernel time, roofline headline numbers,
    CPU baseline and parity counts."""
    rf = r.get("roofline") or {}
    cb = r.get("cpu_baseline")
    fast = r.get("rcp_fast")
    out = {"workload": r["workload"], "value": r["value"], "reference_mrays": r.get("reference_mrays"),
           "kernel_ms": r["kernel_ms_per_launch"], "schedule": (r.get("schedule") or {}).get("name"),
           "roofline": {k: rf.get(k) for k in ("bound", "frac", "kernel_frac", "hbm_measured_frac", "binding_level",
                                               "traffic", "vmem_frac")},
           "cpu_baseline": cb and cb["value"], "parity": compact_parity(cb, fast)}
    ex = r.get("autotune_exploration") or {}
    if ex.get("tuned_vs_saved"):   # a fresh bind's settled schedule against the saved one
        out["tuned_vs_saved"] = ex["tuned_vs_saved"]
    if fast:
        out["rcp_fast_value"] = fast["value"]
    return out


def compact_strong(st):
    if st is None:
        return None
    keep = {k: st[k] for k in ("workload", "rays_traced", "rays_counted", "n_gpus", "shards", "streams", "t1_ms",
                               "tn_ms", "eta", "gather_ms", "eta_with_gather", "value", "value_with_gather",
                               "shard_build_ms", "shard_order_ms", "raygen_ms", "value_with_gather_and_shard",
                               "value_with_raygen", "eta_with_raygen",
                               "shard_rays_equal_frame_batches", "schedule_name",
                               "gathered_equals_single_gpu", "collective") if k in st}
    keep["per_rank_ms_max_min"] = [max(st["per_rank_ms"]), min(st["per_rank_ms"])]
    keep["value_n1_same_run"] = round(st["rays_counted"] / (st["t1_ms"] * 1e-3) / 1e6, 2)
    if st.get("projected_from_one_gpu"):
        keep["projected_from_one_gpu"] = {k: {"tn_ms": v["tn_ms"], "eta": v["eta"]}
                                          for k, v in st["projected_from_one_gpu"].items()}
    return keep


def make_line(args, world, head, extras, strong, tracer_cfg, cells=None):
    """(the one stdout line, the full detail). The line stays under LINE_MAX_BYTES
    (tests/test_bench_line.py builds it from a recorded run)."""
    ref = REFERENCE_MRAYS.get(args.workload)
    spec = workload_spec(args.workload)
    weak = {"workload": args.workload, "value": head["value"], "ms_per_step": head["ms_per_step"],
            "kernel_ms": head["kernel_ms_per_launch"], "n_gpus": world, "rays_counted_all_ranks":
            head["rays_counted_all_ranks"], "gather": head.get("gather")}
    if args.scaling == "strong":
        value, ms_step = strong["value"], strong["tn_ms"]
        config = {"workload": strong["workload"], "scene": STRONG["scene"], "width": STRONG["w"],
                  "height": STRONG["h"], "samples_per_pixel": STRONG["spp"], "rays_total": strong["rays_traced"],
                  "rays_counted": strong["rays_counted"],
                  "ray_type": "diffuse", "rcp": args.rcp,
                  "parallelism": ((f"one RayBuffer in {world} shards of {STRONG['block']}-ray blocks "
                                   + ({1: "dealt by live-ray count", 2: "dealt by the next frame's traversal cost"}.get(
                                       int(STRONG["balance"]), "dealt round-robin (block-cyclic)"))
                                   + {0: "", 1: ", each shard's live blocks first",
                                      2: ", each shard's costly blocks first (the next frame's counters)"}[int(STRONG["order"])]
                                   + ", BVH replicated, no collective in the step")
                                  if STRONG["block"] > 0 else f"one RayBuffer in {world} contiguous shards"),
                  "launch_rays_max": STRONG["max_batch"]}
        steps = args.strong_steps
    else:
        value, ms_step = head["value"], head["ms_per_step"]
        config = {"workload": args.workload, "scene": spec[0], "scene_tris": head["scene_tris"], "width": spec[1],
                  "height": spec[2], "ray_type": spec[3], "rays_per_gpu": head["rays_counted"], "rcp": args.rcp,
                  "parallelism": (f"rays sharded by pixel sample x{world}, BVH replicated "
                                  f"(weak: one {spec[1]}x{spec[2]} sample per GPU, no collective in the step)")}
        steps = args.steps
    # the schedule the timed launches ran, as the library reports it (mrt_trace_info.autotune_candidate):
    # the headline batch's at N = 1, the shards' launches at N > 1
    config["schedule"] = ((head.get("schedule") or {}).get("name") if args.scaling == "weak"
                          else strong.get("schedule_name"))
    line = {
        "metric": METRIC, "value": value, "unit": "Mrays/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": args.scaling,
        "vs_baseline": round(head["value"] / ref, 3) if (ref and args.scaling == "weak") else None,
        "dtype": "f32",
        "data": "synthetic (deterministic stand-in scene with the README triangle count; rays generated on the device)",
        "config": config,
        "roofline": compact_roofline(head["roofline"] if args.scaling == "weak" else strong.get("roofline")),
        "cpu_baseline": ({k: head["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind", "sample", "cpu_model")}
                         if head.get("cpu_baseline") else None),
        "parity": compact_parity(head.get("cpu_baseline"), head.get("rcp_fast")),
        "weak_scaling": weak if args.scaling == "strong" else None,
        "strong_scaling": compact_strong(strong),
        "rcp_fast": ({"value": head["rcp_fast"]["value"], "kernel_ms": head["rcp_fast"]["kernel_ms_per_launch"],
                      "roofline": compact_roofline(head["rcp_fast"]["roofline"])} if head.get("rcp_fast") else None),
        "autotune_exploration": head.get("autotune_exploration"),
        "extra_workloads": [compact_workload(r) for r in extras],
        "readme_cells": ([{k: c[k] for k in ("cell", "value", "x_readme", "agree", "ties") if k in c} for c in cells]
                         if cells else None),
    }
    if strong is not None and args.scaling == "strong" and strong.get("gathered_equals_single_gpu") is False:
        line["error"] = "gathered results differ from the single-GPU results"
    detail = {"args": vars(args), "tracer_config": tracer_cfg, "head": head, "extras": extras, "strong": strong,
              "readme_cells": cells}
    return line, detail


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20, help="minimum warmup steps (warmup also runs >= 0.3 s)")
    ap.add_argument("--workload", default=HEADLINE, help="a WORKLOADS key or <scene>-<ray>-<W>x<H>")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="which measurement is the line's value (both are reported; default weak at N=1 "
                         "(BASELINE configs[1]), strong at N>1 (configs[4]))")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="file for the full per-workload detail ('' = none)")
    ap.add_argument("--rcp", default="exact", choices=["exact", "fast"],
                    help="exact = correctly rounded 1/x (bit-identical to the oracle); fast = v_rcp_f32")
    ap.add_argument("--extra", dest="extra", action="store_true", default=None,
                    help="also measure the AO/diffuse/hairball configs (default on at N=1)")
    ap.add_argument("--no-extra", dest="extra", action="store_false")
    ap.add_argument("--readme-cells", choices=("default", "all", "none"), default="default",
                    help="with the extras (N = 1): the other README cells, README_N1 (default and 'all': every "
                         "cell the headline and extras do not cover, San Miguel's 10.5 M-triangle scene included), "
                         "or none")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling measurement")
    ap.add_argument("--strong-steps", type=int, default=50)
    ap.add_argument("--strong-block", type=int, default=STRONG["block"],
                    help="block-cyclic shard block (rays); 0 = contiguous shards")
    ap.add_argument("--strong-balance", type=int, default=int(STRONG["balance"]), choices=[0, 1, 2],
                    help="0: deal the shard blocks cyclically; 1: by live-ray count, 2: by the next frame's traversal "
                         "cost (mrt.dist.balance_blocks: equal weight per rank)")
    ap.add_argument("--strong-order", type=int, default=int(STRONG["order"]), choices=[0, 1, 2],
                    help="0: each shard's blocks in frame order; 1: in decreasing live-ray count; 2: in decreasing "
                         "traversal cost, counted on the next frame of the same view (mrt.dist.shard_spans priority)")
    ap.add_argument("--strong-streams", type=int, default=STRONG["streams"], choices=[1, 2],
                    help="caller streams the strong-scaling launches alternate over")
    ap.add_argument("--strong-min-launches", type=int, default=STRONG["min_launches"],
                    help="cut every strong-scaling shard into at least this many launches")
    ap.add_argument("--strong-scene", default=STRONG["scene"],
                    help="scene of the strong-scaling RayBuffer (default: BASELINE configs[4]'s hairball)")
    ap.add_argument("--strong-size", default=f"{STRONG['w']}x{STRONG['h']}x{STRONG['spp']}",
                    help="WxHxSPP of the strong-scaling diffuse frame (default 1920x1080x8: 16.6 M rays)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--fetch-threshold", type=int, default=-1)
    ap.add_argument("--lds-stack", type=int, default=0)
    ap.add_argument("--queues", type=int, default=0)
    ap.add_argument("--bvh-cache", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"),
                    help="directory of Compact2 .dat caches (built if missing); '' disables")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL) for real runs; gloo only to rehearse N>1 ranks on one GPU")
    ap.add_argument("--lane-groups", type=int, default=0)
    ap.add_argument("--no-autotune", action="store_true", help="the fixed schedule rule instead of per-size autotuning")
    ap.add_argument("--tune-db", default=None,
                    help="saved schedules to lock (default: the package's mrt/tuned_schedules.json); '' = none, "
                         "every batch size is autotuned during its warmup")
    ap.add_argument("--save-schedules", default=None, help="write the schedules this run settled to this file "
                                                             "(merged into the --tune-db store; tools/tune_db.sh)")
    ap.add_argument("--no-explore", action="store_true", help="skip measuring the autotuner's exploration cost")
    ap.add_argument("--no-fast", action="store_true", help="skip the fast-reciprocal (v_rcp_f32) measurement")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process starts the ranks and only waits (no GPU call here)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    line_out = reserve_line_stdout()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.scaling is None:
        args.scaling = "weak" if world_env == 1 else "strong"

    global STORE, LEARNED
    from mrt.schedules import DEFAULT_PATH, ScheduleStore
    from mrt.tracer import Tracer
    db = DEFAULT_PATH if args.tune_db is None else args.tune_db
    STORE = ScheduleStore(db) if db else None
    if args.save_schedules:
        LEARNED = ScheduleStore(db) if db else ScheduleStore("")

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
    if args.lane_groups:
        cfg["lane_groups"] = args.lane_groups
    if args.no_autotune:
        cfg["autotune"] = 0
    if cfg:
        tracer.set_config(**cfg)
    exact = args.rcp == "exact"
    want_cpu = (rank == 0 and world == 1 and not args.no_cpu)
    scenes = SceneCache(world, rank, args.bvh_cache or None)

    explore = want_cpu and not args.no_explore and not args.no_autotune
    fast = want_cpu and exact and not args.no_fast
    head = run_workload(args.workload, tracer, scenes, world, rank, args.steps, args.warmup, exact, want_cpu,
                        explore, fast)
    log(f"[head] {args.workload}: {head['value']} Mrays/s")
    extras = []
    do_extra = args.extra if args.extra is not None else (world == 1)
    if do_extra:
        for name in EXTRA_N1:
            if name != args.workload:
                r = run_workload(name, tracer, scenes, world, rank, args.steps, args.warmup, exact, want_cpu,
                                 explore, fast)
                extras.append(r)
                log(f"[extra] {name}: {r['value']} Mrays/s (reference {r['reference_mrays']}, "
                    f"cpu {r.get('cpu_baseline', {}).get('value')})")
    cells = []
    readme = {"default": README_N1, "all": README_ALL, "none": []}[args.readme_cells] if do_extra else []
    for name in readme:
        c = readme_cell(name, tracer, scenes, min(args.steps, 50), args.warmup, exact, want_cpu)
        cells.append(c)
        log(f"[readme] {name}: {c['value']} Mrays/s ({c['x_readme']}x README, agree {c.get('agree')})")
    strong = None
    if not args.no_strong or args.scaling == "strong":
        STRONG["min_launches"] = max(1, args.strong_min_launches)
        STRONG["block"] = max(0, args.strong_block)
        STRONG["streams"] = args.strong_streams
        STRONG["balance"] = int(args.strong_balance)
        STRONG["order"] = int(args.strong_order)
        STRONG["scene"] = args.strong_scene
        STRONG["w"], STRONG["h"], STRONG["spp"] = (int(v) for v in args.strong_size.split("x"))
        STRONG["name"] = f"{STRONG['scene']}-diffuse-{STRONG['w']}x{STRONG['h']}x{STRONG['spp']}spp"
        strong = strong_scaling(tracer, scenes, world, rank, args.strong_steps, 3, exact,
                                with_roofline=args.scaling == "strong")
        log(f"[strong] {strong['workload']} n={world}: T1 {strong['t1_ms']} ms, Tn {strong['tn_ms']} ms, "
            f"eta {strong['eta']} (with gather {strong['eta_with_gather']}); projected from one GPU: "
            f"{ {k: v['eta'] for k, v in (strong['projected_from_one_gpu'] or {}).items()} }")

    if rank == 0:
        line, detail = make_line(args, world, head, extras, strong, tracer.config(), cells)
        if args.detail_out:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail_out)), exist_ok=True)
            with open(args.detail_out, "w") as f:
                json.dump(detail, f, indent=1)
            line["detail_file"] = args.detail_out
        text = json.dumps(line, separators=(",", ":"))
        if len(text) > LINE_MAX_BYTES:
            log(f"[line] {len(text)} B > {LINE_MAX_BYTES}: extras dropped from the line (kept in the detail)")
            line["extra_workloads"] = [{"workload": e["workload"], "value": e["value"]}
                                       for e in line.get("extra_workloads") or []]
            text = json.dumps(line, separators=(",", ":"))
        print(text, file=line_out, flush=True)
        if LEARNED is not None:
            LEARNED.save(args.save_schedules)
            log(f"[schedules] saved {sum(len(v) for v in LEARNED.table.values())} to {args.save_schedules}")
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
