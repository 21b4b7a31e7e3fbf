"""Every BASELINE.json config traced on the GPU through the bench's own workload
code (bench.Batches / bench.strong_scaling's Renderer batches) and compared with
the CPU oracle ray by ray:

  configs[1] bunny primary 1024x768       test_gpu_parity.py::test_full_size_bunny_primary_1024x768
  configs[2] conference AO 640x480        any hit: hit/miss identical, every hit that differs from the
                                          oracle's re-verified as a Woop hit with exactly its t (exact and
                                          fast reciprocal)
  configs[3] sponza diffuse, 2 bounces    both bounce batches: closest hit bit-identical
  configs[4] hairball (6 469 561 tris)    diffuse 640x480 (+ per-lane counters), 1920x1080, and the
                                          16.6 M-ray 1920x1080x8spp strong-scaling RayBuffer

The full-size hairball SBVH takes ~35 s to build on the GPU host; it is built
once per session and cached as a .dat under $TMPDIR/mrt_bvhcache (the bench
reads the same cache).
"""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import oracle_lib as O  # noqa: E402


@pytest.fixture(scope="module")
def env():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    scenes = bench.SceneCache(1, 0, os.path.join(os.environ.get("TMPDIR", "/tmp"), "mrt_bvhcache"))
    return bench, scenes, Tracer(0), bench.host_threads()


def trace_and_compare(tracer, rb, bufs, threads, counters=False):
    """GPU (exact rcp, speculative = the bench's mode) against the oracle on the same rays."""
    any_hit = not rb.need_closest_hit
    rays = rb.rays.cpu().numpy()
    want, st, _ = O.trace(rays, *bufs, any_hit=any_hit, stats=counters, threads=threads)
    tracer.trace_batch(rb, exact_rcp=True)
    got = rb.results_numpy()
    if any_hit:   # hit/miss identical; every hit that differs a genuine Woop hit with its t
        assert np.array_equal(got[:, 0] == -1, want[:, 0] == -1), "any-hit hit/miss differs"
        assert np.array_equal(got[want[:, 0] == -1, 1], want[want[:, 0] == -1, 1])
        diff = np.nonzero((got[:, 0] != want[:, 0]) | (got[:, 1] != want[:, 1]))[0]
        bad = O.invalid_hits(rays, got, bufs[1], bufs[2], which=diff)
        assert len(bad) == 0, f"{len(bad)} of {len(diff)} differing any hits are not valid hits, e.g. ray {bad[:5]}"
        print(f"any hit: {len(diff)} of {len(rays)} rays report another valid hit than the oracle's; all genuine")
    else:
        bad = np.nonzero((got[:, 0] != want[:, 0]) | (got[:, 1] != want[:, 1]))[0]
        assert len(bad) == 0, f"{len(bad)} of {len(rays)} rays differ, e.g. ray {bad[:5]}"
    if counters:   # per-lane order: id, t and node/tri/leaf counters bit-identical
        tracer.trace_batch(rb, exact_rcp=True, speculative=False, stats=True)
        got2 = rb.results_numpy()
        assert np.array_equal(got2[:, :2], want[:, :2])
        assert np.array_equal(rb.stats.cpu().numpy()[:, :3], st[:, :3])
        assert st[:, 3].max() == 0, "oracle reports a stack overflow"
    return got


@pytest.mark.parametrize("name", ["conference-ao-640x480", "sponza-diffuse2-640x480", "hairball-diffuse-640x480",
                                  "hairball-primary-640x480", "hairball-diffuse-1920x1080"])
def test_baseline_config_matches_the_oracle(env, name):
    bench, scenes, tracer, threads = env
    scene_name = bench.workload_spec(name)[0]
    e = scenes.get(scene_name)
    bufs = scenes.host_buffers(scene_name)
    batches = bench.Batches(name, e["scene"], e["gbvh"], tracer)
    if name.startswith("sponza-diffuse2"):
        assert len(batches.batches) == 2     # the second bounce is traced and compared too
    if scene_name == "hairball":
        assert e["scene"].num_triangles == 6469561
    counters = name in ("hairball-diffuse-640x480", "sponza-diffuse2-640x480")
    for rb, counted in batches.batches:
        trace_and_compare(tracer, rb, bufs, threads, counters=counters)
        assert 0 < counted <= rb.size


def test_strong_scaling_raybuffer_matches_the_oracle(env):
    """The 16.6 M-ray RayBuffer of the strong-scaling config (hairball diffuse
    1920x1080 x 8 spp, eight RayGen::batching batches of <= 2^21 rays with their
    glibc seeds), traced in the bench's <= 2^21-ray launches, equals the oracle."""
    bench, scenes, tracer, threads = env
    from mrt.dist import shard_launches
    from mrt.raygen import RAY_DIFFUSE
    from mrt.renderer import Renderer
    cfg = bench.STRONG
    e = scenes.get(cfg["scene"])
    bufs = scenes.host_buffers(cfg["scene"])
    tracer.set_bvh(e["gbvh"])
    cam, _ = e["scene"].camera()
    r = Renderer(tracer, e["scene"], max_batch=cfg["max_batch"])
    r.set_params(RAY_DIFFUSE, cfg["spp"])
    r.begin_frame(cam, cfg["w"], cfg["h"])
    parts = [b for b, _ in r.batches()]
    assert len(parts) == 8 and sum(b.size for b in parts) == cfg["w"] * cfg["h"] * cfg["spp"]
    for b in parts:
        for lo, hi in shard_launches(0, b.size, cfg["max_batch"]):
            tracer.trace_async(b.view(lo, hi), exact_rcp=True)
    torch.cuda.synchronize()
    total_bad = 0
    for b in parts:
        want, _, _ = O.trace(b.rays.cpu().numpy(), *bufs, threads=threads)
        got = b.results_numpy()
        total_bad += int(((got[:, 0] != want[:, 0]) | (got[:, 1] != want[:, 1])).sum())
    assert total_bad == 0


@pytest.mark.parametrize("name,queues,waves", [("hairball-diffuse-1920x1080", 1, 16), ("hairball-primary-1024x768", 1, 12),
                                               ("hairball-diffuse-640x480", 1, 12), ("sponza-diffuse-640x480", 0, 20),
                                               ("bunny-primary-1024x768", 0, 20)])
def test_automatic_launch_config(env, name, queues, waves):
    """Default knobs: a batch over a BVH above the 256 MB Infinity Cache runs on one
    global queue with refills at 48 live lanes, 12 waves/CU up to 3 rays per lane of a
    16-wave grid, else 16 (mrt_api.cpp effective_cfg); everything else on static
    strided rounds at 20 waves/CU. Results equal the oracle either way
    (test_baseline_config_matches_the_oracle covers both)."""
    bench, scenes, tracer, threads = env
    e = scenes.get(bench.workload_spec(name)[0])
    batches = bench.Batches(name, e["scene"], e["gbvh"], tracer)
    rb = batches.batches[0][0]
    saved = tracer.config()
    tracer.set_config(autotune=0)   # the fixed rule (autotuning starts from it and may pick another schedule)
    tracer.trace_batch(rb, exact_rcp=True)
    tracer.set_config(**saved)
    assert tracer.last_info["num_queues"] == queues
    assert tracer.last_info["fetch_threshold"] == (48 if queues else 0)
    assert tracer.last_info["grid_waves"] == waves * torch.cuda.get_device_properties(0).multi_processor_count
    saved = tracer.config()
    try:
        tracer.set_config(waves_per_cu=20, autotune=0)   # any explicit distribution knob keeps the static rounds
        tracer.trace_batch(rb, exact_rcp=True)
        assert tracer.last_info["num_queues"] == 0
    finally:
        tracer.set_config(**saved)


def test_autotuned_schedule_settles_and_keeps_results(env):
    """cfg.autotune (default): the first launches of a batch size cycle through eight
    ray-distribution schedules, timed without blocking in runs of four launches (the
    first untimed), then the winner and the runner-up with each stage-2 modifier, then
    the best modifier on the other schedules, and keep the fastest by the median of
    eight samples. Every launch, exploring or settled,
    returns the oracle's closest hits; the settled choice exports and imports."""
    bench, scenes, tracer, threads = env
    name = "bunny-primary-1024x768"
    e = scenes.get(bench.workload_spec(name)[0])
    bufs = scenes.host_buffers(bench.workload_spec(name)[0])
    batches = bench.Batches(name, e["scene"], e["gbvh"], tracer)
    rb = batches.batches[0][0]
    assert tracer.config()["autotune"] == 1
    tracer.set_config(autotune=1)   # a fresh tuning state for this handle
    want, _, _ = O.trace(rb.rays.cpu().numpy(), *bufs, threads=threads)
    seen = set()
    for i in range(600):
        tracer.trace_batch(rb, exact_rcp=True)   # blocking: every launch's timing is read back by the next
        seen.add(tracer.last_info["autotune_candidate"] & 0xff)
        got = rb.results_numpy()
        assert np.array_equal(got[:, :2], want[:, :2]), f"launch {i} (candidate {tracer.last_info['autotune_candidate']})"
        if tracer.last_info["autotune_locked"]:
            break
    assert seen == set(range(13))
    assert tracer.last_info["autotune_locked"] == 1
    # the settled choice round-trips through export/import onto a fresh bind
    saved = tracer.schedules()
    chosen = tracer.last_info["autotune_candidate"]
    assert any(n == rb.size for n, _, _, _ in saved)
    tracer.set_bvh(e["gbvh"])
    tracer.load_schedules(saved)
    tracer.trace_batch(rb, exact_rcp=True)
    assert tracer.last_info["autotune_locked"] == 1 and tracer.last_info["autotune_candidate"] == chosen
    assert np.array_equal(rb.results_numpy()[:, :2], want[:, :2])


def test_nearby_batch_sizes_and_other_streams_take_the_settled_schedule(env):
    """A batch size within 1/32 of a settled one takes its schedule at once (the
    strong-scaling shards of one frame differ by a block or two); a settled batch
    size launched on a second stream keeps its schedule instead of falling back to
    the fixed rule; one beyond 1/32 explores. Results equal the oracle throughout."""
    bench, scenes, tracer, threads = env
    name = "bunny-primary-1024x768"
    e = scenes.get(bench.workload_spec(name)[0])
    bufs = scenes.host_buffers(bench.workload_spec(name)[0])
    rb = bench.Batches(name, e["scene"], e["gbvh"], tracer).batches[0][0]
    tracer.set_config(autotune=1)   # a fresh tuning state
    n = rb.size
    ref = rb.view(0, n)
    for _ in range(600):            # settle size n
        tracer.trace_batch(ref, exact_rcp=True)
        if tracer.last_info["autotune_locked"]:
            break
    assert tracer.last_info["autotune_locked"] == 1
    chosen = tracer.last_info["autotune_candidate"]
    want, _, _ = O.trace(rb.rays.cpu().numpy(), *bufs, threads=threads)
    # a batch 1/64 smaller: inherits the lock on its first launch
    near = rb.view(0, n - n // 64)
    tracer.trace_batch(near, exact_rcp=True)
    assert tracer.last_info["autotune_locked"] == 1 and tracer.last_info["autotune_candidate"] == chosen
    assert np.array_equal(near.results_numpy()[:, :2], want[: near.size, :2])
    # the settled size on a second stream: still its schedule
    s2 = torch.cuda.Stream()
    tracer.trace_batch(ref, exact_rcp=True, stream=s2)
    torch.cuda.synchronize()
    assert tracer.last_info["autotune_locked"] == 1 and tracer.last_info["autotune_candidate"] == chosen
    assert np.array_equal(ref.results_numpy()[:, :2], want[:, :2])
    # a batch 1/8 smaller: too far, it explores
    far = rb.view(0, n - n // 8)
    tracer.trace_batch(far, exact_rcp=True)
    assert tracer.last_info["autotune_locked"] == 0
    assert np.array_equal(far.results_numpy()[:, :2], want[: far.size, :2])
    tracer.set_bvh(e["gbvh"])


def test_secondary_batches_keep_their_own_schedule(env):
    """MRT_TRACE_SECONDARY (RayBuffer.secondary; DeviceRayGen.ao sets it): a batch of secondary
    rays settles its own schedule even when a primary batch of the same size and kernel variant
    has settled one (no inheritance across the two classes), and the two export as separate
    entries (variant | 512). Results equal the oracle in both classes."""
    from mrt.tracer import RayBuffer
    bench, scenes, tracer, threads = env
    name = "bunny-primary-640x480"
    e = scenes.get(bench.workload_spec(name)[0])
    bufs = scenes.host_buffers(bench.workload_spec(name)[0])
    prim = bench.Batches(name, e["scene"], e["gbvh"], tracer).batches[0][0]
    tracer.set_config(autotune=1)   # a fresh tuning state
    sec = RayBuffer(prim.rays.clone(), need_closest_hit=True, secondary=True)
    assert sec.view(0, 10).secondary and not prim.secondary
    for _ in range(600):            # settle the primary class
        tracer.trace_batch(prim, exact_rcp=True)
        if tracer.last_info["autotune_locked"]:
            break
    assert tracer.last_info["autotune_locked"] == 1
    tracer.trace_batch(sec, exact_rcp=True)   # same size and variant, the other class: it explores
    assert tracer.last_info["autotune_locked"] == 0
    for _ in range(600):
        tracer.trace_batch(sec, exact_rcp=True)
        if tracer.last_info["autotune_locked"]:
            break
    assert tracer.last_info["autotune_locked"] == 1
    keys = {(n, v) for n, v, _, _ in tracer.schedules()}
    v0 = next(v for n, v in keys if n == prim.size and not v & 512)
    assert (prim.size, v0 | 512) in keys
    want, _, _ = O.trace(prim.rays.cpu().numpy(), *bufs, threads=threads)
    assert np.array_equal(prim.results_numpy()[:, :2], want[:, :2])
    assert np.array_equal(sec.results_numpy()[:, :2], want[:, :2])
    tracer.set_bvh(e["gbvh"])


# SURVEY §8(a) Note 3 bounds: the "edge" class (an accept/reject flip of one triangle under
# +-1 ulp of 1/Dz) at most 1e-6 of a workload's rays, and never more than one ray below 1e6 rays
EDGE_FRACTION = 1e-6


@pytest.mark.parametrize("name", ["bunny-primary-1024x768", "sponza-diffuse2-640x480", "hairball-diffuse-640x480",
                                  "hairball-diffuse-1920x1080", "conference-ao-640x480"])
def test_fast_rcp_mismatches_are_classified(env, name):
    """SURVEY §8(a) Note 3 at full size on every BASELINE workload: the fast-reciprocal mode
    (v_rcp_f32, the reference's rcp.approx analogue; what launch_tracingKernel and the
    default Tracer use) against the oracle's correctly rounded arithmetic. Closest hit:
    every mismatch is a tie (both triangles valid hits within 4 ulp, <= 1e-5 of the rays)
    or an edge case (oracle_lib.classify_fast_rcp: the oracle's or the GPU's triangle
    changes acceptance when 1/Dz moves by one ulp, re-verified per ray), no other
    mismatch. Any hit: every hit/miss flip is such an edge case
    (oracle_lib.classify_any_hit_flips). Edge cases: at most EDGE_FRACTION of the rays."""
    bench, scenes, tracer, threads = env
    scene_name = bench.workload_spec(name)[0]
    e = scenes.get(scene_name)
    bufs = scenes.host_buffers(scene_name)
    batches = bench.Batches(name, e["scene"], e["gbvh"], tracer)
    total = {"rays": 0, "tie": 0, "edge": 0, "other": 0}
    for rb, _ in batches.batches:
        rays = rb.rays.cpu().numpy()
        any_hit = not rb.need_closest_hit
        want, _, _ = O.trace(rays, *bufs, any_hit=any_hit, threads=threads)
        tracer.trace_batch(rb, exact_rcp=False)
        got = rb.results_numpy()
        if any_hit:
            c = O.classify_any_hit_flips(rays, got, want, bufs[1], bufs[2])
            total["rays"] += len(rays)
            total["edge"] += c["edge"]
            total["other"] += c["other"]
            # every hit or miss that differs from the oracle's is genuine under v_rcp_f32's one-ulp
            # bound on 1/Dz: a Woop hit with exactly its t, or a miss with t = tmax
            diff = np.nonzero((got[:, 0] != want[:, 0]) | (got[:, 1] != want[:, 1]))[0]
            bad = O.invalid_hits(rays, got, bufs[1], bufs[2], which=diff, rcp_ulps=1)
            assert len(bad) == 0, f"{len(bad)} of {len(diff)} differing fast any-hit results are not genuine"
            print(name, c, f"{len(diff)} differing results, all genuine")
            continue
        c = O.classify_fast_rcp(rays, got, want, bufs[1], bufs[2])
        assert c["unclassified"] == 0
        for k in ("rays", "tie", "edge", "other"):
            total[k] += c[k]
        print(name, {k: c[k] for k in ("rays", "mismatch", "tie", "edge", "other")}, c["examples"]["other"][:3])
    assert total["other"] == 0, total
    assert total["tie"] <= max(2, total["rays"] // 100000), total
    assert total["edge"] <= max(1, int(EDGE_FRACTION * total["rays"])), total
