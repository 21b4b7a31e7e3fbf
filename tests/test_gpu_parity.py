"""GPU parity: the HIP traversal behind the C-ABI against the CPU oracle.

Contract:
  * exact-rcp mode (MRT_TRACE_EXACT_RCP), per-lane order (LOCKSTEP_OFF):
        id, t and the per-ray counters bit-identical to the oracle, closest and any-hit;
  * exact-rcp, speculative (the reference's warp-wide postponement):
        closest hit: id and t bit-identical;  any hit: hit/miss identical and the
        reported triangle is a valid hit whose t the oracle's Woop test reproduces bit-exactly;
  * fast rcp (v_rcp_f32): ids identical except exact-t ties, |dt| <= 2 ulp
        (v_rcp_f32 is within 1 ulp of 1/x; one more rounding in Oz * rcp(Dz)).
"""
import ctypes as C
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import kat  # noqa: E402
import mrt  # noqa: E402
import oracle_lib as O  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tracer():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mrt.tracer import Tracer
    return Tracer(0)


def gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True, stats=False):
    from mrt.tracer import GpuBvh, RayBuffer
    g = GpuBvh(bufs)
    tracer.set_bvh(g)
    rb = RayBuffer(rays, need_closest_hit=not any_hit)
    rb.results.fill_(0x5A5A5A5A)   # pads must survive: the trace writes {id, t} only
    tracer.trace_batch(rb, exact_rcp=exact, speculative=spec, stats=stats)
    r = rb.results_numpy()
    assert (r[:, 2:] == 0x5A5A5A5A).all(), "RayResult padding was overwritten"
    return r, (rb.stats.cpu().numpy() if stats else None)


def ulp_diff(a_bits, b_bits):
    a = a_bits.astype(np.int64)
    b = b_bits.astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


def assert_valid_hits(rays, res, oracle_res, bufs, rcp_ulps=0):
    """Every any-hit result that differs from the oracle's is genuine: hit/miss
    identical, and each differing hit a triangle whose Woop test the oracle reproduces with
    exactly the reported t (oracle_lib.invalid_hits, one C pass over all of them; rcp_ulps 1
    for the fast-reciprocal mode, whose 1/Dz may be one ulp off). Returns the rays checked."""
    nodes, woop, tri = bufs
    assert np.array_equal(res[:, 0] == -1, oracle_res[:, 0] == -1), "hit/miss differs"
    diff = np.nonzero((res[:, 0] != oracle_res[:, 0]) | (res[:, 1] != oracle_res[:, 1]))[0]
    bad = O.invalid_hits(rays, res, woop, tri, which=diff, rcp_ulps=rcp_ulps)
    assert len(bad) == 0, (f"{len(bad)} of {len(diff)} differing any-hit results are not valid hits, e.g. ray "
                           f"{bad[0]}: GPU ({res[bad[0], 0]}, {res[bad[0], 1]}) oracle {tuple(oracle_res[bad[0], :2])}")
    return len(diff)


# ---------------------------------------------------------------- known answers
@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("spec", [True, False])
@pytest.mark.parametrize("case", kat.cases(), ids=lambda c: c[0])
def test_known_answers(tracer, case, spec, exact):
    name, scene, rays, any_hit, expected = case
    res, _ = gpu_trace(tracer, scene(), np.stack(rays), any_hit, exact=exact, spec=spec)
    for (rid, rt), got in zip(expected, res):
        assert got[0] == rid, name
        assert got[1] == kat.f2i(rt), name


# ---------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("fname", sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz")))
def test_golden_fixtures(tracer, fname):
    g = np.load(os.path.join(GOLDEN, fname))
    bufs = (g["nodes"], g["woop"], g["tri_index"])
    any_hit = bool(g["any_hit"])
    res, st = gpu_trace(tracer, bufs, g["rays"], any_hit, exact=True, spec=False, stats=True)
    assert np.array_equal(res[:, :2], g["results"][:, :2])
    assert np.array_equal(st[:, :3], g["stats"][:, :3])
    res2, _ = gpu_trace(tracer, bufs, g["rays"], any_hit, exact=True, spec=True)
    if any_hit:
        assert_valid_hits(g["rays"], res2, g["results"], bufs)
    else:
        assert np.array_equal(res2[:, :2], g["results"][:, :2])


# ---------------------------------------------------------------- synthetic scenes
SCENE_CACHE = {}


def scene_setup(name, w, h, kind):
    key = (name, w, h, kind)
    if key not in SCENE_CACHE:
        base, _, param = name.partition(":")   # "hairball:800" = an 800-tube hairball
        scene = mrt.Scene.synthetic(base, int(param or 0), 1)
        bufs = mrt.Bvh.build(scene).buffers()
        cam, ao = scene.camera()
        rays, _ = mrt.primary_rays(cam, w, h)
        if kind != "primary":
            prim, _, _ = O.trace(rays, *bufs, threads=8)
            rays = mrt.ao_rays(rays, prim, scene, ao if kind == "ao" else cam.far)
        any_hit = kind == "ao"
        want, st, _ = O.trace(rays, *bufs, any_hit=any_hit, stats=True, threads=8)
        SCENE_CACHE[key] = (bufs, rays, any_hit, want, st)
    return SCENE_CACHE[key]


WORKLOADS = [("bunny", 320, 240, "primary"), ("conference", 256, 192, "ao"), ("sponza", 256, 192, "diffuse"),
             ("conference", 256, 192, "diffuse"), ("mori", 256, 192, "ao"), ("hairball:800", 256, 192, "diffuse"),
             ("sibenik", 256, 192, "diffuse"), ("fairy", 256, 192, "ao"), ("dragon", 256, 192, "primary")]


@pytest.mark.parametrize("wl", WORKLOADS, ids=lambda w: "-".join(map(str, w)))
def test_exact_lockstep_off_is_bit_identical_with_counters(tracer, wl):
    bufs, rays, any_hit, want, st = scene_setup(*wl)
    res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
    assert np.array_equal(res[:, :2], want[:, :2])
    assert np.array_equal(gst[:, :3], st[:, :3])


@pytest.mark.parametrize("wl", WORKLOADS, ids=lambda w: "-".join(map(str, w)))
def test_exact_speculative(tracer, wl):
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
    if any_hit:
        assert_valid_hits(rays, res, want, bufs)
    else:
        assert np.array_equal(res[:, :2], want[:, :2])


@pytest.mark.parametrize("wl", WORKLOADS, ids=lambda w: "-".join(map(str, w)))
def test_quantized_wide_nodes(tracer, wl):
    """cfg.wide=2: the 64-B nodes' boxes contain the binary boxes, so the traversal
    tests a superset of the binary traversal's leaves. Closest hits equal the
    oracle's except where that superset holds a hit the oracle's own slab test
    rejected at a box boundary (a grazing ray; ~1 in 10^5-10^6 rays): such a hit
    must be a genuine Woop hit no farther than the oracle's. Any-hit results are
    genuine hits with the oracle's hit/miss outcome."""
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    saved = tracer.config()
    try:
        tracer.set_config(wide=2)
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        assert tracer.last_info["node_bytes"] == 64 and tracer.last_info["wide"] == 4
    finally:
        tracer.set_config(**saved)
    if any_hit:
        assert_valid_hits(rays, res, want, bufs)
        return
    diff = np.nonzero((res[:, 0] != want[:, 0]) | (res[:, 1] != want[:, 1]))[0]
    assert len(diff) <= max(2, len(rays) // 10000), f"{len(diff)} rays differ"
    closer = res[diff, 1].view(np.float32) <= want[diff, 1].view(np.float32)
    assert closer.all() and (res[diff, 0] != -1).all(), "a quantized-node hit is farther than the oracle's"
    nodes, woop, tri = bufs
    woop4 = woop.reshape(-1, 4)
    for i in diff:
        cand = np.nonzero((tri == res[i, 0]) & (woop4[:, 0] != np.int32(-2147483648)))[0]
        assert any(O.woop_hit(rays[i], woop, s, float(rays[i][7]))[0] for s in cand), f"ray {i}: not a Woop hit"


@pytest.mark.parametrize("wl", WORKLOADS, ids=lambda w: "-".join(map(str, w)))
def test_fast_rcp_within_tolerance(tracer, wl):
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=False, spec=True)
    assert np.array_equal(res[:, 0] == -1, want[:, 0] == -1)
    hit = want[:, 0] != -1
    if not any_hit:
        # SURVEY §8(a) Note 3: every mismatch classified; none may be a real error
        c = O.classify_fast_rcp(rays, res, want, bufs[1], bufs[2])
        assert c["other"] == 0, c
        assert c["tie"] + c["edge"] <= max(2, len(rays) // 10000), c
        same = hit & (res[:, 0] == want[:, 0])
        assert ulp_diff(res[same, 1], want[same, 1]).max(initial=0) <= 2
    assert np.array_equal(res[~hit, 1], want[~hit, 1])   # misses keep tmax exactly


def test_exact_reciprocal_is_correctly_rounded_for_every_float(tracer):
    """The EXACT variants compute 1/x as v_rcp_f32 + one FMA Newton step; it must
    equal the IEEE division 1.0f / x for all 2^32 inputs (device-side sweep)."""
    from mrt import _lib
    n = C.c_uint64(12345)
    _lib.check(tracer.lib.mrt_selftest_exact_rcp(C.byref(n)))
    assert n.value == 0


# ---------------------------------------------------------------- launch configs
@pytest.mark.parametrize("cfg", [dict(lds_stack=8), dict(lds_stack=32), dict(waves_per_cu=8),
                                 dict(num_queues=1), dict(num_queues=8, fetch_threshold=40),
                                 dict(num_queues=8, waves_per_cu=32, fetch_threshold=64),
                                 dict(num_queues=-1, fetch_threshold=16), dict(num_queues=-1, waves_per_cu=4),
                                 dict(waves_per_cu=4, lds_stack=8, num_queues=3),
                                 dict(lds_stack=32, waves_per_cu=4, fetch_threshold=48),
                                 dict(num_queues=1, fetch_threshold=48, waves_per_cu=16), dict(lane_groups=2),
                                 dict(lane_groups=8), dict(lane_groups=16), dict(lane_groups=64, waves_per_cu=4), dict(spec_slack=0),
                                 dict(spec_slack=63), dict(spec_slack=7, num_queues=2, fetch_threshold=40),
                                 dict(tail_lanes=0), dict(tail_lanes=1), dict(tail_lanes=4),
                                 dict(tail_lanes=16, waves_per_cu=4), dict(tail_lanes=16, lds_stack=8),
                                 dict(tail_lanes=16, num_queues=1, fetch_threshold=48, waves_per_cu=4),
                                 dict(tail_lanes=12, num_queues=8, waves_per_cu=4, static_rounds=2),
                                 dict(tail_lanes=16, num_queues=-1, fetch_threshold=16),
                                 dict(num_queues=8, queue_shared=15, fetch_threshold=48, waves_per_cu=4),
                                 dict(num_queues=8, queue_shared=100, waves_per_cu=4),
                                 dict(num_queues=3, queue_shared=40, fetch_threshold=32, waves_per_cu=4),
                                 dict(num_queues=8, queue_shared=15, fetch_threshold=48, waves_per_cu=20),
                                 dict(num_queues=8, queue_shared=10, queue_block=4096, fetch_threshold=48, waves_per_cu=4),
                                 dict(num_queues=8, queue_block=64, waves_per_cu=4),
                                 dict(num_queues=5, queue_shared=5, queue_block=1024, fetch_threshold=40, waves_per_cu=4),
                                 dict(num_queues=8, queue_block=8192, fetch_threshold=56, waves_per_cu=20),
                                 dict(num_queues=8, queue_block=256, fetch_threshold=56, waves_per_cu=4),
                                 dict(ray_sort=1), dict(ray_sort=1, tail_lanes=0), dict(ray_sort=1, waves_per_cu=4),
                                 dict(ray_sort=1, lane_groups=16), dict(ray_sort=1, waves_per_cu=8, lds_stack=8),
                                 dict(lane_groups=2, waves_per_cu=8), dict(lane_groups=64, tail_lanes=0),
                                 dict(lane_groups=4, waves_per_cu=4), dict(lane_groups=16, waves_per_cu=8, lds_stack=8)],
                         ids=lambda c: ",".join(f"{k}={v}" for k, v in c.items()))
def test_launch_configs_do_not_change_results(tracer, cfg):
    bufs, rays, any_hit, want, st = scene_setup("conference", 256, 192, "diffuse")
    saved = tracer.config()
    try:
        tracer.set_config(**cfg)
        res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
        assert np.array_equal(res[:, :2], want[:, :2]) and np.array_equal(gst[:, :3], st[:, :3])
        res2, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        assert np.array_equal(res2[:, :2], want[:, :2])
    finally:
        tracer.set_config(**saved)


@pytest.mark.parametrize("cfg", [dict(num_queues=8, queue_xcc_mask=3), dict(num_queues=8, queue_xcc_mask=1),
                                 dict(num_queues=8, queue_xcc_mask=3, queue_shared=10),
                                 dict(num_queues=5, queue_xcc_mask=3), dict(num_queues=8, queue_xcc_mask=0)],
                         ids=lambda c: ",".join(f"{k}={v}" for k, v in c.items()))
def test_queues_without_waves_are_still_traced(tracer, cfg):
    """with per-XCD queues a wave takes from queue XCC_ID % num_queues; on a
    device or partition where some queue gets no waves (CPX/DPX, a placement that skips an
    XCD) its rays must still be traced. The test hook queue_xcc_mask masks XCC_ID so that
    only queues 0..mask have waves (mask 1: a quarter of the 8 queues); the queues past the
    first static round hold most of the 307 200-ray batch (4 waves/CU = 65 536 static rays,
    1 024-ray blocks). Every ray equals the oracle, closest hit and per-lane counters."""
    bufs, rays, any_hit, want, st = scene_setup("conference", 640, 480, "diffuse")
    saved = tracer.config()
    try:
        tracer.set_config(queue_block=1024, fetch_threshold=56, waves_per_cu=4, autotune=0, **cfg)
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        assert np.array_equal(res[:, :2], want[:, :2])
        assert tracer.last_info["num_queues"] == cfg["num_queues"]
        res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
        assert np.array_equal(res[:, :2], want[:, :2]) and np.array_equal(gst[:, :3], st[:, :3])
    finally:
        tracer.set_config(**saved)


@pytest.mark.parametrize("wl", [("conference", 640, 480, "ao"), ("mori", 640, 480, "ao"), ("sponza", 640, 480, "diffuse"),
                                ("hairball:800", 640, 480, "diffuse"), ("bunny", 640, 480, "primary")],
                         ids=lambda w: "-".join(map(str, w)))
@pytest.mark.parametrize("waves,groups", [(20, 1), (8, 1), (8, 2), (16, 16)])
def test_static_deal_traces_every_ray_once(tracer, wl, waves, groups):
    """The static strided deal over one round (20 waves/CU: 307 200 rays) and several
    (8 waves/CU), with lane groups: every ray traced exactly once and equal to the oracle —
    closest hits bit-identical, any hits genuine (hit/miss identical)."""
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    saved = tracer.config()
    try:
        tracer.set_config(waves_per_cu=waves, lane_groups=groups, autotune=0)
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        if any_hit:
            assert_valid_hits(rays, res, want, bufs)
        else:
            assert np.array_equal(res[:, :2], want[:, :2])
    finally:
        tracer.set_config(**saved)


@pytest.mark.parametrize("wl", [("conference", 640, 480, "ao"), ("mori", 640, 480, "ao"), ("sponza", 640, 480, "diffuse"),
                                ("hairball:800", 640, 480, "diffuse"), ("bunny", 640, 480, "primary")],
                         ids=lambda w: "-".join(map(str, w)))
@pytest.mark.parametrize("waves", [20, 8])
def test_ray_sort_traces_every_ray_once(tracer, wl, waves):
    """cfg.ray_sort: a one-round static launch deals each workgroup's 256-ray tile by direction
    octant (degenerate rays last). Every ray is traced exactly once and equals the oracle:
    closest hits bit-identical, any hits genuine (hit/miss identical). At 8 waves/CU the
    307 200-ray batch needs several rounds, so the sort is skipped there (the same results)."""
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    saved = tracer.config()
    try:
        tracer.set_config(ray_sort=1, waves_per_cu=waves, autotune=0)
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        if any_hit:
            assert_valid_hits(rays, res, want, bufs)
        else:
            assert np.array_equal(res[:, :2], want[:, :2])
    finally:
        tracer.set_config(**saved)


def test_per_xcd_candidate_uses_one_queue_per_xcd(tracer):
    """The autotuner's per-XCD candidate (2) sizes its queues from the device's XCD count
    (hipDeviceAttributeNumberOfXccs), never more: 8 on an SPX MI355X."""
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, rays, any_hit, want, _ = scene_setup("conference", 640, 480, "diffuse")
    saved = tracer.config()
    try:
        tracer.set_config(autotune=1)
        tracer.set_bvh(GpuBvh(bufs))
        rb = RayBuffer(rays, need_closest_hit=True)
        seen = {}
        for _ in range(40):   # the exploring launches cycle through the eight stage-1 schedules
            tracer.trace_batch(rb, exact_rcp=True)
            seen[tracer.last_info["autotune_candidate"]] = tracer.last_info["num_queues"]
        assert 2 in seen
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert 1 <= seen[2] <= 8 and seen[2] == min(8, max(1, cus // 32))
        assert np.array_equal(rb.results_numpy()[:, :2], want[:, :2])
    finally:
        tracer.set_config(**saved)


def test_deep_stacks_and_rebinding(tracer):
    """An 8-entry LDS ring (deep stacks spill to the slab) and a re-bound BVH."""
    saved = tracer.config()
    try:
        tracer.set_config(lds_stack=8)
        test_rebinding_a_different_bvh(tracer)
        bufs, rays, any_hit, want, st = scene_setup("sponza", 256, 192, "diffuse")
        res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
        assert np.array_equal(res[:, :2], want[:, :2]) and np.array_equal(gst[:, :3], st[:, :3])
    finally:
        tracer.set_config(**saved)


# ---------------------------------------------------------------- concurrency, overflow, limits
def test_concurrent_streams_on_one_handle(tracer):
    """two traces of one handle in flight on two streams at once, on a deep
    scene whose stacks spill past an 8-entry LDS ring: each stream has its own spill
    slab / counters, so both batches equal the oracle."""
    from mrt.tracer import GpuBvh, RayBuffer
    bufs_a, rays_a, _, want_a, _ = scene_setup("hairball:800", 256, 192, "diffuse")
    saved = tracer.config()
    try:
        tracer.set_config(lds_stack=8)
        tracer.set_bvh(GpuBvh(bufs_a))
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        rbs = [RayBuffer(rays_a, need_closest_hit=True) for _ in range(4)]
        torch.cuda.synchronize()
        for k, rb in enumerate(rbs):
            s = s1 if k % 2 == 0 else s2
            with torch.cuda.stream(s):
                tracer.trace_async(rb, exact_rcp=True, speculative=False, stream=s)
        s1.synchronize()
        s2.synchronize()
        for rb in rbs:
            assert np.array_equal(rb.results_numpy()[:, :2], want_a[:, :2])
    finally:
        tracer.set_config(**saved)


def test_two_handles_from_two_host_threads():
    """two tracer handles on one device, each with its own BVH, traced from
    two host threads at once (the C calls release the GIL), blocking and asynchronous calls
    interleaved on each thread's own stream, a set_config per round: every batch equals the
    oracle — no cross-talk through the workspaces' LRU order or the waits."""
    import threading
    from mrt.tracer import GpuBvh, RayBuffer, Tracer
    jobs = [scene_setup("bunny", 320, 240, "primary"), scene_setup("sponza", 256, 192, "diffuse")]
    errors, outs = [], [[], []]

    def worker(k):
        try:
            bufs, rays, any_hit, want, _ = jobs[k]
            t = Tracer(0)
            t.set_bvh(GpuBvh(bufs))
            s = torch.cuda.Stream()
            for rnd in range(6):
                t.set_config(lds_stack=8 if rnd % 2 else 16)
                rbs = [RayBuffer(rays, need_closest_hit=not any_hit) for _ in range(3)]
                with torch.cuda.stream(s):
                    t.trace_async(rbs[0], exact_rcp=True, stream=s)
                    t.trace_batch(rbs[1], exact_rcp=True, stream=s)
                    t.trace_async(rbs[2], exact_rcp=True, stream=s)
                s.synchronize()
                outs[k] += [rb.results_numpy()[:, :2] for rb in rbs]
            assert t.last_info["stack_overflows"] == 0
        except Exception as e:   # noqa: BLE001 — reported by the main thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not errors, errors
    for k in range(2):
        want = jobs[k][3]
        assert len(outs[k]) == 18
        for r in outs[k]:
            assert np.array_equal(r, want[:, :2])


@pytest.mark.parametrize("depth,overflow", [(40, False), (63, False), (64, True), (70, True)])
def test_stack_overflow_is_reported(tracer, depth, overflow):
    """A comb BVH whose ray pushes one far leaf per level (kat.scene_comb): with 70
    levels the reference's 64-entry stack (kepler_dynamic_fetch.cu:47) overflows.
    The blocking trace reports it (MRT_ERR_STACK_OVERFLOW + per-launch count), the
    async path keeps a sticky counter; up to 63 pushes (the reference's capacity: sentinel +
    63) trace exactly to the hand answer, through the spill slab."""
    from mrt import _lib
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, ray, expect = kat.scene_comb(depth)
    saved = tracer.config()
    tracer.set_config(wide=0)   # the reference's capacity is a property of its binary traversal order
    tracer.set_bvh(GpuBvh(bufs))
    n0 = C.c_int64()
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n0), 1))
    rb = RayBuffer(np.stack([ray] * 64), need_closest_hit=True)
    for spec in (False, True):
        if overflow:
            with pytest.raises(_lib.MrtError, match="stack overflow"):
                tracer.trace_batch(rb, exact_rcp=True, speculative=spec)
            assert tracer.lib.mrt_tracer_trace_timed(tracer._h, rb.rays.data_ptr(), rb.results.data_ptr(), rb.size,
                                                     _lib.MRT_TRACE_EXACT_RCP, None, None,
                                                     C.byref(_lib.TraceInfo())) == _lib.MRT_ERR_STACK_OVERFLOW
        else:
            tracer.trace_batch(rb, exact_rcp=True, speculative=spec)
            res = rb.results_numpy()
            assert (res[:, 0] == expect[0]).all() and (res[:, 1] == kat.f2i(expect[1])).all()
    tracer.trace_async(rb, exact_rcp=True)
    n = C.c_int64()
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 1))
    assert (n.value > 0) == overflow
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 0))
    assert n.value == 0
    # the 4-wide traversal may push up to three entries per wide node, so its
    # stack is sized at bind time to the bound tree's worst case (never below the
    # reference's 64): the hand answer at every depth, no overflow, async counter untouched
    tracer.set_config(wide=1)
    bi = tracer.bind_info()
    assert bi["wide_format"] == 1 and bi["stack_capacity"] >= 64
    tracer.trace_batch(rb, exact_rcp=True)
    res = rb.results_numpy()
    assert tracer.last_info["wide"] == 4 and tracer.last_info["stack_overflows"] == 0
    assert tracer.last_info["stack_capacity"] == bi["stack_capacity"]
    assert (res[:, 0] == expect[0]).all() and (res[:, 1] == kat.f2i(expect[1])).all()
    tracer.trace_async(rb, exact_rcp=True)
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 1))
    assert n.value == 0
    tracer.set_config(**saved)


@pytest.mark.parametrize("rays_n", [1, 5, 16, 17, 40])
@pytest.mark.parametrize("depth", [10, 40, 63, 70])
def test_frontier_tail_on_deep_stacks(tracer, depth, rays_n):
    """The frontier tail (cfg.tail_lanes) takes a wave's last <= 16 rays 64/R lanes per
    ray; their stacks stay in the home lanes' LDS and spill columns. A batch of a few
    comb rays enters it at once and pushes through the spill slab: the hand answer for
    every ray, closest and any hit."""
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, ray, expect = kat.scene_comb(depth)
    saved = tracer.config()
    try:
        tracer.set_config(wide=1, tail_lanes=16)
        tracer.set_bvh(GpuBvh(bufs))
        for closest in (True, False):
            rb = RayBuffer(np.stack([ray] * rays_n), need_closest_hit=closest)
            rb.results.fill_(0x5A5A5A5A)
            tracer.trace_batch(rb, exact_rcp=True)
            res = rb.results_numpy()
            assert tracer.last_info["stack_overflows"] == 0
            assert (res[:, 2:] == 0x5A5A5A5A).all()
            if closest:
                assert (res[:, 0] == expect[0]).all() and (res[:, 1] == kat.f2i(expect[1])).all()
            else:
                assert (res[:, 0] >= 0).all()
    finally:
        tracer.set_config(**saved)


@pytest.mark.parametrize("depth", [12, 14])
@pytest.mark.parametrize("rays_n", [1, 3, 16, 17])
def test_frontier_tail_on_wide_lists(tracer, depth, rays_n):
    """a ray that hits every box of a complete 4-ary tree (kat.scene_complete)
    makes the frontier tail's list grow by three per expanded node, past the depth-first
    walk's worst case that sizes the stack. The tail keeps the tree's depth-first bound free
    before a wide step (bind_info stack_bound), so no entry is pushed past stack_capacity:
    no overflow, and the oracle's (and the hand) answer, closest and any hit, a miss and a
    hit in the last leaf."""
    from mrt.tracer import GpuBvh, RayBuffer
    saved = tracer.config()
    try:
        tracer.set_config(wide=1, tail_lanes=16, autotune=0)
        for hit_last in (False, True):
            bufs, ray, expect = kat.scene_complete(depth, hit_last)
            tracer.set_bvh(GpuBvh(bufs))
            bi = tracer.bind_info()
            assert bi["wide_format"] == 1 and bi["stack_bound"] == 3 * depth // 2
            rays = np.stack([ray] * rays_n)
            for closest in (True, False):
                want, _, _ = O.trace(rays, *bufs, any_hit=not closest)
                rb = RayBuffer(rays, need_closest_hit=closest)
                rb.results.fill_(0x5A5A5A5A)
                tracer.trace_batch(rb, exact_rcp=True)
                res = rb.results_numpy()
                assert tracer.last_info["stack_overflows"] == 0
                assert (res[:, 2:] == 0x5A5A5A5A).all()
                assert np.array_equal(res[:, :2], want[:, :2])
                assert (res[:, 0] == expect[0]).all() and (res[:, 1] == kat.f2i(expect[1])).all()
    finally:
        tracer.set_config(**saved)


@pytest.mark.parametrize("wl", WORKLOADS, ids=lambda w: "-".join(map(str, w)))
@pytest.mark.parametrize("tail", [0, 16])
def test_tail_lanes_keep_results(tracer, wl, tail):
    """Closest hits bit-identical to the oracle with the frontier tail off and at its
    widest (the tail tests the leaves that can hold the closest hit; within a step the
    first of equal t in list order wins, as in the sequential loop); any hit: genuine
    hits, same hit/miss."""
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    saved = tracer.config()
    try:
        tracer.set_config(tail_lanes=tail, waves_per_cu=4)
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
    finally:
        tracer.set_config(**saved)
    if any_hit:
        assert_valid_hits(rays, res, want, bufs)
    else:
        assert np.array_equal(res[:, :2], want[:, :2])


def fuzz_rays(scene, n, seed, w=96, h=72):
    """Incoherent rays inside a scene (test_random_rays_fuzz's recipe)."""
    bufs, base, _, _, _ = scene_setup(scene, w, h, "primary")
    prim, _, _ = O.trace(base, *bufs)
    hits = np.nonzero(prim[:, 0] >= 0)[0]
    rng = np.random.default_rng(seed)
    pick = rng.choice(hits, n)
    t = prim[pick, 1].view(np.float32)
    p = base[pick, 0:3] + base[pick, 4:7] * t[:, None]
    extent = float(np.ptp(p, axis=0).max())
    rays = np.empty((n, 8), np.float32)
    rays[:, 0:3] = p + rng.normal(0.0, 0.05 * extent, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 3] = np.where(rng.random(n) < 0.5, 0.0, rng.uniform(0.0, 0.01 * extent, n))
    rays[:, 7] = np.where(rng.random(n) < 0.2, np.inf, rng.uniform(0.05, 2.0, n) * extent)
    return bufs, rays


@pytest.mark.parametrize("scene", ["bunny", "hairball:800", "sibenik"])
def test_frontier_tail_group_widths(tracer, scene):
    """The frontier tail gives a wave's last R <= 16 rays 64/R lanes each (F = 16/R entries
    per round trip) and widens the groups as rays finish. Batches of 1..64 rays land in
    one wave, so every group width (4..64 lanes), the regroups, the window's overflow onto
    the home stack and the pops back from it all run: closest hits bit-identical to the
    oracle, any hits genuine with the same hit/miss, no stack overflow."""
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, rays = fuzz_rays(scene, 1200, 7)
    want = {a: O.trace(rays, *bufs, any_hit=a, threads=8)[0] for a in (False, True)}
    saved = tracer.config()
    try:
        tracer.set_config(wide=1, tail_lanes=16, autotune=0)
        tracer.set_bvh(GpuBvh(bufs))
        lo = 0
        for n in (1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33, 64, 1, 1, 2, 3):
            for any_hit in (False, True):
                rb = RayBuffer(rays[lo:lo + n], need_closest_hit=not any_hit)
                rb.results.fill_(0x5A5A5A5A)
                tracer.trace_batch(rb, exact_rcp=True)
                res = rb.results_numpy()
                assert tracer.last_info["stack_overflows"] == 0
                assert (res[:, 2:] == 0x5A5A5A5A).all()
                if any_hit:
                    assert_valid_hits(rays[lo:lo + n], res, want[True][lo:lo + n], bufs)
                else:
                    assert np.array_equal(res[:, :2], want[False][lo:lo + n, :2]), f"batch of {n} at {lo}"
            lo += n
    finally:
        tracer.set_config(**saved)


def test_timed_trace_keeps_async_overflow_count(tracer):
    """a blocking trace counts its own overflows in a slot of its own; the
    sticky counter of earlier asynchronous launches on the stream is not reset by it."""
    from mrt import _lib
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, ray, expect = kat.scene_comb(70)
    saved = tracer.config()
    tracer.set_config(wide=0)
    tracer.set_bvh(GpuBvh(bufs))
    n = C.c_int64()
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 1))
    rb = RayBuffer(np.stack([ray] * 64), need_closest_hit=True)
    tracer.trace_async(rb, exact_rcp=True, speculative=False)        # overflows, sticky
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 1))
    one = n.value                                                    # one launch's pushes past capacity
    assert one == 64 * (70 - 63)
    tracer.trace_async(rb, exact_rcp=True, speculative=False)
    with pytest.raises(_lib.MrtError, match=f"{one} stack pushes"):
        tracer.trace_batch(rb, exact_rcp=True, speculative=False)    # its own count
    _lib.check(tracer.lib.mrt_tracer_stack_overflows(tracer._h, C.byref(n), 1))
    assert n.value == one   # the async launch's count: not reset by the blocking one, not added to
    tracer.set_config(**saved)


def test_oversized_batch_rejected(tracer):
    """ray/result addressing stays inside int32 — more than 2^30 rays per
    launch is refused before anything is read (the caller splits the batch)."""
    from mrt.tracer import GpuBvh
    tracer.set_bvh(GpuBvh(kat.scene_two_floors()))
    dummy = torch.zeros(16, dtype=torch.int32, device="cuda")
    rc = tracer.lib.mrt_tracer_trace(tracer._h, dummy.data_ptr(), dummy.data_ptr(), (1 << 30) + 1, 0, None, None)
    assert rc == 5   # MRT_ERR_TOO_LARGE


def test_invalid_config_rejected(tracer):
    from mrt._lib import MrtError
    with pytest.raises(MrtError):
        tracer.set_config(lds_stack=12)
    with pytest.raises(MrtError):
        tracer.set_config(num_queues=9)
    with pytest.raises(MrtError):
        tracer.set_config(lane_groups=3)
    with pytest.raises(MrtError):
        tracer.set_config(spec_slack=64)
    with pytest.raises(MrtError):
        tracer.set_config(wide=3)


# ---------------------------------------------------------------- edge cases
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097])
def test_ragged_batch_sizes(tracer, n):
    bufs, rays, any_hit, want, _ = scene_setup("bunny", 320, 240, "primary")
    res, _ = gpu_trace(tracer, bufs, rays[:n], False, exact=True, spec=True)
    assert np.array_equal(res[:, :2], want[:n, :2])


def special_rays(base, seed=7):
    """Rays with the values a caller can hand the kernel without meaning to: axis-parallel
    directions with +-0 components (the 2^-80 clamp keeps the zero's sign), a zero
    direction, denormal components (flushed), NaN / inf components, tmin > tmax,
    tmin == tmax, a huge negative tmin, tmax = inf / NaN, origins 1e30 away, and rays
    starting exactly on their own first hit point. Built from primary rays `base`."""
    rng = np.random.default_rng(seed)
    k = 192
    sel = rng.choice(len(base), k)
    o, tmin, d, tmax = base[sel, 0:3], base[sel, 3], base[sel, 4:7], base[sel, 7]
    groups = []

    def add(o_=None, tmin_=None, d_=None, tmax_=None):
        r = np.empty((k, 8), np.float32)
        r[:, 0:3] = o if o_ is None else o_
        r[:, 3] = tmin if tmin_ is None else tmin_
        r[:, 4:7] = d if d_ is None else d_
        r[:, 7] = tmax if tmax_ is None else tmax_
        groups.append(r)

    for axis in range(3):
        dd = np.zeros((k, 3), np.float32)
        dd[:, axis] = np.where(rng.random(k) < 0.5, 1.0, -1.0)
        dd[k // 2:, (axis + 1) % 3] = -0.0
        add(d_=dd)
    add(d_=np.zeros((k, 3), np.float32))
    dd = d.copy()
    dd[:, 0] = np.float32(1e-40)
    dd[: k // 2, 1] = np.float32(-3e-39)
    add(d_=dd)
    for j in range(3):
        oo = o.copy()
        oo[:, j] = np.nan
        add(o_=oo)
        dd = d.copy()
        dd[:, j] = np.nan
        add(d_=dd)
        dd = d.copy()
        dd[:, j] = np.where(rng.random(k) < 0.5, np.inf, -np.inf)
        add(d_=dd)
    add(tmin_=tmax + 1.0)
    add(tmin_=tmax)
    add(tmin_=np.full(k, -1e30, np.float32))
    add(tmax_=np.full(k, np.inf, np.float32))
    add(tmax_=np.full(k, np.nan, np.float32))
    add(tmin_=np.full(k, np.nan, np.float32))
    add(o_=(o - d * np.float32(1e30)).astype(np.float32))
    return np.concatenate(groups)


@pytest.mark.parametrize("scene", ["bunny", "hairball:800", "sponza"])
def test_special_value_rays(tracer, scene):
    """Edge-value rays (special_rays) traced against the oracle: the per-lane order walks
    the same Compact2 nodes with the same arithmetic, so id, t and the counters are
    bit-identical whatever the values; the speculative 4-wide mode gives the same
    closest hits and the same any-hit hit/miss."""
    bufs, base, _, _, _ = scene_setup(scene, 64, 48, "primary")
    rays = special_rays(base)
    # rays that start on their first hit point (t of the hit along the ray, tmin 0)
    prim, _, _ = O.trace(base, *bufs)
    hit = np.nonzero(prim[:, 0] >= 0)[0][:192]
    on = base[hit].copy()
    on[:, 0:3] = on[:, 0:3] + on[:, 4:7] * prim[hit, 1].view(np.float32)[:, None]
    on[:, 3] = 0.0
    rays = np.concatenate([rays, on.astype(np.float32)])
    for any_hit in (False, True):
        want, st, _ = O.trace(rays, *bufs, any_hit=any_hit, stats=True)
        res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
        assert np.array_equal(res[:, :2], want[:, :2]), f"per-lane order, any_hit={any_hit}"
        assert np.array_equal(gst[:, :3], st[:, :3]), f"per-lane counters, any_hit={any_hit}"
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        if any_hit:
            assert np.array_equal(res[:, 0] == -1, want[:, 0] == -1), "speculative any-hit hit/miss"
        else:
            bad = np.nonzero((res[:, 0] != want[:, 0]) | (res[:, 1] != want[:, 1]))[0]
            assert len(bad) == 0, f"speculative closest hit differs on rays {bad[:8]} (of {len(rays)})"


@pytest.mark.parametrize("scene", ["bunny", "conference", "hairball:800", "sibenik"])
@pytest.mark.parametrize("seed", [1, 2])
def test_random_rays_fuzz(tracer, scene, seed):
    """Incoherent random rays inside the scene: origins scattered around the primary
    hit points, uniform directions, random tmin/tmax (some infinite). Both modes against
    the oracle: per-lane order bit-identical with counters, speculative 4-wide closest
    hits identical, any-hit hit/miss identical with every reported hit a valid one."""
    bufs, base, _, _, _ = scene_setup(scene, 96, 72, "primary")
    prim, _, _ = O.trace(base, *bufs)
    hits = np.nonzero(prim[:, 0] >= 0)[0]
    rng = np.random.default_rng(seed)
    n = 12000
    pick = rng.choice(hits, n)
    t = prim[pick, 1].view(np.float32)
    p = base[pick, 0:3] + base[pick, 4:7] * t[:, None]
    extent = float(np.ptp(p, axis=0).max())
    rays = np.empty((n, 8), np.float32)
    rays[:, 0:3] = p + rng.normal(0.0, 0.05 * extent, (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 3] = np.where(rng.random(n) < 0.5, 0.0, rng.uniform(0.0, 0.01 * extent, n))
    rays[:, 7] = np.where(rng.random(n) < 0.2, np.inf, rng.uniform(0.05, 2.0, n) * extent)
    for any_hit in (False, True):
        want, st, _ = O.trace(rays, *bufs, any_hit=any_hit, stats=True, threads=8)
        res, gst = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=False, stats=True)
        assert np.array_equal(res[:, :2], want[:, :2])
        assert np.array_equal(gst[:, :3], st[:, :3])
        res, _ = gpu_trace(tracer, bufs, rays, any_hit, exact=True, spec=True)
        if any_hit:
            assert_valid_hits(rays, res, want, bufs)
        else:
            assert np.array_equal(res[:, :2], want[:, :2])


def test_empty_batch_returns_zero_ms(tracer):
    from mrt.tracer import GpuBvh, RayBuffer
    tracer.set_bvh(GpuBvh(kat.scene_two_floors()))
    rb = RayBuffer(np.zeros((0, 8), np.float32))
    assert tracer.trace_batch(rb) == 0.0


def test_trace_before_bind_fails(tracer):
    from mrt._lib import MrtError
    from mrt.tracer import RayBuffer, Tracer
    t = Tracer(0)
    rb = RayBuffer(np.zeros((4, 8), np.float32))
    with pytest.raises(MrtError):
        t.trace_batch(rb)
    lib = t.lib
    rc = lib.mrt_tracer_trace(t._h, rb.rays.data_ptr(), rb.results.data_ptr(), 4, 0, None, None)
    assert rc == 2   # MRT_ERR_NOT_BOUND


def test_rebinding_a_different_bvh(tracer):
    b1, rays1, _, want1, _ = scene_setup("bunny", 320, 240, "primary")
    b2, rays2, any2, want2, _ = scene_setup("mori", 256, 192, "ao")
    r1, _ = gpu_trace(tracer, b1, rays1, False)
    r2, _ = gpu_trace(tracer, b2, rays2, True, spec=False)
    r1b, _ = gpu_trace(tracer, b1, rays1, False)
    assert np.array_equal(r1[:, :2], want1[:, :2]) and np.array_equal(r1b[:, :2], want1[:, :2])
    assert np.array_equal(r2[:, :2], want2[:, :2])


def test_reference_compat_entry_points(tracer):
    """bind_CudaBVHTexture + launch_tracingKernel + copy_tracing_results, exactly
    the reference call sequence of CudaTracer::traceBatch (CudaTracer.cc:142-177)."""
    from mrt import _lib
    bufs, rays, any_hit, want, _ = scene_setup("bunny", 320, 240, "primary")
    lib = _lib.trace_lib()
    nodes, woop, tri = (torch.from_numpy(b).cuda() for b in bufs)
    r = torch.from_numpy(rays).cuda()
    out = torch.zeros((len(rays), 4), dtype=torch.int32, device="cuda")
    lib.bind_CudaBVHTexture(nodes.data_ptr(), nodes.numel() * 4, woop.data_ptr(), woop.numel() * 4, tri.data_ptr(),
                            tri.numel() * 4)
    block = (C.c_int32 * 2)(32, 4)
    ms = lib.launch_tracingKernel(180 * 128, block, len(rays), False, r.data_ptr(), out.data_ptr(),
                                  nodes.data_ptr(), None, None, None, woop.data_ptr(), None, None, tri.data_ptr())
    assert ms > 0.0
    host = np.zeros((len(rays), 4), np.int32)
    lib.copy_tracing_results(host.ctypes.data, out.data_ptr(), len(rays))
    # The compat launch keeps the reference's fast reciprocal (rcp.approx there,
    # v_rcp_f32 here): ids identical, t within the fast-mode tolerance.
    assert np.array_equal(host[:, 0], want[:, 0])
    assert ulp_diff(host[:, 1], want[:, 1]).max() <= 2
    lib.unbind_CudaBVHTexture()


@pytest.mark.parametrize("wl", [("bunny", 320, 240, "primary"), ("conference", 256, 192, "ao")],
                         ids=lambda w: "-".join(map(str, w)))
def test_cpp_host_links_reference_prototypes(tmp_path, wl):
    """A C++ CudaTracer written against the reference's CudaTracerKernels.hh:42-52
    prototypes (tests/cpp/cuda_tracer_dropin.cpp), linked to libmrt.so, run as a
    child process: the reference's host side works unchanged on top of the library."""
    import subprocess
    exe = os.path.join(REPO, "gpu-ray-tracing_amd", "lib", "cuda_tracer_dropin")
    assert os.path.exists(exe), "build it: make -C gpu-ray-tracing_amd"
    bufs, rays, any_hit, want, _ = scene_setup(*wl)
    names = []
    for name, arr in zip(("nodes", "woop", "tri", "rays"), (*bufs, rays)):
        path = tmp_path / f"{name}.bin"
        np.ascontiguousarray(arr).tofile(path)
        names.append(str(path))
    out = tmp_path / "results.bin"
    r = subprocess.run([exe, *names, str(int(any_hit)), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, np.int32).reshape(-1, 4)
    assert len(got) == len(rays)
    # launch_tracingKernel keeps the reference's fast reciprocal (rcp.approx there, v_rcp_f32 here).
    if any_hit:
        assert np.array_equal(got[:, 0] == -1, want[:, 0] == -1)
    else:
        assert np.array_equal(got[:, 0], want[:, 0])
        assert ulp_diff(got[:, 1], want[:, 1]).max() <= 2
    assert not got[:, 2:].any()   # RayResult pads untouched


def test_async_trace_on_a_side_stream(tracer):
    from mrt.tracer import GpuBvh, RayBuffer
    bufs, rays, any_hit, want, _ = scene_setup("sponza", 256, 192, "diffuse")
    tracer.set_bvh(GpuBvh(bufs))
    s = torch.cuda.Stream()
    rb = RayBuffer(rays, need_closest_hit=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        tracer.trace_async(rb, exact_rcp=True, stream=s)
    s.synchronize()
    assert np.array_equal(rb.results_numpy()[:, :2], want[:, :2])


# ---------------------------------------------------------------- full size
def test_full_size_bunny_primary_1024x768(tracer):
    """The bench's headline workload, bit-identical to the oracle on every ray."""
    bufs, rays, any_hit, want, st = scene_setup("bunny", 1024, 768, "primary")
    res, _ = gpu_trace(tracer, bufs, rays, False, exact=True, spec=True)
    assert np.array_equal(res[:, :2], want[:, :2])
    res2, gst = gpu_trace(tracer, bufs, rays, False, exact=True, spec=False, stats=True)
    assert np.array_equal(gst[:, :3], st[:, :3])


def test_repeated_launches_are_deterministic(tracer):
    bufs, rays, any_hit, want, _ = scene_setup("conference", 256, 192, "ao")
    a, _ = gpu_trace(tracer, bufs, rays, True, exact=True, spec=False)
    for _ in range(3):
        b, _ = gpu_trace(tracer, bufs, rays, True, exact=True, spec=False)
        assert np.array_equal(a[:, :2], b[:, :2])
