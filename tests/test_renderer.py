"""Frame orchestration (mrt/renderer.py): RayGen::batching and Renderer::nextBatch
(RayGen.cc:124-142, Renderer.cc:242-291), the glibc rand() batch seeds (RayGen.cc:106),
and the device AO/diffuse generator against an independent numpy restatement of
rayGenAOKernel (oracle/raygen_oracle.py, RayGenKernels.cu:117-227)."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import mrt  # noqa: E402
import oracle_lib as O  # noqa: E402
import raygen_oracle as RO  # noqa: E402
from mrt.renderer import MAX_BATCH_RAYS, GlibcRand, batching  # noqa: E402


@pytest.mark.parametrize("seed", [1, 12345, 0x7FFFFFFF, 0x80000001])
def test_glibc_rand_restatement_equals_the_c_library(seed):
    """The reference seeds each AO batch with rand() (RayGen.cc:106), never srand'ed:
    the restated generator must equal glibc's own rand() for the same seed."""
    libc = C.CDLL("libc.so.6")
    libc.srand.argtypes = [C.c_uint]
    libc.srand(seed)
    want = [libc.rand() for _ in range(1000)]
    r = GlibcRand(seed)
    assert [r() for _ in range(1000)] == want


def test_glibc_rand_known_answers():
    r = GlibcRand()
    assert [r() for _ in range(3)] == [1804289383, 846930886, 1681692777]   # glibc's documented first outputs
    assert mrt.AO_SEED == 1804289383


def test_batching_follows_raygen():
    """RayGen::batching with maxBatchSize 2^21 (Renderer.cc:46): 1920x1080 primaries at
    8 samples -> 7 batches of 262144 primaries and one of 238592."""
    n, s = 1920 * 1080, 8
    ranges, start = [], 0
    while (r := batching(n, s, start)) is not None:
        ranges.append(r)
        start = r[1]
    assert len(ranges) == 8
    assert all(hi - lo == MAX_BATCH_RAYS // s for lo, hi in ranges[:7])
    assert ranges[-1] == (7 * 262144, n)
    assert batching(307200, 1, 0) == (0, 307200)            # README frames: one batch
    assert batching(307200, 1, 307200) is None
    assert batching(10, 3, 9, max_batch=4) == (9, 10)       # maxBatch / numSamples primaries (floor)
    with pytest.raises(mrt._lib.MrtError):
        batching(10, 8, 0, max_batch=4)


def test_hash_angle_restatement_matches_the_host_generator():
    """The numpy Jenkins hash (RayGenKernels.cu:36-47,162-167) against the product's host
    generator on a single-triangle scene whose basis is known."""
    scene = mrt.Scene.from_arrays([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]])
    prim = np.zeros((5, 8), np.float32)
    prim[:, 0:3] = [0.25, 0.25, 1.0]
    prim[:, 4:7] = [0.0, 0.0, -1.0]
    prim[:, 7] = 10.0
    res = np.zeros((5, 4), np.int32)
    res[:, 0] = 0
    res[:, 1] = np.float32(1.0).view(np.int32)
    host = mrt.ao_rays(prim, res, scene, 5.0, 1, 77)
    want = RO.ao_rays(prim, res, scene.arrays()[2], 1, 5.0, 77)
    assert np.array_equal(host[:, 0:3].view(np.uint32), want["origin"].view(np.uint32))
    assert np.abs(host[:, 4:7] - want["dir"]).max() < 4e-6
    assert (host[:, 6] > 0).all()                            # hemisphere of the viewer-facing normal (+z)


# ---------------------------------------------------------------- GPU


@pytest.fixture(scope="module")
def sponza():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mrt.tracer import GpuBvh, Tracer
    scene = mrt.Scene.synthetic("sponza", 0, 1)
    bufs = mrt.Bvh.build(scene).buffers()
    t = Tracer(0)
    t.set_bvh(GpuBvh(bufs))
    return scene, bufs, t


def check_rays_against_raygen_oracle(batch_rays, prim_rays, prim_res, normals, samples, max_dist, seed):
    want = RO.ao_rays(prim_rays, prim_res, normals, samples, max_dist, seed)
    got = batch_rays
    assert np.array_equal(got[:, 0:3].view(np.uint32), want["origin"].view(np.uint32)), "origin"
    assert np.array_equal(got[:, 3].view(np.uint32), want["tmin"].view(np.uint32)), "tmin"
    assert np.array_equal(got[:, 7].view(np.uint32), want["tmax"].view(np.uint32)), "tmax"
    assert np.abs(got[:, 4:7] - want["dir"]).max() < 1e-5, "direction"
    live = want["tmax"] > 0
    cosn = (got[live, 4:7].astype(np.float64) * want["normal"][live]).sum(1)
    assert (cosn >= -1e-6).all(), "a sample left the viewer-facing hemisphere"


@pytest.mark.gpu
@pytest.mark.parametrize("ray_type,samples,w,h", [(2, 8, 640, 480), (1, 16, 400, 360), (2, 1, 320, 240)])
def test_renderer_batches_equal_the_oracle(sponza, ray_type, samples, w, h):
    """A frame traced as RayGen::batching batches: 640x480x8 diffuse = 2.46 M rays -> two
    batches (2^21 + 360448). Every batch: rays equal the numpy rayGenAOKernel restatement
    with that batch's glibc seed, results equal the oracle traced over the same rays, and
    the frame's pixels (reconstructed batch by batch) equal the oracle's reconstruction."""
    from mrt.renderer import Renderer
    scene, bufs, t = sponza
    cam, ao = scene.camera()
    normals = scene.arrays()[2]
    r = Renderer(t, scene)
    r.set_params(ray_type, samples, ao)
    r.begin_frame(cam, w, h)
    prim_rays, prim_res = r.primary.rays.cpu().numpy(), r.primary.results_numpy()
    assert r.total_num_rays() == int((prim_res[:, 0] != -1).sum()) * samples
    seeds = GlibcRand()
    pixels = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    starts, total, bres = [], 0, []
    while r.next_batch():
        seed = seeds()
        t_ms = r.trace_batch()
        assert t_ms > 0
        assert r.batch.size <= MAX_BATCH_RAYS
        lo = r.batch_start // samples
        n = r.batch.size // samples
        rays = r.batch.rays.cpu().numpy()
        check_rays_against_raygen_oracle(rays, prim_rays[lo:lo + n], prim_res[lo:lo + n], normals, samples,
                                         ao if ray_type == 1 else cam.far, seed)
        want, _, _ = O.trace(rays, *bufs, any_hit=ray_type == 1, threads=8)
        got = r.batch.results_numpy()
        if ray_type == 1:
            assert np.array_equal(got[:, 0] == -1, want[:, 0] == -1)
            # reconstruct from the oracle's hits: any-hit ids may legitimately differ
            r.batch.results[:, :2] = torch.from_numpy(np.ascontiguousarray(want[:, :2])).cuda()
        else:
            assert np.array_equal(got[:, :2], want[:, :2])
        r.update_result(pixels)
        bres.append(want)
        starts.append(r.batch_start)
        total += r.batch.size
    assert total == w * h * samples
    per_batch = MAX_BATCH_RAYS // samples * samples
    assert starts == list(range(0, total, per_batch))
    assert len(starts) == -(-total // per_batch)
    # the frame's pixels, reconstructed batch by batch on the device, equal the oracle's
    # reconstruction of the whole frame from the concatenated batch results
    mat, sh = O.tri_colors(normals)
    want_px = O.reconstruct(ray_type, samples, r.slot_to_id.cpu().numpy(), prim_res, np.concatenate(bres), mat, sh,
                            w * h)
    assert np.array_equal(pixels.cpu().numpy().view(np.uint32), want_px)


@pytest.mark.gpu
@pytest.mark.parametrize("ray_type,samples,w,h,max_batch,block,world", [
    (2, 8, 320, 240, 1 << 16, 1024, 3),     # 10 batches; blocks a multiple of the samples
    (1, 3, 97, 61, 1 << 12, 100, 2),        # ragged: 3 samples, 100-ray blocks, a partial last block
    (2, 1, 160, 120, 1 << 21, 4096, 1),     # one batch, the whole frame live blocks first
    (1, 256, 24, 16, 1 << 16, 2048, 2),     # the tiled generator at its sample limit (256 per input ray)
    (2, 512, 16, 12, 1 << 21, 1024, 2),     # more samples than the tile's LDS slots: the per-ray generator
])
def test_secondary_blocks_equal_the_frame_batches(sponza, ray_type, samples, w, h, max_batch, block, world):
    """Renderer.secondary_blocks (mrt_raygen_ao_blocks): each rank's shard of
    the frame generated directly in its trace order (live blocks first) is bit-identical to
    the frame's RayGen::batching batches gathered at the shard's blocks, and the shards
    together hold every ray of the frame once. The live counts per block from the primary
    pass equal the generated rays' own (tmax >= 0)."""
    from mrt.dist import block_weights, live_block_weights, shard_blocks_device, shard_spans, spans_index
    from mrt.renderer import Renderer
    scene, bufs, t = sponza
    cam, ao = scene.camera()
    r = Renderer(t, scene, max_batch=max_batch)
    r.set_params(ray_type, samples, ao)
    r.begin_frame(cam, w, h)
    n = w * h * samples
    frame = torch.cat([b.rays for b, _ in r.batches()])      # seeds drawn here, in batch order
    assert frame.shape[0] == n and r.num_batches() == -(-w * h // (max_batch // samples))
    wdev = live_block_weights(r.primary.results, samples, block)
    assert torch.equal(wdev.cpu(), block_weights(frame, block).cpu())
    prio = wdev.cpu().numpy()
    seen = torch.zeros(n, dtype=torch.int32, device="cuda")
    for rank in range(world):
        blocks, m = shard_blocks_device(n, world, rank, block, priority=wdev, device="cuda")
        shard = r.secondary_blocks(blocks, m, block)
        assert shard.secondary and shard.need_closest_hit == (ray_type == 2)
        idx = spans_index(shard_spans(n, world, rank, block, None, prio), "cuda")
        assert shard.size == m == idx.numel()
        assert torch.equal(shard.rays, frame.index_select(0, idx)), f"rank {rank}: shard rays differ"
        seen.index_add_(0, idx, torch.ones_like(idx, dtype=torch.int32))
    assert bool((seen == 1).all())


@pytest.mark.gpu
def test_secondary_blocks_rejects_bad_lists(sponza):
    from mrt.renderer import Renderer
    scene, _, t = sponza
    cam, ao = scene.camera()
    r = Renderer(t, scene)
    r.set_params(1, 2, ao)
    r.begin_frame(cam, 32, 32)
    blocks = torch.arange(0, 8, dtype=torch.int32, device="cuda")
    with pytest.raises(mrt._lib.MrtError):
        r.secondary_blocks(blocks, 8 * 64 + 1, 64)           # more rays than the blocks hold
    with pytest.raises(mrt._lib.MrtError):
        r.secondary_blocks(torch.arange(0, 40, dtype=torch.int32, device="cuda"), 40 * 64, 64)   # > the frame's 32
    out = r.secondary_blocks(blocks[:0], 0, 64)
    assert out.size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("samples,w,h,block,world", [(8, 320, 240, 1024, 3), (3, 97, 61, 128, 2), (1, 160, 120, 4096, 1),
                                                    (2, 200, 100, 8192, 2)])
def test_library_shard_order_equals_the_host_deal(sponza, samples, w, h, block, world):
    """mrt_shard_blocks (Renderer.shard): every rank's blocks, in frame order and live blocks
    first, equal the host's deal (shard_blocks with live_priority — the gather's spans), and the
    shard's rays equal the frame's batches at those positions; a 8192-ray block exercises the
    quantized keys."""
    from mrt.dist import live_block_weights, live_priority, shard_blocks, shard_spans, spans_index
    from mrt.renderer import Renderer
    scene, bufs, t = sponza
    cam, ao = scene.camera()
    r = Renderer(t, scene, max_batch=1 << 15)
    r.set_params(2, samples, ao)
    r.begin_frame(cam, w, h)
    n = w * h * samples
    frame = torch.cat([b.rays for b, _ in r.batches()])
    prio = live_priority(live_block_weights(r.primary.results, samples, block).cpu(), block)
    for order in (0, 1):
        for rank in range(world):
            blocks, m = r.gen.shard_blocks(r.primary, samples, block, world, rank, order)
            want = shard_blocks(n, world, rank, block, priority=prio if order else None)
            assert np.array_equal(blocks.cpu().numpy(), want), f"order {order} rank {rank}"
            shard = r.shard(world, rank, block, order=order)
            idx = spans_index(shard_spans(n, world, rank, block, None, prio if order else None), "cuda")
            assert shard.size == m == idx.numel()
            assert torch.equal(shard.rays, frame.index_select(0, idx))
