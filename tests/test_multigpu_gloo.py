"""World-size-2/3 rehearsal of the multi-GPU path with gloo: the BVH is
replicated from rank 0, rays are sharded (contiguous ranges, or block-cyclic
blocks), each rank traces its shard, and the results are gathered to rank 0 in
ray order. On CPU the oracle
stands in for the per-GPU tracer; the GPU test runs two ranks on one MI355X
through the real HIP tracer (mrt.dist.trace_shard, the bench's strong-scaling
step) and gathers with gather_results."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mrt.dist import local_rays, shard_launches, shard_range, shard_spans


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, block=0):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "gpu-ray-tracing_amd"))
    import mrt
    import oracle_lib as O
    from mrt.dist import gather_results, replicate_buffers

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene = mrt.Scene.synthetic("mori", 0, 1)
    bufs = mrt.Bvh.build(scene).buffers() if rank == 0 else None
    nodes, woop, tri = (t.numpy() for t in replicate_buffers(bufs, src=0, device=torch.device("cpu")))
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 61, 37)          # ragged: 2257 rays, not a multiple of the world size
    mine = local_rays(torch.from_numpy(rays), shard_spans(len(rays), world, rank, block)).numpy()
    res, _, _ = O.trace(mine, nodes, woop, tri)
    full = gather_results(torch.from_numpy(res), len(rays), dst=0, block=block)
    if rank == 0:
        want, _, _ = O.trace(rays, *mrt.Bvh.build(scene).buffers())
        np.save(out_path, np.stack([full.numpy()[:, 0], want[:, 0], full.numpy()[:, 1], want[:, 1]]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,block", [(2, 0), (3, 0), (2, 100), (3, 64)])
def test_replicate_shard_gather(tmp_path, world, block):
    """block 0: contiguous shards; block > 0: block-cyclic shards (a ragged last block)."""
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, block), nprocs=world, join=True)
    a = np.load(out)
    assert np.array_equal(a[0], a[1]) and np.array_equal(a[2], a[3])


def test_block_cyclic_spans_partition():
    """Every ray in exactly one shard; blocks dealt round-robin; shard sizes within one block."""
    for n in (0, 1, 99, 100, 101, 16588800):
        for w in (1, 2, 3, 8):
            for block in (1, 100, 1 << 14):
                spans = [shard_spans(n, w, r, block) for r in range(w)]
                flat = sorted(s for sp in spans for s in sp)
                assert sum(b - a for a, b in flat) == n
                assert all(flat[i][1] == flat[i + 1][0] for i in range(len(flat) - 1))
                if n and w > 1:
                    assert all(a // block % w == r for r, sp in enumerate(spans) for a, _ in sp)
                sizes = [sum(b - a for a, b in sp) for sp in spans]
                assert max(sizes) - min(sizes) <= max(block, 1)


def test_shard_launches_balanced():
    assert shard_launches(0, 16588800, 1 << 21) == [(i * 2073600, (i + 1) * 2073600) for i in range(8)]
    assert shard_launches(100, 2073700, 1 << 21, 2) == [(100, 1036900), (1036900, 2073700)]
    assert shard_launches(5, 5, 10) == []
    spans = shard_launches(0, 12345, 1000, 3)
    assert len(spans) == 13 and spans[0][0] == 0 and spans[-1][1] == 12345
    assert max(b - a for a, b in spans) <= 1000


def test_shard_ranges_partition():
    for n in (0, 1, 7, 64, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _gpu_worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "gpu-ray-tracing_amd"))
    import mrt
    from mrt.dist import gather_results, replicate_buffers, trace_shard
    from mrt.raygen import DeviceRayGen
    from mrt.tracer import GpuBvh, Tracer

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene = mrt.Scene.synthetic("hairball", 800, 1)
    bufs = mrt.Bvh.build(scene).buffers() if rank == 0 else None
    rep = replicate_buffers(bufs, src=0, device=torch.device("cpu"))
    tracer = Tracer(0)
    tracer.set_bvh(GpuBvh(tuple(rep)))
    cam, _ = scene.camera()
    gen = DeviceRayGen(scene)
    prim, _ = gen.primary(cam, 173, 91)
    tracer.trace_batch(prim, exact_rcp=True)
    rays = gen.ao(prim, 3, cam.far, closest_hit=True)   # one fixed RayBuffer, identical on every rank
    local = trace_shard(tracer, rays, world, rank, max_rays=4096, block=1000)   # block-cyclic, several launches
    torch.cuda.synchronize()
    full = gather_results(local.results.cpu(), rays.size, dst=0, block=1000)
    if rank == 0:
        np.save(out_path + ".rays.npy", rays.rays.cpu().numpy())
        np.save(out_path + ".res.npy", full.numpy())
        for name, b in zip(("nodes", "woop", "tri"), rep):
            np.save(out_path + f".{name}.npy", b.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_trace_shards_and_gather(tmp_path):
    """Two gloo ranks sharing one MI355X: replicate -> shard (strong scaling: one fixed
    RayBuffer, block-cyclic shards of 1000-ray blocks, <= 4096-ray launches) -> HIP
    trace -> gather to rank 0;
    the gathered {id, t} equal the oracle over the whole buffer."""
    import oracle_lib as O
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path / "g")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    rays = np.load(out + ".rays.npy")
    got = np.load(out + ".res.npy")
    bufs = tuple(np.load(out + f".{n}.npy") for n in ("nodes", "woop", "tri"))
    want, _, _ = O.trace(rays, *bufs, threads=8)
    assert len(got) == len(rays) == 173 * 91 * 3
    assert np.array_equal(got, want[:, :2])


def test_block_sums_and_weights():
    """Per-block traversal cost (mrt.dist.block_sums, the strong-scaling cost order) and the
    live-ray count (block_weights): a ragged last block is summed over its rays only."""
    from mrt.dist import block_sums, block_weights
    v = torch.arange(10, dtype=torch.int32)
    assert block_sums(v, 4).tolist() == [6, 22, 17]
    rays = torch.zeros((10, 8))
    rays[[0, 5, 9], 7] = -1.0
    assert block_weights(rays, 4).tolist() == [3, 3, 1]
    spans = shard_spans(10, 1, 0, 4, priority=block_sums(v, 4))
    assert spans == [(4, 8), (0, 4), (8, 10)]   # costliest block first, the partial last block last
    assert shard_spans(12, 1, 0, 4, priority=[6, 22, 17]) == [(4, 12), (0, 4)]   # adjacent blocks 1, 2 merged


def test_live_block_weights_follow_the_primary_hits():
    """live_block_weights: a frame's secondary ray is live (tmax >= 0) iff its primary ray hit
    (RayGenKernels.cu:117-227), so the live count per block of the frame's ray order is known
    from the primary results: equal to block_weights of the generated rays, for block sizes
    that are and are not multiples of the samples, with a partial last block."""
    from mrt.dist import block_weights, live_block_weights
    g = torch.Generator().manual_seed(5)
    for n_prim, spp, block in ((37, 4, 8), (37, 3, 8), (50, 1, 7), (64, 8, 64), (5, 2, 64)):
        res = torch.zeros((n_prim, 4), dtype=torch.int32)
        res[:, 0] = torch.where(torch.rand(n_prim, generator=g) < 0.6, torch.randint(0, 9, (n_prim,), generator=g), -1)
        rays = torch.zeros((n_prim * spp, 8))
        rays[:, 7] = torch.where(res[:, 0] >= 0, 100.0, -1.0).repeat_interleave(spp)
        assert live_block_weights(res, spp, block).tolist() == block_weights(rays, block).tolist()


@pytest.mark.parametrize("n,block,world", [(1000, 64, 3), (1024, 64, 4), (17, 5, 2), (64, 64, 2)])
def test_shard_blocks_device_matches_the_host_order(n, block, world):
    """shard_blocks_device (the device deal used to generate shards) equals shard_blocks and
    shard_spans on the host for the same priorities: every rank's blocks in the same order,
    the ray counts right, the partial block last, every ray in exactly one shard."""
    from mrt.dist import shard_blocks, shard_blocks_device, spans_index
    nb = -(-n // block)
    pr = np.random.RandomState(n).randint(0, 5, size=nb)
    seen = np.zeros(n, int)
    for prio in (None, pr):
        for r in range(world):
            host = shard_blocks(n, world, r, block, priority=prio)
            dev, m = shard_blocks_device(n, world, r, block, priority=None if prio is None else torch.tensor(prio))
            assert dev.dtype == torch.int32 and np.array_equal(dev.numpy(), host)
            if n % block and (nb - 1) in host:
                assert host[-1] == nb - 1
            idx = spans_index(shard_spans(n, world, r, block, None, prio)).numpy()
            assert len(idx) == m
            if prio is not None:
                seen[idx] += 1
    assert (seen == 1).all()


def test_partial_block_last_with_negative_priorities():
    """live_priority's values are <= 0: the frame's partial last block still comes last."""
    from mrt.dist import live_priority, shard_blocks, shard_blocks_device
    n, block = 17751, 128
    nb = -(-n // block)
    w = np.random.RandomState(3).randint(0, block + 1, size=nb)
    pr = live_priority(w, block)
    for r in range(2):
        host = shard_blocks(n, 2, r, block, priority=pr)
        dev, _ = shard_blocks_device(n, 2, r, block, priority=torch.from_numpy(pr))
        assert np.array_equal(host, dev.numpy())
        if (nb - 1) % 2 == r:
            assert host[-1] == nb - 1
