"""The RCCL ("nccl") branches of mrt/dist.py dry-run on the CPU:
torch.distributed is replaced by an in-process fake — one thread per rank,
point-to-point messages through queues, broadcast from the source rank's tensor —
that reports the "nccl" backend, so the device-tensor code paths (buffers kept
where they land, irecv into slices of the result, index_copy_ of block-cyclic
shards) run with their real shapes, offsets and ordering. The device check is
swapped for one that accepts CPU tensors (there is no GPU here); every other
check stays, and the ones that must fail loudly are exercised."""
from __future__ import annotations

import queue
import threading

import numpy as np
import pytest
import torch

from mrt import dist as D


class FakeNccl:
    """A world of `world` ranks in threads of one process."""

    def __init__(self, world):
        self.world = world
        self.local = threading.local()
        self.p2p = {(s, d): queue.Queue() for s in range(world) for d in range(world)}
        self.bcast = [queue.Queue() for _ in range(world)]
        self.log = []
        self.lock = threading.Lock()

    # torch.distributed surface used by mrt.dist
    def get_rank(self):
        return self.local.rank

    def get_world_size(self):
        return self.world

    def get_backend(self):
        return "nccl"

    def broadcast(self, t, src):
        r = self.local.rank
        if r == src:
            for d in range(self.world):
                if d != src:
                    self.bcast[d].put(t.clone())
        else:
            got = self.bcast[r].get(timeout=10)
            assert got.shape == t.shape and got.dtype == t.dtype, (got.shape, t.shape)
            t.copy_(got)

    def send(self, t, dst):
        with self.lock:
            self.log.append(("send", self.local.rank, dst, tuple(t.shape)))
        assert t.is_contiguous()
        self.p2p[(self.local.rank, dst)].put(t.clone())

    def irecv(self, t, src):
        me = self.local.rank
        with self.lock:
            self.log.append(("irecv", me, src, tuple(t.shape)))

        class Req:
            def wait(_):
                got = self.p2p[(src, me)].get(timeout=10)
                assert got.shape == t.shape and got.dtype == t.dtype, (got.shape, t.shape)
                t.copy_(got)
        return Req()

    def run(self, fn):
        out, errs = [None] * self.world, []

        def body(r):
            self.local.rank = r
            try:
                out[r] = fn(r)
            except Exception as e:   # noqa: BLE001 - re-raised in the main thread
                errs.append(e)
        th = [threading.Thread(target=body, args=(r,)) for r in range(self.world)]
        for t in th:
            t.start()
        for t in th:
            t.join(30)
        if errs:
            raise errs[0]
        return out


@pytest.fixture
def fake(monkeypatch):
    def make(world):
        f = FakeNccl(world)
        monkeypatch.setattr(D, "dist", f)
        monkeypatch.setattr(D, "_on_device", lambda t: True)
        return f
    return make


def results_for(n):
    """A RayResult array whose rows identify their ray: id = ray, t bits = 7 * ray."""
    r = torch.zeros((n, 4), dtype=torch.int32)
    r[:, 0] = torch.arange(n, dtype=torch.int32)
    r[:, 1] = 7 * torch.arange(n, dtype=torch.int32)
    r[:, 2:] = -5   # pads never travel
    return r


@pytest.mark.parametrize("world,block", [(2, 0), (3, 0), (8, 0), (2, 1000), (3, 4096), (8, 16384), (8, 1)])
def test_gather_results_nccl_branch(fake, world, block):
    n = 100_003
    full_ref = results_for(n)
    f = fake(world)

    def rank_fn(r):
        idx = D.spans_index(D.shard_spans(n, world, r, block))
        return D.gather_results(full_ref[idx].contiguous(), n, dst=0, block=block)
    out = f.run(rank_fn)
    assert all(o is None for o in out[1:])
    assert torch.equal(out[0], full_ref[:, :2])
    # the root receives one message per peer with a non-empty shard, sized to that shard, 8 B per ray
    recvs = [e for e in f.log if e[0] == "irecv"]
    assert sorted(e[2] for e in recvs) == [r for r in range(1, world) if D.shard_spans(n, world, r, block)]
    for _, _, src, shape in recvs:
        assert shape == (sum(b - a for a, b in D.shard_spans(n, world, src, block)), 2)


def test_gather_results_rejects_bad_input(fake):
    f = fake(2)
    n = 1000

    def wrong_size(r):
        return D.gather_results(results_for(10), n, block=0)
    with pytest.raises(ValueError, match="holds 10 results"):
        f.run(wrong_size)
    f = fake(1)
    with pytest.raises(TypeError, match="int32"):
        f.run(lambda r: D.gather_results(results_for(n).float(), n))
    with pytest.raises(TypeError, match="int32"):
        f.run(lambda r: D.gather_results(results_for(n)[:, 0].contiguous(), n))


def test_gather_results_rejects_host_tensors_under_nccl(monkeypatch):
    f = FakeNccl(1)
    monkeypatch.setattr(D, "dist", f)   # the real device check: a CPU tensor is refused under RCCL
    with pytest.raises(ValueError, match="device tensors"):
        f.run(lambda r: D.gather_results(results_for(10), 10))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_replicate_buffers_nccl_branch(fake, world):
    rng = np.random.default_rng(world)
    bufs = [rng.integers(-2**31, 2**31 - 1, size=s, dtype=np.int32) for s in (64, 1000, 17)]
    f = fake(world)
    out = f.run(lambda r: D.replicate_buffers(bufs if r == 0 else None, src=0, device="cpu"))
    for r in range(world):
        assert len(out[r]) == 3
        for got, want in zip(out[r], bufs):
            assert got.dtype == torch.int32 and np.array_equal(got.numpy(), want)


def test_replicate_buffers_rejects_non_int32(fake):
    f = fake(1)
    with pytest.raises(TypeError, match="int32"):
        f.run(lambda r: D.replicate_buffers([np.zeros(4, np.float32)], src=0, device="cpu"))
    with pytest.raises(ValueError, match="1-D"):
        f.run(lambda r: D.replicate_buffers([np.zeros((2, 2), np.int32)], src=0, device="cpu"))


@pytest.mark.parametrize("world,block", [(2, 0), (8, 0), (3, 777), (8, 16384)])
def test_shard_layout_covers_every_ray_once(world, block):
    """The strong-scaling shards (bench.py strong_scaling): every ray in exactly one
    shard, each shard's launches cover it in order within the 2^21-ray batch limit."""
    n = 16_588_800 // 64
    seen = torch.zeros(n, dtype=torch.int32)
    for r in range(world):
        spans = D.shard_spans(n, world, r, block)
        idx = D.spans_index(spans)
        seen[idx] += 1
        k = int(idx.numel())
        launches = D.shard_launches(0, k, 1 << 16)
        assert launches[0][0] == 0 and launches[-1][1] == k
        assert all(b - a <= 1 << 16 for a, b in launches)
        assert all(launches[i][1] == launches[i + 1][0] for i in range(len(launches) - 1))
    assert bool((seen == 1).all())


def test_balance_blocks_deals_equal_counts_and_live_rays():
    """balance_blocks: every block owned once; the ranks get the same number of blocks
    (±1) and live rays within one block's weight; the same weights give the same deal."""
    rng = np.random.default_rng(3)
    for nblocks, world in ((1013, 8), (1013, 3), (7, 8), (64, 1), (0, 4)):
        w = rng.integers(0, 16385, size=nblocks)
        w[: nblocks // 4] = 0                       # dead blocks (sky) in one region
        owners = D.balance_blocks(torch.from_numpy(w), world)
        assert owners.shape == (nblocks,) and np.array_equal(owners, D.balance_blocks(w, world))
        counts = np.bincount(owners, minlength=world)
        loads = np.bincount(owners, weights=w, minlength=world)
        if nblocks:
            assert counts.max() - counts.min() <= 1
            assert loads.max() - loads.min() <= w.max()


def test_block_weights_count_live_rays():
    rays = torch.zeros((10, 8))
    rays[:, 7] = torch.tensor([1.0, -1.0, 0.0, 5.0, -1.0, -1.0, 2.0, 3.0, -1.0, 1.0])
    assert D.block_weights(rays, 4).tolist() == [3, 2, 1]
    with pytest.raises(ValueError):
        D.block_weights(rays, 0)


@pytest.mark.parametrize("world,block", [(2, 1000), (8, 4096), (3, 777)])
def test_gather_results_with_a_weighted_deal(fake, world, block):
    """Shards dealt by balance_blocks gather back into ray order (nccl branch)."""
    n = 100_003
    full_ref = results_for(n)
    nblocks = -(-n // block)
    owners = D.balance_blocks(np.random.default_rng(world).integers(0, block, nblocks), world)
    seen = torch.zeros(n, dtype=torch.int32)
    for r in range(world):
        seen[D.spans_index(D.shard_spans(n, world, r, block, owners))] += 1
    assert bool((seen == 1).all())
    f = fake(world)

    def rank_fn(r):
        idx = D.spans_index(D.shard_spans(n, world, r, block, owners))
        return D.gather_results(full_ref[idx].contiguous(), n, dst=0, block=block, owners=owners)
    out = f.run(rank_fn)
    assert torch.equal(out[0], full_ref[:, :2])
    with pytest.raises(ValueError, match="block owners"):
        D.shard_spans(n, world, 0, block, owners[:-1])


@pytest.mark.parametrize("world,block,balanced", [(1, 1000, False), (2, 1000, False), (8, 4096, True), (3, 777, False)])
def test_priority_orders_blocks_and_gathers_back(fake, world, block, balanced):
    """shard_spans(..., priority=w): each rank's blocks in decreasing w (ties in
    frame order), every ray still in exactly one shard, and gather_results puts
    the results back in ray order (nccl branch)."""
    n = 100_003
    nblocks = -(-n // block)
    rng = np.random.default_rng(block)
    w = rng.integers(0, 5, nblocks)
    owners = D.balance_blocks(w, world) if balanced else None
    seen = torch.zeros(n, dtype=torch.int32)
    for r in range(world):
        spans = D.shard_spans(n, world, r, block, owners, w)
        firsts = [a // block for a, _ in spans if a // block != nblocks - 1]   # the partial last block comes last
        assert all(w[x] >= w[y] for x, y in zip(firsts, firsts[1:]))
        if any(a // block == nblocks - 1 for a, _ in spans):
            assert spans[-1][1] == n
        seen[D.spans_index(spans)] += 1
    assert bool((seen == 1).all())
    full_ref = results_for(n)
    f = fake(world)

    def rank_fn(r):
        idx = D.spans_index(D.shard_spans(n, world, r, block, owners, w))
        return D.gather_results(full_ref[idx].contiguous(), n, dst=0, block=block, owners=owners, priority=w)
    out = f.run(rank_fn)
    assert torch.equal(out[0], full_ref[:, :2])
    with pytest.raises(ValueError, match="block priorities"):
        D.shard_spans(n, world, 0, block, owners, w[:-1])
