"""Multi-GPU ray sharding: the Compact2 BVH is replicated on
every rank, the RayBuffer is split into shards (contiguous ranges, or
block-cyclic blocks so that every shard samples the whole frame), every rank
traces its shard with its own persistent grid, and hit results are gathered to
the root only when the caller needs them in one place. Blocks can be dealt by
live-ray weight (balance_blocks) instead of cyclically.

One process per GPU over torch.distributed ("nccl" = RCCL on ROCm; "gloo"
for the CPU tests). The trace itself needs no collective.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def _on_device(t: torch.Tensor) -> bool:
    """RCCL moves HBM-resident tensors only (tests/test_dist_mock.py replaces this
    check to dry-run the nccl branches on the CPU)."""
    return t.device.type == "cuda"


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n rays for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def block_weights(rays: torch.Tensor, block: int) -> torch.Tensor:
    """Live rays per block-ray block of a RayBuffer (float32 [n, 8]): rays whose
    tmax is not negative. The AO/diffuse generators give the samples of a pixel
    whose primary ray missed tmax = -1 (RayGenKernels.cu:117-227); the trace
    retires such a ray at once, so a block's cost follows its live rays. One
    reduction over the tmax column, on the buffer's device."""
    if block <= 0:
        raise ValueError("block_weights: block must be positive")
    n = rays.shape[0]
    live = (rays[:, 7] >= 0).to(torch.int64)
    pad = (-n) % block
    if pad:
        live = torch.cat([live, live.new_zeros(pad)])
    return live.view(-1, block).sum(1)


def block_sums(values: torch.Tensor, block: int) -> torch.Tensor:
    """Per-block sums of a per-ray value (e.g. a traced frame's node + triangle counts,
    the STATS counters): the traversal cost of each block-ray block, a finer priority
    for shard_spans than block_weights' live-ray count."""
    if block <= 0:
        raise ValueError("block_sums: block must be positive")
    v = values.to(torch.int64).reshape(-1)
    pad = (-v.numel()) % block
    if pad:
        v = torch.cat([v, v.new_zeros(pad)])
    return v.view(-1, block).sum(1)


def balance_blocks(weights, world: int) -> np.ndarray:
    """Owner rank of every block (int32 [nblocks]): the blocks in decreasing weight
    (ties: lower index first) dealt in serpentine order — ranks 0..world-1, then
    world-1..0, and so on. Every rank gets the same number of blocks (±1), so the
    shards hold the same number of rays, and the live rays balance to within one
    block's weight (a pure weight-greedy deal hands all the dead blocks to one
    rank: retiring 10 M dead rays took 1.9 ms on one MI355X). Deterministic, so
    every rank computes the same owners from the same weights. Used with
    shard_spans(..., owners=...): each rank keeps its blocks in frame order."""
    w = np.asarray(weights.cpu() if isinstance(weights, torch.Tensor) else weights, dtype=np.int64)
    if w.ndim != 1 or world < 1:
        raise ValueError("balance_blocks: 1-D weights and world >= 1 expected")
    order = np.argsort(-w, kind="stable")
    j = np.arange(len(w))
    pos, rnd = j % world, j // world
    owners = np.empty(len(w), dtype=np.int32)
    owners[order] = np.where(rnd % 2 == 0, pos, world - 1 - pos)
    return owners


def shard_blocks(n: int, world: int, rank: int, block: int, owners=None, priority=None) -> np.ndarray:
    """The block ids (int64) of `rank`'s block-cyclic shard of n rays in trace order:
    block i to rank i % world (or owners[i]), in frame order or, with priority (one value
    >= 0 per block, e.g. block_weights), in decreasing priority (ties in frame order). The
    frame's last block, when partial (n % block != 0), always comes last, so a shard's
    rays are whole blocks followed by at most one short one (what mrt_raygen_ao_blocks
    generates)."""
    if block <= 0:
        raise ValueError("shard_blocks: block must be positive")
    nblocks = -(-n // block)
    if owners is not None:
        owners = np.asarray(owners)
        if len(owners) != nblocks:
            raise ValueError(f"shard_spans: {len(owners)} block owners for {nblocks} blocks of {block} rays")
        mine = np.flatnonzero(owners == rank)
    else:
        mine = np.arange(rank, nblocks, world)
    if priority is not None and len(mine):
        pr = np.asarray(priority.cpu() if isinstance(priority, torch.Tensor) else priority)
        if len(pr) != nblocks:
            raise ValueError(f"shard_spans: {len(pr)} block priorities for {nblocks} blocks of {block} rays")
        key = -np.asarray(pr[mine], dtype=np.float64)
        if n % block:
            key[mine == nblocks - 1] = np.inf     # the partial block last
        mine = mine[np.argsort(key, kind="stable")]
    return mine.astype(np.int64)


def shard_blocks_device(n: int, world: int, rank: int, block: int, owners=None, priority=None, device=None):
    """shard_blocks on the device, without a host sync: (int32 block ids on `device`, the
    number of rays they hold). priority: a device tensor (e.g. live_block_weights); the
    order is shard_blocks' (a stable sort of the same keys), so gather_results /
    shard_spans with the same priority on the host put the results back."""
    nblocks = -(-n // block)
    if owners is not None:
        mine_h = np.flatnonzero(np.asarray(owners) == rank)
    else:
        mine_h = np.arange(rank, nblocks, world)
    partial = n % block
    last_mine = len(mine_h) > 0 and int(mine_h[-1]) == nblocks - 1
    num_rays = len(mine_h) * block - ((block - partial) if partial and last_mine else 0)
    mine = (torch.from_numpy(mine_h).to(device) if owners is not None
            else torch.arange(rank, nblocks, world, dtype=torch.int64, device=device))
    if priority is not None and len(mine_h):
        if priority.numel() != nblocks:
            raise ValueError(f"shard_blocks_device: {priority.numel()} block priorities for {nblocks} blocks")
        key = -priority.to(device)[mine].to(torch.float64)
        if partial and last_mine:
            key = torch.where(mine == nblocks - 1, torch.full_like(key, float("inf")), key)
        mine = mine[torch.argsort(key, stable=True)]
    return mine.to(torch.int32), int(num_rays)


def live_block_weights(primary_results: torch.Tensor, num_samples: int, block: int) -> torch.Tensor:
    """block_weights of a frame's AO/diffuse rays known before they exist: a secondary ray
    is live (tmax >= 0) exactly when its primary ray hit (RayGenKernels.cu:117-227), so the
    live rays per block-ray block of the frame's ray order (input p's samples at p*S..)
    follow from the primary pass's results (RayResult int32 [n, 4]) — one reduction on
    their device, int64 [ceil(n*S / block)]."""
    if block <= 0 or num_samples < 1:
        raise ValueError("live_block_weights: block and num_samples must be positive")
    hit = (primary_results[:, 0] >= 0).to(torch.int64)
    total = hit.numel() * num_samples
    nblocks = -(-total // block)
    if block % num_samples == 0:
        per = block // num_samples
        pad = nblocks * per - hit.numel()
        if pad:
            hit = torch.cat([hit, hit.new_zeros(pad)])
        return hit.view(-1, per).sum(1) * num_samples
    live = hit.repeat_interleave(num_samples)
    pad = nblocks * block - total
    if pad:
        live = torch.cat([live, live.new_zeros(pad)])
    return live.view(-1, block).sum(1)


KEY_MAX = 4094   # mrt_shard_blocks' live-order keys: 12 bits (4095 = the partial last block)


def live_priority(weights, block: int) -> np.ndarray:
    """The host priority (for shard_blocks / shard_spans / gather_results) whose order is
    mrt_shard_blocks' live-first order: decreasing live count, quantized to mrt_shard_blocks'
    12-bit key when block > 4094 (key = ceil((block - live) * 4094 / block))."""
    w = np.asarray(weights.cpu() if isinstance(weights, torch.Tensor) else weights, dtype=np.int64)
    key = block - w
    if block > KEY_MAX:
        key = (key * KEY_MAX + block - 1) // block
    return -key


def shard_spans(n: int, world: int, rank: int, block: int = 0, owners=None, priority=None) -> list[tuple[int, int]]:
    """The ray ranges of `rank`'s shard of n rays. block = 0: one contiguous range
    (shard_range). block > 0: block-cyclic — the buffer cut into block-ray blocks,
    block i to rank i % world — so every shard draws from the whole frame. A
    frame's RayBuffer is in pixel order (AO/diffuse samples of a pixel adjacent,
    RayGenKernels.cu:117-227), so contiguous shards are image regions of unequal
    cost: on the hairball 1920x1080x8spp buffer the 8 contiguous shards took
    0.59-1.12 ms on one MI355X, which caps eta(8) at 0.54. owners (block > 0):
    block i to rank owners[i] instead (balance_blocks). priority (block > 0, one
    value per block, e.g. block_weights): the rank's blocks in decreasing priority
    (ties in frame order, a partial last block last: shard_blocks) instead of frame
    order, so a launch that deals its rays in order starts its costly blocks first
    and ends on the cheap ones (with world = 1: the whole buffer reordered). Blocks
    adjacent in the result are merged."""
    if block <= 0 or (world == 1 and priority is None):
        lo, hi = shard_range(n, world, rank)
        return [(lo, hi)] if hi > lo else []
    mine = shard_blocks(n, world, rank, block, owners, priority)
    if len(mine) == 0:
        return []
    # the blocks' ranges, adjacent ones merged (vectorised: a 16.6 M-ray buffer has 16 k blocks)
    starts = mine * block
    ends = np.minimum(n, starts + block)
    first = np.ones(len(mine), bool)
    first[1:] = starts[1:] != ends[:-1]
    heads = np.flatnonzero(first)
    last = np.append(heads[1:] - 1, len(mine) - 1)
    return list(zip(starts[heads].tolist(), ends[last].tolist()))


def spans_index(spans, device=None) -> torch.Tensor:
    """int64 ray indices of a list of ranges, in order (a handful of kernels
    whatever the number of ranges: a block-cyclic shard has hundreds)."""
    if not spans:
        return torch.empty(0, dtype=torch.int64, device=device)
    starts = torch.tensor([a for a, _ in spans], dtype=torch.int64, device=device)
    lens = torch.tensor([b - a for a, b in spans], dtype=torch.int64, device=device)
    first = torch.cumsum(lens, 0) - lens                    # position of each range's first index
    total = int(sum(b - a for a, b in spans))
    pos = torch.arange(total, dtype=torch.int64, device=device)
    return torch.repeat_interleave(starts - first, lens, output_size=total) + pos


def local_rays(rays: torch.Tensor, spans) -> torch.Tensor:
    """The shard's rays (float32 [k, 8]) as one contiguous array (a view when the
    shard is one range), so the rank traces it like any RayBuffer."""
    if len(spans) == 1:
        a, b = spans[0]
        return rays[a:b]
    return torch.index_select(rays, 0, spans_index(spans, rays.device))


def replicate_buffers(bufs, src: int = 0, device=None):
    """Broadcast int32 buffers (e.g. Compact2 nodes/woop/triIndex) from rank `src`;
    other ranks pass None. Returns tensors on `device` on every rank: with RCCL
    they stay in HBM (the BVH crosses xGMI once and is bound in place, GpuBvh
    accepts them without a copy); with gloo they are CPU tensors."""
    rank = dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                             if nccl else torch.device("cpu"))
    dev = torch.device(dev)
    if nccl and not _on_device(torch.empty(0, device=dev)):
        raise ValueError("replicate_buffers: RCCL (nccl) broadcasts device tensors; got device " + str(dev))
    if rank == src:
        if bufs is None or len(bufs) == 0:
            raise ValueError("replicate_buffers: the source rank must pass the buffers")
        for b in bufs:
            dt = b.dtype if isinstance(b, torch.Tensor) else np.asarray(b).dtype
            if dt not in (torch.int32, np.int32, np.dtype(np.int32)):
                raise TypeError(f"replicate_buffers: int32 buffers expected (Compact2 words), got {dt}")
            if (b.dim() if isinstance(b, torch.Tensor) else np.ndim(b)) != 1:
                raise ValueError("replicate_buffers: flat 1-D buffers expected")
    count = len(bufs) if rank == src else 0
    meta = torch.tensor([count], dtype=torch.int64, device=dev)
    dist.broadcast(meta, src)
    count = int(meta.item())
    sizes = torch.tensor([len(b) for b in bufs] if rank == src else [0] * count, dtype=torch.int64, device=dev)
    dist.broadcast(sizes, src)
    out = []
    for i in range(count):
        if rank == src:
            b = bufs[i]
            t = (b.to(dev, torch.int32) if isinstance(b, torch.Tensor)
                 else torch.from_numpy(np.ascontiguousarray(b, np.int32)).to(dev))
        else:
            t = torch.empty(int(sizes[i]), dtype=torch.int32, device=dev)
        if t.numel() != int(sizes[i]) or t.device != dev:
            raise RuntimeError("replicate_buffers: buffer shape/device changed before the broadcast")
        dist.broadcast(t, src)
        out.append(t)
    return out


def shard_launches(lo: int, hi: int, max_rays: int, min_launches: int = 1):
    """The shard [lo, hi) cut into launches of at most max_rays rays (the reference
    traces at most 2^21 rays per launch, Renderer.cc:46). With min_launches > 1 a
    shard is cut into at least that many launches; the cuts are balanced (sizes
    differ by at most one ray)."""
    n = hi - lo
    if n <= 0:
        return []
    k = max(min_launches, -(-n // max_rays))
    return [(lo + a, lo + b) for a, b in (shard_range(n, k, i) for i in range(k)) if b > a]


def trace_shard(tracer, rays, world: int, rank: int, max_rays: int = 1 << 21, exact_rcp: bool = True,
                stream=None, block: int = 0, owners=None, priority=None):
    """Strong-scaling step of one rank: trace its shard of the RayBuffer `rays`
    (every rank holds the same buffer) in launches of at most max_rays rays,
    stream-ordered. block = 0: the contiguous shard, results written in place;
    returns (lo, hi). block > 0: the block-cyclic shard, gathered into a local
    RayBuffer first; returns that buffer (its results are the shard's, in
    shard_spans order — what gather_results(..., block=block, owners=owners)
    expects). owners: balance_blocks' deal of the blocks, or None (cyclic);
    priority: the order of the blocks within the shard (shard_spans)."""
    if block <= 0 or (world == 1 and priority is None):
        lo, hi = shard_range(rays.size, world, rank)
        for a, b in shard_launches(lo, hi, max_rays):
            tracer.trace_async(rays.view(a, b), exact_rcp=exact_rcp, stream=stream)
        return lo, hi
    from .tracer import RayBuffer
    local = RayBuffer(local_rays(rays.rays, shard_spans(rays.size, world, rank, block, owners, priority)),
                      rays.need_closest_hit, secondary=getattr(rays, "secondary", False))
    if stream is not None:
        # the local buffer was built on the current stream: the launches on `stream` wait for it
        stream.wait_stream(torch.cuda.current_stream())
    for a, b in shard_launches(0, local.size, max_rays):
        tracer.trace_async(local.view(a, b), exact_rcp=exact_rcp, stream=stream)
    return local


def gather_results(local: torch.Tensor, n_total: int, dst: int = 0, block: int = 0, owners=None, priority=None):
    """Gather every rank's RayResult shard (int32 [k, 4], the shard's rays in
    shard_spans order) to rank `dst` in ray order with point-to-point send/recv
    (RCCL has no gather primitive; the root receives from all peers at once over
    their direct xGMI links). Only the 8 useful bytes per ray (id, t) travel; a
    block-cyclic shard arrives as one message and is scattered into place with
    one index_copy_. Returns the full array on `dst`, None elsewhere."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if local.dtype != torch.int32 or local.dim() != 2 or local.shape[1] < 2:
        raise TypeError(f"gather_results: RayResult rows (int32 [k, >=2]) expected, got {local.dtype} "
                        f"{tuple(local.shape)}")
    if dist.get_backend() == "nccl" and not _on_device(local):
        raise ValueError("gather_results: RCCL (nccl) moves device tensors; got a " + local.device.type + " tensor")
    mine = sum(b - a for a, b in shard_spans(n_total, world, rank, block, owners, priority))
    if local.shape[0] != mine:
        raise ValueError(f"gather_results: rank {rank} holds {local.shape[0]} results, its shard of {n_total} "
                         f"rays has {mine}")
    payload = local[:, :2].contiguous()
    if rank != dst:
        if payload.shape[0] > 0:
            dist.send(payload, dst)
        return None
    full = torch.empty((n_total, 2), dtype=torch.int32, device=local.device)
    reqs, scatter = [], []
    for r in range(world):
        spans = shard_spans(n_total, world, r, block, owners, priority)
        count = sum(b - a for a, b in spans)
        if count == 0:
            continue
        if len(spans) == 1:
            lo, hi = spans[0]
            if r == dst:
                full[lo:hi].copy_(payload)
            else:
                reqs.append(dist.irecv(full[lo:hi], r))
        else:
            buf = payload if r == dst else torch.empty((count, 2), dtype=torch.int32, device=local.device)
            if r != dst:
                reqs.append(dist.irecv(buf, r))
            scatter.append((spans_index(spans, local.device), buf))
    for q in reqs:
        q.wait()
    for idx, buf in scatter:
        full.index_copy_(0, idx, buf)
    return full
