"""Multi-GPU ray sharding: the Compact2 BVH is replicated on
every rank, the RayBuffer is split into contiguous shards, every rank traces
its shard with its own persistent grid, and hit results are gathered to the
root only when the caller needs them in one place.

One process per GPU over torch.distributed ("nccl" = RCCL on ROCm; "gloo"
for the CPU tests). The trace itself needs no collective.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n rays for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def replicate_buffers(bufs, src: int = 0, device=None):
    """Broadcast int32 buffers (e.g. Compact2 nodes/woop/triIndex) from rank `src`;
    other ranks pass None. Returns tensors on `device` on every rank: with RCCL
    they stay in HBM (the BVH crosses xGMI once and is bound in place, GpuBvh
    accepts them without a copy); with gloo they are CPU tensors."""
    rank = dist.get_rank()
    dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                             if dist.get_backend() == "nccl" else torch.device("cpu"))
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
        dist.broadcast(t, src)
        out.append(t)
    return out


def shard_launches(lo: int, hi: int, max_rays: int):
    """The shard [lo, hi) cut into launches of at most max_rays rays (the reference
    traces at most 2^21 rays per launch, Renderer.cc:46)."""
    return [(a, min(hi, a + max_rays)) for a in range(lo, hi, max_rays)]


def trace_shard(tracer, rays, world: int, rank: int, max_rays: int = 1 << 21, exact_rcp: bool = True,
                stream=None):
    """Strong-scaling step of one rank: trace its contiguous shard of the RayBuffer
    `rays` (every rank holds the same buffer) in launches of at most max_rays rays,
    stream-ordered, results written in place. Returns the shard's (lo, hi)."""
    lo, hi = shard_range(rays.size, world, rank)
    for a, b in shard_launches(lo, hi, max_rays):
        tracer.trace_async(rays.view(a, b), exact_rcp=exact_rcp, stream=stream)
    return lo, hi


def gather_results(local: torch.Tensor, n_total: int, dst: int = 0):
    """Gather every rank's RayResult shard (int32 [k, 4]) to rank `dst` in ray
    order with point-to-point send/recv (RCCL has no gather primitive; the root
    receives from all peers at once over their direct xGMI links). Only the
    8 useful bytes per ray (id, t) travel. Returns the full array on `dst`,
    None elsewhere."""
    world, rank = dist.get_world_size(), dist.get_rank()
    payload = local[:, :2].contiguous()
    if rank != dst:
        if payload.shape[0] > 0:
            dist.send(payload, dst)
        return None
    full = torch.empty((n_total, 2), dtype=torch.int32, device=local.device)
    reqs = []
    for r in range(world):
        lo, hi = shard_range(n_total, world, r)
        if r == dst:
            full[lo:hi].copy_(payload)
        elif hi > lo:
            reqs.append(dist.irecv(full[lo:hi], r))
    for q in reqs:
        q.wait()
    return full
