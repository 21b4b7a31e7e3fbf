"""World-size-2 rehearsal of the multi-GPU path on CPU with gloo: the BVH is
replicated from rank 0, rays are sharded contiguously, each rank traces its
shard (here with the CPU oracle standing in for the per-GPU tracer), and the
results are gathered to rank 0 in ray order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mrt.dist import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
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
    nodes, woop, tri = replicate_buffers(bufs, src=0, device=torch.device("cpu"))
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 61, 37)          # ragged: 2257 rays, not a multiple of the world size
    lo, hi = shard_range(len(rays), world, rank)
    res, _, _ = O.trace(rays[lo:hi], nodes, woop, tri)
    full = gather_results(torch.from_numpy(res), len(rays), dst=0)
    if rank == 0:
        want, _, _ = O.trace(rays, *mrt.Bvh.build(scene).buffers())
        np.save(out_path, np.stack([full.numpy()[:, 0], want[:, 0], full.numpy()[:, 1], want[:, 1]]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_replicate_shard_gather(tmp_path, world):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    a = np.load(out)
    assert np.array_equal(a[0], a[1]) and np.array_equal(a[2], a[3])


def test_shard_ranges_partition():
    for n in (0, 1, 7, 64, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
