"""Frame orchestration on one device: the reference Renderer (src/rt/cuda/Renderer.cc:44-300)
and RayGen's batching (src/rt/ray/RayGen.cc:77-142) over the C-ABI.

  beginFrame      Renderer.cc:112-152   primary rays (Morton order) in one RayBuffer; for AO /
                                        diffuse frames they are traced first (untimed pre-pass)
  getTotalNumRays Renderer.cc:221-238   w*h for primary; primary hits * samples otherwise
  nextBatch       Renderer.cc:242-291   the next <= maxBatchSize rays (RayGen::batching,
                                        RayGen.cc:124-142): primaries [lo, hi) with
                                        hi = min(n, lo + maxBatch / numSamples), numSamples rays each,
                                        seeded by the next glibc rand() (RayGen.cc:106)
  traceBatch      Renderer.cc:295-300   CudaTracer::traceBatch of the current batch -> ms
  updateResult    Renderer.cc:421-445   reconstructKernel of the batch into the frame's pixels

The reference draws every AO/diffuse batch seed from the C library's rand()
(RayGen.cc:106; App never seeds it, so the sequence starts at glibc's
1804289383); GlibcRand restates glibc's TYPE_3 generator so batch k of a frame
gets the same seed here. Batches above 2^21 rays never exist: a frame of any
size and sample count is traced as several launches, like the reference.
"""
from __future__ import annotations

import torch

from . import _lib
from .host import Camera, Scene
from .raygen import RAY_AO, RAY_DIFFUSE, RAY_PRIMARY, DeviceRayGen, DeviceReconstructor
from .tracer import RayBuffer, Tracer

MAX_BATCH_RAYS = 1 << 21   # Renderer.cc:46 m_raygen(1 << 21)


class GlibcRand:
    """glibc rand() (random_r TYPE_3: additive feedback r[i] = r[i-31] + r[i-3] over a
    table seeded by 16807 * r mod (2^31 - 1), first 310 outputs discarded, >> 1)."""

    def __init__(self, seed: int = 1):
        r = [seed & 0xFFFFFFFF]
        for i in range(1, 31):
            prev = r[-1] - (1 << 32) if r[-1] >= (1 << 31) else r[-1]
            hi, lo = divmod(prev, 127773) if prev >= 0 else (-((-prev) // 127773), -((-prev) % 127773))
            word = 16807 * lo - 2836 * hi
            r.append(word + 2147483647 if word < 0 else word)
        r += r[:3]
        for _ in range(310):
            r.append((r[-31] + r[-3]) & 0xFFFFFFFF)
        self._r = r[-34:]

    def __call__(self) -> int:
        v = (self._r[-31] + self._r[-3]) & 0xFFFFFFFF
        self._r = self._r[1:] + [v]
        return v >> 1


def batching(num_input: int, num_samples: int, start: int, max_batch: int = MAX_BATCH_RAYS):
    """RayGen::batching (RayGen.cc:124-142): the next input range [lo, hi) from `start`,
    or None when every input ray is done."""
    if num_samples < 1 or max_batch < num_samples:
        raise _lib.MrtError(f"batching: {num_samples} samples do not fit a {max_batch}-ray batch")
    if start >= num_input:
        return None
    lo = start
    return lo, min(num_input, lo + max_batch // num_samples)


class Renderer:
    """Renderer.cc on one device: one frame = a primary RayBuffer plus, for AO and
    diffuse, a sequence of <= max_batch-ray secondary batches."""

    def __init__(self, tracer: Tracer, scene: Scene, max_batch: int = MAX_BATCH_RAYS, exact_rcp: bool = True,
                 rand: GlibcRand | None = None):
        self.tracer = tracer
        self.scene = scene
        self.max_batch = int(max_batch)
        self.exact_rcp = exact_rcp
        self.rand = rand if rand is not None else GlibcRand()
        self.gen = DeviceRayGen(scene)
        self._recon = None
        self.ray_type, self.num_samples, self.ao_radius = RAY_PRIMARY, 1, 5.0
        self.primary: RayBuffer | None = None
        self.slot_to_id: torch.Tensor | None = None
        self.batch: RayBuffer | None = None
        self.batch_start = 0      # first ray of the current batch in the frame's secondary-ray sequence
        self._next_input = 0      # RayGen's m_aoStartIdx
        self._new_batch = True
        self._seeds: list[int] = []   # this frame's batch seeds, drawn from rand() in batch order

    def set_params(self, ray_type: int = RAY_PRIMARY, num_samples: int = 1, ao_radius: float = 5.0) -> None:
        if ray_type not in (RAY_PRIMARY, RAY_AO, RAY_DIFFUSE):
            raise _lib.MrtError(f"unknown ray type {ray_type}")
        self.ray_type, self.num_samples, self.ao_radius = ray_type, int(num_samples), float(ao_radius)

    def begin_frame(self, cam: Camera, w: int, h: int, subpixel=(0.5, 0.5)) -> None:
        self.cam, self.w, self.h = cam, w, h
        self.primary, self.slot_to_id = self.gen.primary(cam, w, h, subpixel=subpixel)
        if self.ray_type != RAY_PRIMARY:
            self.tracer.trace_batch(self.primary, exact_rcp=self.exact_rcp)
        self.batch, self.batch_start, self._next_input, self._new_batch = None, 0, 0, True
        self._seeds = []

    def total_num_rays(self) -> int:
        if self.ray_type == RAY_PRIMARY:
            return self.primary.size
        return self.gen.count_hits(self.primary) * self.num_samples

    def next_batch(self) -> bool:
        if self.batch is not None:
            self.batch_start += self.batch.size
        self.batch = None
        if self.ray_type == RAY_PRIMARY:
            if not self._new_batch:
                return False
            self._new_batch = False
            self.batch = self.primary
            return True
        rng = batching(self.primary.size, self.num_samples, self._next_input, self.max_batch)
        if rng is None:
            return False
        lo, hi = rng
        self._next_input = hi
        self.batch = self.gen.ao(self.primary, self.num_samples, self._max_dist(),
                                 seed=self.batch_seeds(lo // self._batch_inputs() + 1)[-1],
                                 closest_hit=self.ray_type == RAY_DIFFUSE, first=lo, count=hi - lo)
        return True

    def _max_dist(self) -> float:
        return self.ao_radius if self.ray_type == RAY_AO else self.cam.far

    def _batch_inputs(self) -> int:
        return self.max_batch // self.num_samples      # RayGen::batching's primaries per batch

    def num_batches(self) -> int:
        """Secondary batches of the frame (RayGen::batching, RayGen.cc:124-142)."""
        return -(-self.primary.size // self._batch_inputs()) if self.ray_type != RAY_PRIMARY else 1

    def batch_seeds(self, count: int | None = None) -> list[int]:
        """The seeds of the frame's first `count` (default: all) secondary batches: one
        rand() per batch in batch order (RayGen.cc:106), drawn once per frame and shared by
        next_batch and secondary_blocks, so both see the same sequence."""
        count = self.num_batches() if count is None else count
        while len(self._seeds) < count:
            self._seeds.append(self.rand())
        return self._seeds[:count]

    def secondary_blocks(self, blocks: torch.Tensor, num_rays: int, block_rays: int, stream=None) -> RayBuffer:
        """The frame's AO/diffuse rays at a list of block_rays-ray blocks of its ray order
        (the order next_batch's batches hold them in), generated directly in list order on the
        device (mrt_raygen_ao_blocks) — a rank's shard of the frame, or the whole frame with
        its costly blocks first, with no frame-order buffer and no gather. Bit-identical to
        the same positions of the batches. num_rays: the rays listed (mrt.dist.shard_blocks_device)."""
        if self.ray_type == RAY_PRIMARY or self.primary is None:
            raise _lib.MrtError("secondary_blocks needs an AO or diffuse frame (set_params, begin_frame)")
        return self.gen.ao_blocks(self.primary, self.num_samples, self._max_dist(), self.batch_seeds(),
                                  self._batch_inputs(), blocks, block_rays, num_rays,
                                  closest_hit=self.ray_type == RAY_DIFFUSE, stream=stream)

    def shard(self, world: int, rank: int, block_rays: int, order: int = 1, stream=None) -> RayBuffer:
        """Rank's shard of the frame's AO/diffuse rays for a world-rank job, generated in its
        trace order on the device: block i of block_rays rays to rank i % world, live blocks
        first (order 1) or in frame order (0) — mrt_shard_blocks, then secondary_blocks. Two
        ranks' shards hold disjoint rays; together, the frame (mrt.dist.gather_results with
        block=block_rays and priority=mrt.dist.live_priority(...) puts results back)."""
        if self.ray_type == RAY_PRIMARY or self.primary is None:
            raise _lib.MrtError("shard needs an AO or diffuse frame (set_params, begin_frame)")
        blocks, n = self.gen.shard_blocks(self.primary, self.num_samples, block_rays, world, rank, order, stream)
        return self.secondary_blocks(blocks, n, block_rays, stream)

    def trace_batch(self) -> float:
        if self.batch is None:
            raise _lib.MrtError("Renderer.trace_batch without a batch (call next_batch)")
        return self.tracer.trace_batch(self.batch, exact_rcp=self.exact_rcp)

    def update_result(self, pixels: torch.Tensor | None = None) -> torch.Tensor:
        """reconstructKernel of the current batch into `pixels` (w*h ABGR int32)."""
        if self._recon is None:
            self._recon = DeviceReconstructor(self.scene)
        n = 1 if self.ray_type == RAY_PRIMARY else self.num_samples
        return self._recon.reconstruct(self.ray_type, self.primary, self.slot_to_id, self.w * self.h, self.batch,
                                       num_samples=n, pixels=pixels, first_primary=self.batch_start // n)

    def batches(self):
        """Every batch of the frame (generated, not traced) as (RayBuffer, first ray) pairs."""
        out = []
        while self.next_batch():
            out.append((self.batch, self.batch_start))
        return out
