"""Device ray generation and hit counting (mirror of the reference's RayGen,
src/rt/ray/RayGen.cc:50-120, and countHitsKernel, RendererKernels.cu:112-162),
over the mrt_raygen_* / mrt_count_hits entry points of include/mrt.h.

The per-ray arithmetic is the host generator's (mrt.host.primary_rays /
ao_rays): primary rays come out bit-identical, AO/diffuse directions within a
few ulp (device cosf/sinf). Pixel tables and the camera matrix are computed on
the host, as in the reference (PixelTable.cc, Renderer.cc:126-129).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .host import AO_SEED, Camera, Scene, pixel_table
from .tracer import RayBuffer, _stream_ptr


def nscreen_to_world(cam: Camera, w: int, h: int) -> np.ndarray:
    out = (C.c_float * 16)()
    c = cam.to_c()
    _lib.check_host(_lib.host_lib().mrth_camera_nscreen_to_world(C.byref(c), w, h, out))
    return np.array(out, np.float32)


class DeviceRayGen:
    """RayGen on one device: primary rays, AO/diffuse rays, hit counts."""

    def __init__(self, scene: Scene | None = None, device=None):
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.lib = _lib.trace_lib()
        self._tables = {}
        self.normals = None
        self.num_tris = 0
        if scene is not None:
            _, _, normals = scene.arrays()
            self.normals = torch.from_numpy(np.ascontiguousarray(normals, np.float32)).to(self.device)
            self.num_tris = scene.num_triangles

    def _table(self, w: int, h: int) -> torch.Tensor:
        if (w, h) not in self._tables:
            self._tables[(w, h)] = torch.from_numpy(pixel_table(w, h)).to(self.device)
        return self._tables[(w, h)]

    def primary(self, cam: Camera, w: int, h: int, stream=None, subpixel=(0.5, 0.5)) -> tuple[RayBuffer, torch.Tensor]:
        """RayGen::primary: w*h closest-hit rays in Morton pixel order + slot->pixel ids.
        subpixel: sample position inside each pixel (the reference's is the centre)."""
        m = nscreen_to_world(cam, w, h)
        origin = np.array(cam.position, np.float32)
        rays = torch.empty((w * h, 8), dtype=torch.float32, device=self.device)
        slot_to_id = torch.empty(w * h, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.mrt_raygen_primary_subpixel(m.ctypes.data_as(C.POINTER(C.c_float)),
                                                        origin.ctypes.data_as(C.POINTER(C.c_float)), float(cam.far), w,
                                                        h, float(subpixel[0]), float(subpixel[1]),
                                                        self._table(w, h).data_ptr(), rays.data_ptr(),
                                                        slot_to_id.data_ptr(), None, _stream_ptr(stream)))
        return RayBuffer(rays, need_closest_hit=True, device=self.device), slot_to_id

    def ao(self, rays: RayBuffer, num_samples: int, max_dist: float, seed: int = AO_SEED, closest_hit: bool = False,
           stream=None, first: int = 0, count: int | None = None) -> RayBuffer:
        """RayGen::ao over a traced batch: num_samples hemisphere rays per input ray
        (any-hit for AO; closest_hit=True with max_dist=far is the diffuse bounce).
        first/count select the input rays [first, first + count) — one batch of
        RayGen::batching (RayGen.cc:77-120: firstInputSlot, numInputRays); the
        rotation hash and the output slots count from the batch's first ray."""
        if self.normals is None:
            raise _lib.MrtError("DeviceRayGen.ao needs the scene's triangle normals (pass scene=)")
        n = rays.size - first if count is None else count
        if first < 0 or n < 0 or first + n > rays.size:
            raise _lib.MrtError(f"input range [{first}, {first + n}) outside the {rays.size}-ray batch")
        out = torch.empty((n * num_samples, 8), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.mrt_raygen_ao(rays.rays.data_ptr() + 32 * first, rays.results.data_ptr() + 16 * first, n,
                                          self.normals.data_ptr(), self.num_tris, num_samples, float(max_dist),
                                          seed & 0xFFFFFFFF, out.data_ptr(), None, None, _stream_ptr(stream)))
        return RayBuffer(out, need_closest_hit=closest_hit, device=self.device, secondary=True)

    def ao_blocks(self, rays: RayBuffer, num_samples: int, max_dist: float, seeds, batch_inputs: int,
                  blocks: torch.Tensor, block_rays: int, num_rays: int, closest_hit: bool = False,
                  stream=None) -> RayBuffer:
        """The frame's AO/diffuse rays for a list of blocks of its ray order (mrt_raygen_ao_blocks):
        the rays RayGen::batching's batches (batch_inputs input rays each, seeded by seeds[k])
        hold at positions blocks[i] * block_rays + [0, block_rays), concatenated in list order —
        e.g. one rank's shard of the frame in its trace order, generated directly. blocks: int32
        device tensor; num_rays: the rays listed (a partial last block of the frame, when listed,
        must be the last entry: mrt.dist.shard_blocks_device keeps it there)."""
        if self.normals is None:
            raise _lib.MrtError("DeviceRayGen.ao_blocks needs the scene's triangle normals (pass scene=)")
        if blocks.dtype != torch.int32 or blocks.dim() != 1 or blocks.device != torch.device(self.device):
            raise _lib.MrtError("ao_blocks: blocks must be a 1-D int32 tensor on the generator's device")
        sd = (C.c_uint32 * max(1, len(seeds)))(*[s & 0xFFFFFFFF for s in seeds])
        out = torch.empty((num_rays, 8), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.mrt_raygen_ao_blocks(rays.rays.data_ptr(), rays.results.data_ptr(), rays.size,
                                                 self.normals.data_ptr(), self.num_tris, num_samples, float(max_dist),
                                                 C.cast(sd, C.c_void_p), len(seeds), batch_inputs, blocks.data_ptr(),
                                                 blocks.numel(), block_rays, num_rays, out.data_ptr(),
                                                 _stream_ptr(stream)))
        return RayBuffer(out, need_closest_hit=closest_hit, device=self.device, secondary=True)

    def shard_blocks(self, primary: RayBuffer, num_samples: int, block_rays: int, world: int, rank: int,
                     order: int = 1, stream=None) -> tuple[torch.Tensor, int]:
        """mrt_shard_blocks: rank's blocks (block i to rank i % world) of the frame's AO/diffuse
        ray order, in frame order (order 0) or live blocks first (1: decreasing live rays from
        the primary pass's results, ties in frame order, a partial last block last), as an int32
        device tensor, and the rays they hold — two small launches, no host sync."""
        n = C.c_int32(0)
        m = C.c_int64(0)
        _lib.check(self.lib.mrt_shard_blocks(None, primary.size, num_samples, block_rays, world, rank, 0, None, 0,
                                             C.byref(n), C.byref(m), None))
        blocks = torch.empty(max(1, n.value), dtype=torch.int32, device=self.device)
        _lib.check(self.lib.mrt_shard_blocks(primary.results.data_ptr(), primary.size, num_samples, block_rays, world,
                                             rank, order, blocks.data_ptr(), blocks.numel(), C.byref(n), C.byref(m),
                                             _stream_ptr(stream)))
        return blocks[:n.value], m.value

    def count_hits_async(self, rays: RayBuffer, stream=None) -> torch.Tensor:
        """Device int32 scalar: results with id >= 0 (no host sync)."""
        out = torch.empty(1, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.mrt_count_hits(rays.results.data_ptr(), rays.size, out.data_ptr(), _stream_ptr(stream)))
        return out

    def count_hits(self, rays: RayBuffer, stream=None) -> int:
        return int(self.count_hits_async(rays, stream).item())


RAY_PRIMARY, RAY_AO, RAY_DIFFUSE = 0, 1, 2


class DeviceReconstructor:
    """Renderer's reconstruction step on one device (reference Renderer.cc:421-445 +
    reconstructKernel, RendererKernels.cu:60-108): traced batches -> ABGR pixels in HBM."""

    def __init__(self, scene: Scene, device=None):
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.lib = _lib.trace_lib()
        mat, sh = scene.tri_colors()
        self.material = torch.from_numpy(mat.view(np.int32)).to(self.device)
        self.shaded = torch.from_numpy(sh.view(np.int32)).to(self.device)

    def reconstruct(self, ray_type: int, primary: RayBuffer, slot_to_id: torch.Tensor, num_pixels: int,
                    batch: RayBuffer | None = None, num_samples: int = 1, pixels: torch.Tensor | None = None,
                    batch_id_to_slot: torch.Tensor | None = None, stream=None, first_primary: int = 0) -> torch.Tensor:
        """num_pixels int32 (ABGR bits) pixels; batch defaults to the primary batch.
        AO/diffuse batches hold num_samples rays per primary ray (mrt_raygen_ao's layout);
        a batch of RayGen::batching covers the primaries [first_primary, first_primary +
        batch.size / num_samples) (Renderer::updateResult, Renderer.cc:421-445)."""
        if batch is None:
            batch = primary
        if ray_type == RAY_PRIMARY and (num_samples != 1 or batch.size != primary.size or first_primary):
            raise _lib.MrtError("primary reconstruction takes the primary batch with one ray per pixel")
        if batch.size % num_samples:
            raise _lib.MrtError(f"batch holds {batch.size} rays, not a multiple of {num_samples}")
        n_primary = batch.size // num_samples
        if first_primary < 0 or first_primary + n_primary > primary.size:
            raise _lib.MrtError(f"batch covers primaries [{first_primary}, {first_primary + n_primary}) "
                                f"outside the {primary.size}-ray primary batch")
        if slot_to_id.numel() != primary.size:
            raise _lib.MrtError("slot_to_id must hold one pixel id per primary ray")
        if pixels is None:
            pixels = torch.zeros(num_pixels, dtype=torch.int32, device=self.device)
        b2s = None if batch_id_to_slot is None else batch_id_to_slot.data_ptr()
        _lib.check(self.lib.mrt_reconstruct(ray_type, num_samples, first_primary, n_primary, slot_to_id.data_ptr(),
                                            primary.results.data_ptr(), b2s, batch.results.data_ptr(),
                                            self.material.data_ptr(), self.shaded.data_ptr(), pixels.data_ptr(),
                                            _stream_ptr(stream)))
        return pixels
