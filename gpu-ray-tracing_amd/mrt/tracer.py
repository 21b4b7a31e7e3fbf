"""Device-side mirror of the reference's tracing classes, over lib/libmrt.so.

  GpuBvh     <- CudaBVH      (src/rt/cuda/CudaBVH.cc:55-116): Compact2 buffers resident in HBM
  RayBuffer  <- RayBuffer    (src/rt/ray/RayBuffer.cc:53-81): Ray[n] in, RayResult[n] out, on device
  Tracer     <- CudaTracer   (src/rt/cuda/CudaTracer.cc:84-177): setBVH / traceBatch(RayBuffer&) -> ms

Device memory and streams come from PyTorch (plumbing); every launch goes
through the C-ABI of include/mrt.h. There is no CPU path: without a GPU the
Tracer constructor raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .host import Bvh


def _stream_ptr(stream) -> int | None:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream or None


class GpuBvh:
    """Compact2 node / Woop / triIndex buffers uploaded to the current device."""

    def __init__(self, bvh: Bvh | tuple, device=None):
        """bvh: a host Bvh, or (nodes, woop, triIndex) as int32 numpy arrays or tensors
        (device tensors, e.g. from mrt.dist.replicate_buffers, are bound in place)."""
        nodes, woop, tri = bvh.buffers() if isinstance(bvh, Bvh) else bvh
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())

        def upload(a):
            if isinstance(a, torch.Tensor):
                return a.to(dev, torch.int32).contiguous()
            return torch.from_numpy(np.ascontiguousarray(a, np.int32)).to(dev)
        self.nodes, self.woop, self.tri_index = upload(nodes), upload(woop), upload(tri)
        self.device = dev

    @property
    def node_bytes(self) -> int:
        return self.nodes.numel() * 4

    @property
    def woop_bytes(self) -> int:
        return self.woop.numel() * 4

    @property
    def tri_index_bytes(self) -> int:
        return self.tri_index.numel() * 4

    @property
    def total_bytes(self) -> int:
        return self.node_bytes + self.woop_bytes + self.tri_index_bytes


class RayBuffer:
    """Ray[n] (32 B) and RayResult[n] (16 B) arrays on the device.

    needClosestHit selects the trace mode exactly like the reference
    (anyHit = !needClosestHit, CudaTracer.cc:172)."""

    def __init__(self, rays, need_closest_hit: bool = True, device=None, results: torch.Tensor | None = None,
                 secondary: bool = False):
        """results: an existing int32 [n, 4] device tensor to write into (e.g. a
        slice of a larger RayResult array, for the shards of one RayBuffer).
        secondary: the rays are AO / diffuse / later-bounce rays (a tuning hint, MRT_TRACE_SECONDARY:
        the autotuner keeps their schedule apart from a primary batch of the same size)."""
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if isinstance(rays, torch.Tensor):
            self.rays = rays.to(dev, torch.float32).contiguous().view(-1, 8)
        else:
            self.rays = torch.from_numpy(np.ascontiguousarray(rays, np.float32).reshape(-1, 8)).to(dev)
        if results is None:
            results = torch.zeros((self.rays.shape[0], 4), dtype=torch.int32, device=dev)
        elif tuple(results.shape) != (self.rays.shape[0], 4) or not results.is_contiguous() or \
                results.dtype != torch.int32:
            raise ValueError("results must be a contiguous int32 [n, 4] tensor matching the rays")
        self.results = results
        self.need_closest_hit = need_closest_hit
        self.secondary = bool(secondary)
        self.stats = None

    def view(self, lo: int, hi: int) -> "RayBuffer":
        """Rays [lo, hi) of this buffer as a RayBuffer sharing its rays and results."""
        return RayBuffer(self.rays[lo:hi], self.need_closest_hit, self.rays.device, self.results[lo:hi],
                         secondary=self.secondary)

    @property
    def size(self) -> int:
        return int(self.rays.shape[0])

    def results_numpy(self) -> np.ndarray:
        return self.results.cpu().numpy()

    def hit_ids(self) -> np.ndarray:
        return self.results_numpy()[:, 0]

    def hit_t(self) -> np.ndarray:
        return self.results_numpy()[:, 1].view(np.float32)


class Tracer:
    """Persistent-wave BVH tracer for one HIP device (mirror of CudaTracer)."""

    def __init__(self, device: int | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("mrt.Tracer needs a HIP device; there is no CPU fallback")
        self.lib = _lib.trace_lib()
        self.device = torch.cuda.current_device() if device is None else int(device)
        h = C.c_void_p()
        _lib.check(self.lib.mrt_tracer_create(self.device, C.byref(h)))
        self._h = h
        self.bvh: GpuBvh | None = None

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self.lib.mrt_tracer_destroy(self._h)
            self._h = C.c_void_p()

    # -- configuration -------------------------------------------------------
    def config(self) -> dict:
        c = _lib.LaunchCfg()
        _lib.check(self.lib.mrt_tracer_get_config(self._h, C.byref(c)))
        return {k: getattr(c, k) for k, _ in c._fields_}

    def set_config(self, **kw) -> None:
        cur = self.config()
        cur.update(kw)
        c = _lib.LaunchCfg(**cur)
        _lib.check(self.lib.mrt_tracer_set_config(self._h, C.byref(c)))

    def bind_info(self) -> dict:
        """What the last bind derived: wall ms, wide-node bytes/format, stack capacity."""
        b = _lib.BindInfo()
        _lib.check(self.lib.mrt_tracer_bind_info(self._h, C.byref(b)))
        return {k: getattr(b, k) for k, _ in b._fields_}

    def schedules(self) -> list:
        """The autotuner's settled schedules [(num_rays, variant, candidate, version)]."""
        n = C.c_int32()
        _lib.check(self.lib.mrt_tracer_tune_export(self._h, None, 0, C.byref(n)))
        arr = (_lib.TunedSchedule * max(1, n.value))()
        _lib.check(self.lib.mrt_tracer_tune_export(self._h, arr, n.value, C.byref(n)))
        return [(e.num_rays, e.variant, e.candidate, e.version) for e in arr[:n.value]]

    def load_schedules(self, entries) -> None:
        """Lock schedules saved by schedules() from an earlier run on the same BVH
        (call after set_bvh: binding forgets them)."""
        entries = list(entries)
        arr = (_lib.TunedSchedule * max(1, len(entries)))(*[_lib.TunedSchedule(*e) for e in entries])
        _lib.check(self.lib.mrt_tracer_tune_import(self._h, arr, len(entries)))

    # -- CudaTracer API --------------------------------------------------------
    def set_bvh(self, bvh: GpuBvh) -> None:
        """setBVH + bind_CudaBVHTexture (CudaTracer.cc:142-146); re-binding is allowed."""
        _lib.check(self.lib.mrt_tracer_bind(self._h, bvh.nodes.data_ptr(), bvh.node_bytes, bvh.woop.data_ptr(),
                                            bvh.woop_bytes, bvh.tri_index.data_ptr(), bvh.tri_index_bytes))
        self.bvh = bvh

    def flags(self, rays: RayBuffer, exact_rcp=False, speculative=True, stats=False) -> int:
        f = 0 if rays.need_closest_hit else _lib.MRT_TRACE_ANY_HIT
        if exact_rcp:
            f |= _lib.MRT_TRACE_EXACT_RCP
        if not speculative:
            f |= _lib.MRT_TRACE_LOCKSTEP_OFF
        if stats:
            f |= _lib.MRT_TRACE_STATS
        if getattr(rays, "secondary", False):
            f |= _lib.MRT_TRACE_SECONDARY
        return f

    def trace_async(self, rays: RayBuffer, exact_rcp=False, speculative=True, stats=False, stream=None) -> None:
        """Stream-ordered trace of the whole batch (no host sync)."""
        if self.bvh is None:
            raise _lib.MrtError("Tracer: No BVH!")   # CudaTracer.cc:129-130
        f = self.flags(rays, exact_rcp, speculative, stats)
        sp = None
        if stats:
            if rays.stats is None or rays.stats.shape[0] != rays.size:
                rays.stats = torch.zeros((rays.size, 4), dtype=torch.int32, device=rays.rays.device)
            sp = rays.stats.data_ptr()
        _lib.check(self.lib.mrt_tracer_trace(self._h, rays.rays.data_ptr(), rays.results.data_ptr(), rays.size, f,
                                             sp, _stream_ptr(stream)))

    def launcher(self, rays: RayBuffer, exact_rcp=False, speculative=True, stream=None):
        """A zero-argument callable that re-issues trace_async(rays, ...) with every
        argument resolved once: one C call per launch, for tight launch loops."""
        if self.bvh is None:
            raise _lib.MrtError("Tracer: No BVH!")
        fn, h = self.lib.mrt_tracer_trace, self._h
        args = (rays.rays.data_ptr(), rays.results.data_ptr(), rays.size, self.flags(rays, exact_rcp, speculative),
                None, _stream_ptr(stream))
        check = _lib.check

        def launch():
            rc = fn(h, *args)
            if rc:
                check(rc)
        launch.stream = stream if stream is not None else torch.cuda.current_stream()
        return launch

    def trace_batch(self, rays: RayBuffer, exact_rcp=False, speculative=True, stats=False, stream=None) -> float:
        """CudaTracer::traceBatch: blocking, returns the launch's milliseconds (0 for no rays)."""
        if self.bvh is None:
            raise _lib.MrtError("Tracer: No BVH!")
        f = self.flags(rays, exact_rcp, speculative, stats)
        sp = None
        if stats:
            if rays.stats is None or rays.stats.shape[0] != rays.size:
                rays.stats = torch.zeros((rays.size, 4), dtype=torch.int32, device=rays.rays.device)
            sp = rays.stats.data_ptr()
        info = _lib.TraceInfo()
        _lib.check(self.lib.mrt_tracer_trace_timed(self._h, rays.rays.data_ptr(), rays.results.data_ptr(), rays.size,
                                                   f, sp, _stream_ptr(stream), C.byref(info)))
        self.last_info = {k: getattr(info, k) for k, _ in info._fields_}
        return float(info.kernel_ms)
