"""mrt — MI355X BVH ray-traversal engine (drop-in for the reference's
CudaTracer::traceBatch hot path). See DESIGN.md at the repository root.

Host-side pieces (scenes, SBVH, Compact2, ray generation) import without a GPU;
the tracer (mrt.tracer) needs torch + a HIP device.
"""
from . import _lib
from .host import AO_SEED, Bvh, Camera, Scene, ao_rays, count_hits, pixel_table, primary_rays, woopify, write_ppm

__all__ = ["_lib", "AO_SEED", "Bvh", "Camera", "Scene", "ao_rays", "count_hits", "pixel_table", "primary_rays",
           "woopify", "write_ppm"]
