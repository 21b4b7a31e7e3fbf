#!/usr/bin/env python3
"""Render one frame the way the reference's App does (App.cc:137-210, Renderer.cc:
221-238,421-445): primary rays -> trace -> [AO / diffuse rays -> trace] ->
reconstruct -> image, all on the device; writes a PPM and prints one JSON line
with the trace rate (rays counted / trace time, App.cc:204) and the reconstruct
time.

  python tools/render_frame.py --scene sponza --ray-type diffuse --samples 8 \
      --width 640 --height 480 --out gpurun_out/sponza-diffuse.ppm
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))

import torch  # noqa: E402

import mrt  # noqa: E402
from mrt.raygen import RAY_AO, RAY_DIFFUSE, RAY_PRIMARY, DeviceRayGen, DeviceReconstructor  # noqa: E402
from mrt.tracer import GpuBvh, Tracer  # noqa: E402

TYPES = {"primary": RAY_PRIMARY, "ao": RAY_AO, "diffuse": RAY_DIFFUSE}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--obj", default=None, help="an OBJ file instead of a synthetic stand-in")
    ap.add_argument("--ray-type", choices=sorted(TYPES), default="primary")
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--out", default="gpurun_out/frame.ppm")
    a = ap.parse_args()
    if not torch.cuda.is_available():
        raise SystemExit("render_frame needs a GPU")
    scene = mrt.Scene.from_obj(a.obj) if a.obj else mrt.Scene.synthetic(a.scene, 0, 1)
    cam, ao_radius = scene.camera()
    tracer = Tracer(0)
    tracer.set_bvh(GpuBvh(mrt.Bvh.build(scene).buffers()))
    gen, rec = DeviceRayGen(scene), DeviceReconstructor(scene)
    w, h, rt = a.width, a.height, TYPES[a.ray_type]

    prim, slot_to_id = gen.primary(cam, w, h)
    ms = tracer.trace_batch(prim)
    counted = w * h   # every primary ray counts; secondary rays only where the primary hit (bench.py)
    batch, n = None, 1
    if rt != RAY_PRIMARY:
        n = a.samples
        batch = gen.ao(prim, n, ao_radius if rt == RAY_AO else cam.far, closest_hit=rt == RAY_DIFFUSE)
        counted = gen.count_hits(prim) * n
        ms = tracer.trace_batch(batch)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    pixels = rec.reconstruct(rt, prim, slot_to_id, w * h, batch=batch, num_samples=n)
    end.record()
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    mrt.write_ppm(a.out, pixels.cpu().numpy(), w, h)
    print(json.dumps({"scene": a.obj or a.scene, "ray_type": a.ray_type, "width": w, "height": h, "samples": n,
                      "trace_ms": round(ms, 4), "rays_counted": counted,
                      "mrays_per_s": round(counted / ms / 1e3, 2) if ms > 0 else None,
                      "reconstruct_ms": round(start.elapsed_time(end), 4), "image": a.out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
