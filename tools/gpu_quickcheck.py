"""Quick end-to-end GPU check: trace synthetic scenes on the GPU in every kernel
mode and compare with the CPU oracle. Prints one line per case."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
import mrt
from mrt.tracer import GpuBvh, RayBuffer, Tracer
import oracle_lib as O

def main():
    tr = Tracer()
    print("config", tr.config(), flush=True)
    for name, w, h in [("mori", 320, 240), ("bunny", 640, 480), ("conference", 640, 480)]:
        sc = mrt.Scene.synthetic(name, 0, 1)
        bvh = mrt.Bvh.build(sc)
        nodes, woop, tri = bvh.buffers()
        g = GpuBvh((nodes, woop, tri))
        tr.set_bvh(g)
        cam, ao = sc.camera()
        rays, _ = mrt.primary_rays(cam, w, h)
        ores, ost, _ = O.trace(rays, nodes, woop, tri, stats=True, threads=8)
        for exact in (True, False):
            for spec in (False, True):
                rb = RayBuffer(rays, need_closest_hit=True)
                ms = tr.trace_batch(rb, exact_rcp=exact, speculative=spec, stats=(not spec))
                r = rb.results_numpy()
                same_id = (r[:, 0] == ores[:, 0]).mean()
                same_all = ((r[:, 0] == ores[:, 0]) & (r[:, 1] == ores[:, 1])).mean()
                extra = ""
                if not spec:
                    s = rb.stats.cpu().numpy()
                    extra = f" stats_equal={(s[:, :3] == ost[:, :3]).all()}"
                print(f"{name} primary exact={exact} spec={spec}: {ms:.3f} ms {len(rays)/ms/1e3:.1f} Mrays/s id_eq={same_id:.6f} all_eq={same_all:.6f}{extra} info={tr.last_info}", flush=True)
        # AO rays from oracle primary results
        aor = mrt.ao_rays(rays, ores, sc, ao)
        oao, oaost, _ = O.trace(aor, nodes, woop, tri, any_hit=True, stats=True, threads=8)
        for spec in (False, True):
            rb = RayBuffer(aor, need_closest_hit=False)
            ms = tr.trace_batch(rb, exact_rcp=True, speculative=spec)
            r = rb.results_numpy()
            hit_eq = ((r[:, 0] != -1) == (oao[:, 0] != -1)).mean()
            all_eq = ((r[:, 0] == oao[:, 0]) & (r[:, 1] == oao[:, 1])).mean()
            print(f"{name} AO spec={spec}: {ms:.3f} ms hit_eq={hit_eq:.6f} all_eq={all_eq:.6f}", flush=True)

if __name__ == "__main__":
    main()
