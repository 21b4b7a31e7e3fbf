"""Fixed-cost probe: rays that miss the root box (1 node visit each)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import torch
import mrt
from mrt.tracer import GpuBvh, RayBuffer, Tracer

def main():
    torch.cuda.set_device(0)
    tr = Tracer(0)
    sc = mrt.Scene.synthetic("mori", 0, 1)
    tr.set_bvh(GpuBvh(mrt.Bvh.build(sc)))
    for n in (1, 64, 4096, 65536, 307200, 786432):
        rays = np.zeros((n, 8), np.float32)
        rays[:, 0:3] = (0, 10, 0); rays[:, 4:7] = (0, 1, 0); rays[:, 7] = 100.0   # pointing away
        rb = RayBuffer(rays)
        for w in (0, 8, 32):
            tr.set_config(waves_per_cu=w)
            ms = sorted(tr.trace_batch(rb, exact_rcp=True) for _ in range(12))[2:-2]
            s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
            s.record(); 
            for _ in range(20): tr.trace_async(rb, exact_rcp=True)
            e.record(); e.synchronize()
            print(f"n={n:7d} waves={w:2d}: trace_batch median {np.median(ms)*1e3:7.1f} us; back-to-back async {s.elapsed_time(e)/20*1e3:7.1f} us/launch", flush=True)
    tr.set_config(waves_per_cu=0)

if __name__ == "__main__":
    main()
