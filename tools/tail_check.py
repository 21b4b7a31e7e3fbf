"""Single-launch check of tail export/resume configs: ms per trace (both passes),
records exported, and equality with the first config's results. Prints per launch."""
import json, os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
import torch
import bench
from mrt.tracer import Tracer

def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "bunny-primary-640x480"
    cfgs = [json.loads(c) for c in sys.argv[2:]] or [{"tail_lanes": -1}, {"tail_lanes": 32, "tail_after_us": 30}]
    torch.cuda.set_device(0)
    t0 = time.time()
    scene, bufs, _, _ = bench.bvh_for(bench.workload_spec(w)[0], 1, 0)
    tr = Tracer(0)
    b = bench.Batches(w, scene, bufs, tr)
    print(f"{w}: setup {time.time() - t0:.1f} s", flush=True)
    rb = b.batches[-1][0]
    ref = None
    for c in cfgs:
        tr.set_config(**c)
        for i in range(4):
            ms = tr.trace_batch(rb, exact_rcp=True)
            out = rb.results_numpy()[:, :2].copy()
            if ref is None:
                ref = out
            same = np.array_equal(out, ref) if rb.need_closest_hit else bool(((out[:, 0] != -1) == (ref[:, 0] != -1)).all())
            print(f"  {c} launch {i}: {ms:.4f} ms same={same} info={tr.last_info}", flush=True)

if __name__ == "__main__":
    main()
