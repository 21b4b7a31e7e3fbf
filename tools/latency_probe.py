"""Single-ray latency probe: the slowest bunny ray traced alone (and x64 in one
wave) by several library variants (tools/build_variant.sh), interleaved.
Slopes against the padded variants give the cost of one dependent VALU op and
of one dependent node load per traversal step."""
import os, sys
import ctypes as C
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd")); sys.path.insert(0, os.path.join(REPO, "tools"))
import torch
import bench
import ab
from mrt import _lib
from mrt.tracer import Tracer, RayBuffer


def main():
    torch.cuda.set_device(0)
    wl = "bunny-primary-1024x768"
    tr = Tracer(0)
    scene, bufs, _, _ = bench.bvh_for("bunny", 1, 0)
    b = bench.Batches(wl, scene, bufs, tr)
    rb = b.batches[0][0]
    tr.trace_batch(rb, exact_rcp=True, speculative=False, stats=True)
    st = rb.stats.cpu().numpy().astype(np.int64)
    steps = st[:, 0] + st[:, 1] + st[:, 2]
    rays = rb.rays.cpu().numpy()
    i = int(np.argmax(steps))
    print(f"slowest ray: {st[i, 0]} nodes {st[i, 1]} tris {st[i, 2]} leaves")
    sets = {"x1": rays[i:i + 1], "x64": np.repeat(rays[i:i + 1], 64, 0), "full": rays}
    g = b.gbvh
    stream = torch.cuda.current_stream()
    libs = []
    for d in sys.argv[1:]:
        lib = ab.load(d)
        h = C.c_void_p()
        assert lib.mrt_tracer_create(0, C.byref(h)) == 0
        assert lib.mrt_tracer_bind(h, g.nodes.data_ptr(), g.node_bytes, g.woop.data_ptr(), g.woop_bytes,
                                   g.tri_index.data_ptr(), g.tri_index_bytes) == 0
        libs.append((d, lib, h))
    res = {(d, k): [] for d, _, _ in libs for k in sets}
    bufs_ = {k: RayBuffer(v) for k, v in sets.items()}
    for r in range(6):
        for d, lib, h in libs:
            for k, sb in bufs_.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(stream)
                for _ in range(10):
                    lib.mrt_tracer_trace(h, sb.rays.data_ptr(), sb.results.data_ptr(), sb.size, 2, None, stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                if r:
                    res[(d, k)].append(e0.elapsed_time(e1) / 10)
    for d, _, _ in libs:
        print(f"  {d:24s} " + "  ".join(f"{k}: {np.median(res[(d, k)]) * 1000:8.1f} us" for k in sets))


if __name__ == "__main__":
    main()
