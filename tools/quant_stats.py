"""Per-ray traversal counters of the exact and the quantized 4-wide nodes (cfg.wide 1 / 2) on the
same batches: wide-node visits, triangle tests and 16-B lane loads (7 per exact node, 4 per quantized
node, 3 per triangle), from the kernel's STATS variant. Usage: python tools/quant_stats.py WORKLOAD..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    from mrt.tracer import Tracer
    torch.cuda.set_device(0)
    scenes = bench.SceneCache(1, 0, "/tmp/mrt_bvhcache")
    for wl in sys.argv[1:]:
        e = scenes.get(bench.workload_spec(wl)[0])
        tr = Tracer(0)
        b = bench.Batches(wl, e["scene"], e["gbvh"], tr)
        for wide, loads in ((1, 7), (2, 4)):
            tr.set_config(wide=wide, autotune=0)
            n = t = rays = 0
            for rb, _ in b.batches:
                tr.trace_batch(rb, exact_rcp=True, speculative=True, stats=True)
                s = rb.stats.to(torch.int64)
                n, t, rays = n + s[:, 0].sum().item(), t + s[:, 1].sum().item(), rays + rb.size
                rb.stats = None
            print(f"{wl:26s} wide={wide}: nodes/ray {n / rays:6.2f}  tris/ray {t / rays:6.2f}  "
                  f"16-B lane loads/ray {(n * loads + 3 * t) / rays:6.1f}", flush=True)


if __name__ == "__main__":
    main()
