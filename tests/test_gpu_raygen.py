"""Device ray generation and hit counting (mrt_raygen_primary / mrt_raygen_ao /
mrt_count_hits) against the host generator, which runs the same per-ray code
(csrc/raygen_common.hpp) on the CPU."""
import numpy as np
import pytest
import torch

import mrt
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gen():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mrt.raygen import DeviceRayGen
    return DeviceRayGen


def ftz(a):
    """Host floats with denormals flushed (the device runs FTZ)."""
    a = a.copy()
    a[np.abs(a) < np.float32(1.1754944e-38)] = 0.0
    return a


@pytest.mark.parametrize("subpixel", [(0.25, 0.75), (0.0, 0.999)])
def test_subpixel_primary_rays_match_the_host_bit_for_bit(gen, subpixel):
    scene = mrt.Scene.synthetic("bunny", 0, 1)
    cam, _ = scene.camera()
    host_rays, _ = mrt.primary_rays(cam, 160, 120, subpixel=subpixel)
    rb, _ = gen(scene).primary(cam, 160, 120, subpixel=subpixel)
    assert np.array_equal(rb.rays.cpu().numpy().view(np.uint32), ftz(host_rays).view(np.uint32))


@pytest.mark.parametrize("scene_name,w,h", [("bunny", 320, 240), ("conference", 333, 217), ("mori", 64, 9),
                                            ("sponza", 1, 1)])
def test_primary_rays_match_the_host_bit_for_bit(gen, scene_name, w, h):
    scene = mrt.Scene.synthetic(scene_name, 0, 1)
    cam, _ = scene.camera()
    host_rays, host_slots = mrt.primary_rays(cam, w, h)
    rb, slots = gen(scene).primary(cam, w, h)
    dev = rb.rays.cpu().numpy()
    assert np.array_equal(slots.cpu().numpy(), host_slots)
    assert np.array_equal(dev.view(np.uint32), ftz(host_rays).view(np.uint32))


@pytest.mark.parametrize("samples", [1, 4])
def test_ao_rays_match_the_host(gen, samples):
    scene = mrt.Scene.synthetic("conference", 0, 1)
    cam, ao = scene.camera()
    prim, _ = mrt.primary_rays(cam, 200, 150)
    bufs = mrt.Bvh.build(scene).buffers()
    res, _, _ = O.trace(prim, *bufs, threads=8)
    host = mrt.ao_rays(prim, res, scene, ao, samples, mrt.AO_SEED)

    from mrt.tracer import RayBuffer
    g = gen(scene)
    rb = RayBuffer(prim)
    rb.results.copy_(torch.from_numpy(res.view(np.int32).reshape(-1, 4)))
    dev = g.ao(rb, samples, ao).rays.cpu().numpy()
    # origin, tmin, tmax: same arithmetic, no transcendental -> identical bits
    for c in (0, 1, 2, 3, 7):
        assert np.array_equal(dev[:, c].view(np.uint32), ftz(host[:, c]).view(np.uint32)), f"column {c}"
    # directions go through cosf/sinf (ocml vs glibc): a few ulp
    assert np.abs(dev[:, 4:7] - host[:, 4:7]).max() < 4e-6
    assert np.allclose(np.linalg.norm(dev[:, 4:7], axis=1), 1.0, atol=1e-5)


def test_diffuse_frame_on_the_device_matches_the_host_pipeline(gen):
    """primary -> trace -> diffuse bounce -> trace, all on the device, against the
    same pipeline with host-generated rays and the oracle."""
    from mrt.tracer import GpuBvh, Tracer
    scene = mrt.Scene.synthetic("sponza", 0, 1)
    cam, _ = scene.camera()
    bufs = mrt.Bvh.build(scene).buffers()
    t = Tracer(0)
    t.set_bvh(GpuBvh(bufs))
    g = gen(scene)
    prim, _ = g.primary(cam, 256, 192)
    t.trace_batch(prim, exact_rcp=True)
    hits = g.count_hits(prim)
    sec = g.ao(prim, 1, cam.far, closest_hit=True)
    t.trace_batch(sec, exact_rcp=True)

    host_prim, _ = mrt.primary_rays(cam, 256, 192)
    hres, _, _ = O.trace(host_prim, *bufs, threads=8)
    assert np.array_equal(prim.results_numpy()[:, :2], hres[:, :2])   # bit-identical primary rays
    assert hits == mrt.count_hits(hres)
    host_sec = mrt.ao_rays(host_prim, hres, scene, cam.far, 1, mrt.AO_SEED)
    hsec, _, _ = O.trace(host_sec, *bufs, threads=8)
    dres = sec.results_numpy()
    # ulp-level direction differences may flip a grazing ray; nothing more
    assert (dres[:, 0] != hsec[:, 0]).mean() < 2e-3
    assert abs(g.count_hits(sec) - mrt.count_hits(hsec)) <= 0.002 * len(hsec)


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 100_000, 1_000_003])
def test_count_hits(gen, n):
    from mrt.tracer import RayBuffer
    rng = np.random.default_rng(n)
    rb = RayBuffer(np.zeros((n, 8), np.float32))
    ids = np.where(rng.random(n) < 0.37, rng.integers(0, 1 << 30, n), -1).astype(np.int32)
    rb.results[:, 0] = torch.from_numpy(ids).cuda()
    assert gen().count_hits(rb) == int((ids >= 0).sum())


def test_per_sample_ao_kernel_matches_the_per_ray_kernel(gen):
    """numSamples > 1 runs one thread per output ray (coalesced writes); its sample 0 of
    every input ray must be the per-ray kernel's (numSamples == 1) bits."""
    from mrt.tracer import GpuBvh, Tracer
    scene = mrt.Scene.synthetic("conference", 0, 1)
    cam, ao = scene.camera()
    t = Tracer(0)
    t.set_bvh(GpuBvh(mrt.Bvh.build(scene).buffers()))
    g = gen(scene)
    prim, _ = g.primary(cam, 123, 45)
    t.trace_batch(prim)
    one = g.ao(prim, 1, ao).rays.cpu().numpy()
    many = g.ao(prim, 7, ao).rays.cpu().numpy().reshape(-1, 7, 8)
    assert np.array_equal(many[:, 0].view(np.uint32), one.view(np.uint32))
    assert len(np.unique(many[:, :, 4])) > len(one)   # the other samples are distinct directions
