"""Frame reconstruction — the consumer of the traced batches (reference
reconstructKernel, src/rt/cuda/RendererKernels.cu:60-108, fed by
Renderer.cc:421-445, with Scene::Scene's colour tables, Scene.cc:47-80).

CPU tests pin the oracle (tests/oracle_lib.py -> oracle/trace_oracle.c) with
hand-computed answers and check the host colour tables against it; GPU tests
compare mrt_reconstruct bit for bit with the oracle on traced frames. Parity
unpinned against executed reference output (none exists)."""
import ctypes as C
import os

import numpy as np
import pytest
import torch

import mrt
import oracle_lib as O

BG = 0xFFCC6633          # toABGR(0.2, 0.4, 0.8, 1) with the device's truncation: 51, 102, 204, 255
GREY = 0xFFBFBFBF        # 0.75 * 255 = 191.25 -> 191 (host rounds, device truncates: both 191)


def res(ids):
    r = np.zeros((len(ids), 4), np.int32)
    r[:, 0] = ids
    return r


# ---------------------------------------------------------------- CPU: the oracle
def test_tri_colors_known_answers():
    light = np.array([1, 2, 3], np.float32) / np.float32(np.sqrt(np.float32(14)))
    normals = np.stack([light, -light, np.zeros(3, np.float32)])
    mat, sh = O.tri_colors(normals)
    assert (mat == GREY).all()                       # diffuse 0.75 grey, alpha 1
    assert sh[0] == GREY                             # facing the light: k = 1
    assert sh[1] == 0xFF000000                       # facing away: k = 0
    assert sh[2] == 0xFF606060                       # k = 1/2: 0.375 * 255 = 95.625 rounds to 96


def test_host_tri_colors_equal_the_oracle():
    scene = mrt.Scene.synthetic("conference", 0, 1)
    _, _, normals = scene.arrays()
    mat, sh = scene.tri_colors()
    omat, osh = O.tri_colors(normals)
    assert np.array_equal(mat, omat) and np.array_equal(sh, osh)
    assert len(np.unique(sh)) > 20                   # shading varies with the normal


def test_obj_materials_reach_the_colour_tables(tmp_path):
    """mtllib/usemtl (MeshWavefrontIO.cc:114-200,366-384): per-submesh Kd and d, submeshes
    flattened in order of creation (Scene.cc:63-82); faces before any usemtl, and faces after
    a usemtl naming no loaded material, join the default submesh."""
    open(os.path.join(tmp_path, "m.mtl"), "w").write(
        "newmtl red\nKa 0 0 0\nKd 1 0 0\nd 0.5\n# comment\nnewmtl blue\nKd 0 0 1\n")
    open(os.path.join(tmp_path, "s.obj"), "w").write(
        "mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 0 0 1\n"
        "f 1 2 3\nusemtl blue\nf 1 2 4\nusemtl red\nf 1 3 4\nusemtl blue\nf 2 3 4\nusemtl nomtl\nf 1 3 2\n")
    scene = mrt.Scene.from_obj(os.path.join(tmp_path, "s.obj"))
    mat, sh = scene.tri_colors()
    # flattened order: default submesh (faces 1 and 5: 'nomtl' is undefined), blue (faces 2, 4), red (face 3)
    assert mat.tolist() == [GREY, GREY, 0xFFFF0000, 0xFFFF0000, 0x800000FF]   # d 0.5 -> 127.5 rounds to 128
    _, tris, _ = scene.arrays()
    assert tris.tolist() == [[0, 1, 2], [0, 2, 1], [0, 1, 3], [1, 2, 3], [0, 2, 3]]
    diffuse = np.array([[.75, .75, .75, 1], [.75, .75, .75, 1], [0, 0, 1, 1], [0, 0, 1, 1], [1, 0, 0, .5]], np.float32)
    omat, osh = O.tri_colors(scene.arrays()[2], diffuse)
    assert np.array_equal(mat, omat) and np.array_equal(sh, osh)
    assert (sh >> 24 == 255).all()                    # shaded colours are opaque (Scene.cc:80)


def test_obj_without_material_library_and_bad_indices(tmp_path):
    """MeshWavefrontIO.cc:317-384: with no mtllib every usemtl names an unknown material, so
    all faces stay in the default submesh in file order; a face index outside the vertex list
    becomes the reference's vertex -1 (position 0,0,0); a 'v' line with four values is invalid
    and skipped (it takes no index); an unparsable face is skipped."""
    open(os.path.join(tmp_path, "s.obj"), "w").write(
        "v 1 1 1\nv 1 0 0 1\nv 2 0 0\nv 0 2 0\nusemtl red\nf 1 2 3\nusemtl blue\nf 1 3 9\nf 1 x 3\nf -3 -2 -1\n")
    scene = mrt.Scene.from_obj(os.path.join(tmp_path, "s.obj"))
    v, t, _ = scene.arrays()
    assert scene.num_triangles == 3
    pos = v[t]   # (tri, corner, xyz)
    assert pos.tolist() == [[[1, 1, 1], [2, 0, 0], [0, 2, 0]],
                            [[1, 1, 1], [0, 2, 0], [0, 0, 0]],
                            [[1, 1, 1], [2, 0, 0], [0, 2, 0]]]
    mat, _ = scene.tri_colors()
    assert (mat == GREY).all()


def test_reconstruct_primary_known_answers():
    # two pixels traced in swapped order: slot 0 -> pixel 1 (hit tri 1), slot 1 -> pixel 0 (miss)
    shaded = np.array([0, 0xFF00FF00], np.uint32)
    p = res([1, -1])
    pix = O.reconstruct(0, 1, [1, 0], p, p, shaded, shaded, 2)
    assert pix.tolist() == [BG, 0xFF00FF00]


def test_reconstruct_ao_known_answers():
    prim = res([5, -1])
    # primary 0 (hit): 3 of 4 samples unblocked -> (0.75, 0.75, 0.75, 1); primary 1 missed -> background
    batch = res([-1, 7, -1, -1, -1, -1, -1, -1])
    pix = O.reconstruct(1, 4, [0, 1], prim, batch, np.zeros(8, np.uint32), np.zeros(8, np.uint32), 2)
    assert pix.tolist() == [GREY, BG]
    # every sample blocked -> black with alpha 1
    pix = O.reconstruct(1, 4, [0, 1], prim, res([3] * 8), np.zeros(8, np.uint32), np.zeros(8, np.uint32), 2)
    assert pix[0] == 0xFF000000


def test_reconstruct_diffuse_known_answers():
    material = np.array([0xFF0000FF, 0], np.uint32)  # tri 0: red
    shaded = np.array([0, 0xFFFFFFFF], np.uint32)    # tri 1 shades white
    prim = res([0, -1])
    batch = res([-1, 1, -1, -1])                      # two bounces each: miss (white) + white, miss + miss
    pix = O.reconstruct(2, 2, [0, 1], prim, batch, material, shaded, 2)
    assert pix[0] == 0xFF0000FF                       # white * red
    assert pix[1] == BG                               # white * background


def test_reconstruct_honours_slot_maps_and_batch_window():
    prim = res([-1, -1, -1])
    batch = res([2, -1])                              # one AO sample per primary ray of the window
    shaded = np.zeros(3, np.uint32)
    # window = primaries 1..2 of the frame (firstPrimary 1): batch task i -> batch slot b2s[i]
    pix = O.reconstruct(1, 1, [2, 0, 1], res([-1, 4, 4]), batch, shaded, shaded, 3, batch_id_to_slot=[1, 0],
                        first_primary=1, num_primary=2)
    assert pix.tolist() == [0xFFFFFFFF, 0xFF000000, 0]
    del prim


def test_write_ppm(tmp_path):
    px = np.array([0xFF0000FF, 0xFF00FF00, 0xFFFF0000, 0xFFFFFFFF], np.uint32)   # ABGR: red, green, blue, white
    path = os.path.join(tmp_path, "f.ppm")
    mrt.write_ppm(path, px, 2, 2, flip=False)
    data = open(path, "rb").read()
    assert data.startswith(b"P6\n2 2\n255\n")
    assert data[-12:] == bytes([255, 0, 0, 0, 255, 0, 0, 0, 255, 255, 255, 255])
    mrt.write_ppm(path, px, 2, 2)                    # flipped: bottom row first
    assert open(path, "rb").read()[-12:] == bytes([0, 0, 255, 255, 255, 255, 255, 0, 0, 0, 255, 0])


# ---------------------------------------------------------------- GPU: mrt_reconstruct
@pytest.fixture(scope="module")
def frame():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mrt.raygen import DeviceRayGen, DeviceReconstructor
    from mrt.tracer import GpuBvh, Tracer
    scene = mrt.Scene.synthetic("sponza", 0, 1)
    cam, ao = scene.camera()
    bufs = mrt.Bvh.build(scene).buffers()
    t = Tracer(0)
    t.set_bvh(GpuBvh(bufs))
    return scene, cam, ao, bufs, t, DeviceRayGen(scene), DeviceReconstructor(scene)


def _oracle_pixels(scene, ray_type, n, s2i, pres, bres, w, h):
    mat, sh = O.tri_colors(scene.arrays()[2])
    return O.reconstruct(ray_type, n, s2i, pres, bres, mat, sh, w * h)


@pytest.mark.gpu
@pytest.mark.parametrize("ray_type,samples", [(0, 1), (1, 1), (1, 8), (2, 1), (2, 4)])
def test_device_reconstruct_equals_the_oracle(frame, ray_type, samples):
    scene, cam, ao, bufs, t, g, rec = frame
    w, h = 160, 96
    prim, s2i = g.primary(cam, w, h)
    t.trace_batch(prim, exact_rcp=True)
    batch = None
    if ray_type == 1:
        batch = g.ao(prim, samples, ao)
    elif ray_type == 2:
        batch = g.ao(prim, samples, cam.far, closest_hit=True)
    if batch is not None:
        t.trace_batch(batch, exact_rcp=True)
    pix = rec.reconstruct(ray_type, prim, s2i, w * h, batch=batch, num_samples=samples)
    dev = pix.cpu().numpy().view(np.uint32)
    bres = (batch if batch is not None else prim).results_numpy()
    want = _oracle_pixels(scene, ray_type, samples, s2i.cpu().numpy(), prim.results_numpy(), bres, w, h)
    assert np.array_equal(dev, want)
    # a real image, not a constant (AO: background, black, white and the partial levels)
    assert len(np.unique(dev)) >= (3 if ray_type == 1 else 9)


@pytest.mark.gpu
def test_device_primary_frame_end_to_end(frame, tmp_path):
    """Device raygen -> trace -> reconstruct against host rays -> oracle trace -> oracle reconstruct."""
    scene, cam, ao, bufs, t, g, rec = frame
    w, h = 200, 150
    prim, s2i = g.primary(cam, w, h)
    t.trace_batch(prim)                              # production mode: closest hit bit-identical
    dev = rec.reconstruct(0, prim, s2i, w * h).cpu().numpy().view(np.uint32)
    host_rays, host_s2i = mrt.primary_rays(cam, w, h)
    hres, _, _ = O.trace(host_rays, *bufs, threads=8)
    assert np.array_equal(dev, _oracle_pixels(scene, 0, 1, host_s2i, hres, hres, w, h))
    mrt.write_ppm(os.path.join(tmp_path, "sponza.ppm"), dev, w, h)


@pytest.mark.gpu
def test_device_reconstruct_rejects_bad_shapes(frame):
    scene, cam, ao, bufs, t, g, rec = frame
    prim, s2i = g.primary(cam, 8, 8)
    with pytest.raises(mrt._lib.MrtError):   # 64 rays are not whole 3-sample groups
        rec.reconstruct(1, prim, s2i, 64, batch=prim, num_samples=3)
    with pytest.raises(mrt._lib.MrtError):   # 16 primaries from primary 60 run past the 64-ray primary batch
        rec.reconstruct(1, prim, s2i, 64, batch=prim, num_samples=4, first_primary=60)
    with pytest.raises(mrt._lib.MrtError):   # primary reconstruction takes the whole primary batch
        rec.reconstruct(0, prim, s2i, 64, batch=prim, first_primary=1)


def test_reconstruct_argument_checks_without_gpu():
    lib = mrt._lib.trace_lib()
    assert lib.mrt_reconstruct(3, 1, 0, 1, 1, 1, None, 1, 1, 1, 1, None) == 1     # bad ray type
    assert lib.mrt_reconstruct(0, 2, 0, 1, 1, 1, None, 1, 1, 1, 1, None) == 1     # primary takes one ray
    assert lib.mrt_reconstruct(1, 1, 0, 0, None, None, None, None, None, None, None, None) == 0   # empty


class ReconstructInput(C.Structure):
    """RendererKernels.hh:46-61, field for field (mrt.h mrt_reconstruct_input)."""
    _fields_ = [("numRaysPerPrimary", C.c_int32), ("firstPrimary", C.c_int32), ("numPrimary", C.c_int32),
                ("isPrimary", C.c_bool), ("isAO", C.c_bool), ("isDiffuse", C.c_bool),
                ("primarySlotToID", C.c_void_p), ("primaryResults", C.c_void_p), ("batchIDToSlot", C.c_void_p),
                ("batchResults", C.c_void_p), ("triMaterialColor", C.c_void_p), ("triShadedColor", C.c_void_p),
                ("pixels", C.c_void_p)]


class CountHitsInput(C.Structure):
    """RendererKernels.hh:65-70 (mrt.h mrt_count_hits_input)."""
    _fields_ = [("numRays", C.c_int32), ("rayResults", C.c_void_p), ("raysPerThread", C.c_int32)]


def test_compat_input_struct_layout():
    assert ReconstructInput.primarySlotToID.offset == 16 and C.sizeof(ReconstructInput) == 72
    assert CountHitsInput.rayResults.offset == 8 and C.sizeof(CountHitsInput) == 24


@pytest.mark.gpu
def test_reference_compat_launchers(frame):
    """launch_reconstructKernel / launch_countHitsKernel called the way Renderer.cc:421-445 does."""
    scene, cam, ao, bufs, t, g, rec = frame
    w, h, n = 96, 64, 4
    prim, s2i = g.primary(cam, w, h)
    t.trace_batch(prim)
    batch = g.ao(prim, n, ao)
    t.trace_batch(batch)
    want = rec.reconstruct(1, prim, s2i, w * h, batch=batch, num_samples=n).cpu().numpy()
    ident = torch.arange(batch.size, dtype=torch.int32, device=prim.results.device)
    pixels = torch.zeros(w * h, dtype=torch.int32, device=prim.results.device)
    inp = ReconstructInput(n, 0, prim.size, False, True, False, s2i.data_ptr(), prim.results.data_ptr(),
                           ident.data_ptr(), batch.results.data_ptr(), rec.material.data_ptr(),
                           rec.shaded.data_ptr(), pixels.data_ptr())
    lib = mrt._lib.trace_lib()
    lib.launch_reconstructKernel(prim.size, C.byref(inp))
    assert np.array_equal(pixels.cpu().numpy(), want)
    blk = (C.c_int32 * 2)(32, 8)
    cnt = CountHitsInput(batch.size, batch.results.data_ptr(), 16)
    assert lib.launch_countHitsKernel(batch.size, blk, C.byref(cnt)) == g.count_hits(batch)


@pytest.mark.gpu
@pytest.mark.parametrize("ray_type,samples", [(1, 20), (2, 17), (1, 3)])
def test_tiled_and_gathering_paths_agree_on_ragged_frames(frame, ray_type, samples):
    """The LDS-staged kernel (identity layout, tiles of 16 samples) against the gathering
    kernel (explicit batchIdToSlot) and the oracle, on a frame that fills no block exactly."""
    scene, cam, ao, bufs, t, g, rec = frame
    w, h = 97, 33
    prim, s2i = g.primary(cam, w, h)
    t.trace_batch(prim)
    batch = g.ao(prim, samples, ao if ray_type == 1 else cam.far, closest_hit=ray_type == 2)
    t.trace_batch(batch)
    tiled = rec.reconstruct(ray_type, prim, s2i, w * h, batch=batch, num_samples=samples).cpu().numpy()
    ident = torch.arange(batch.size, dtype=torch.int32, device=prim.results.device)
    gathered = rec.reconstruct(ray_type, prim, s2i, w * h, batch=batch, num_samples=samples,
                               batch_id_to_slot=ident).cpu().numpy()
    assert np.array_equal(tiled, gathered)
    want = _oracle_pixels(scene, ray_type, samples, s2i.cpu().numpy(), prim.results_numpy(), batch.results_numpy(),
                          w, h)
    assert np.array_equal(tiled.view(np.uint32), want)


class RayGenPrimaryInput(C.Structure):
    """RayGenKernels.hh:40-51 (mrt.h mrt_raygen_primary_input)."""
    _fields_ = [("origin", C.c_float * 3), ("nscreenToWorld", C.c_float * 16), ("w", C.c_int32), ("h", C.c_int32),
                ("maxDist", C.c_float), ("rays", C.c_void_p), ("idToSlot", C.c_void_p), ("slotToID", C.c_void_p),
                ("indexToPixel", C.c_void_p)]


class RayGenAOInput(C.Structure):
    """RayGenKernels.hh:55-68 (mrt.h mrt_raygen_ao_input)."""
    _fields_ = [("firstInputSlot", C.c_int32), ("numInputRays", C.c_int32), ("numSamples", C.c_int32),
                ("maxDist", C.c_float), ("randomSeed", C.c_uint32), ("inRays", C.c_void_p),
                ("inResults", C.c_void_p), ("outRays", C.c_void_p), ("outIDToSlot", C.c_void_p),
                ("outSlotToID", C.c_void_p), ("normals", C.c_void_p)]


def test_raygen_input_struct_layout():
    assert RayGenPrimaryInput.rays.offset == 88 and C.sizeof(RayGenPrimaryInput) == 120
    assert RayGenAOInput.inRays.offset == 24 and C.sizeof(RayGenAOInput) == 72


@pytest.mark.gpu
def test_reference_compat_raygen_launchers(frame):
    """launch_rayGenPrimaryKernel / launch_rayGenAOKernel (RayGen.cc:50-120 call shapes) produce
    the same rays as the stream-ordered entry points; firstInputSlot offsets the input only."""
    from mrt.raygen import nscreen_to_world
    from mrt.tracer import RayBuffer
    scene, cam, ao, bufs, t, g, rec = frame
    w, h = 64, 40
    dev = prim_dev = torch.device("cuda", 0)
    want, want_s2i = g.primary(cam, w, h)
    rays = torch.zeros((w * h, 8), dtype=torch.float32, device=dev)
    s2i = torch.zeros(w * h, dtype=torch.int32, device=dev)
    i2s = torch.zeros(w * h, dtype=torch.int32, device=dev)
    table = torch.from_numpy(mrt.pixel_table(w, h)).to(dev)
    inp = RayGenPrimaryInput((C.c_float * 3)(*cam.position), (C.c_float * 16)(*nscreen_to_world(cam, w, h)), w, h,
                             float(cam.far), rays.data_ptr(), i2s.data_ptr(), s2i.data_ptr(), table.data_ptr())
    lib = mrt._lib.trace_lib()
    lib.launch_rayGenPrimaryKernel(w * h, C.byref(inp))
    assert torch.equal(rays.view(torch.int32), want.rays.view(torch.int32)) and torch.equal(s2i, want_s2i)
    assert torch.equal(i2s[s2i.long()], torch.arange(w * h, dtype=torch.int32, device=dev))
    t.trace_batch(want)
    first, n, samples = 100, 500, 3
    sub = RayBuffer(want.rays[first:first + n].clone(), device=prim_dev)
    sub.results.copy_(want.results[first:first + n])
    expect = g.ao(sub, samples, ao).rays
    out = torch.zeros((n * samples, 8), dtype=torch.float32, device=dev)
    o2s = torch.zeros(n * samples, dtype=torch.int32, device=dev)
    ainp = RayGenAOInput(first, n, samples, float(ao), mrt.AO_SEED, want.rays.data_ptr(), want.results.data_ptr(),
                         out.data_ptr(), o2s.data_ptr(), None, g.normals.data_ptr())
    lib.launch_rayGenAOKernel(n, C.byref(ainp))
    assert torch.equal(out.view(torch.int32), expect.view(torch.int32))
    assert torch.equal(o2s, torch.arange(n * samples, dtype=torch.int32, device=dev))
