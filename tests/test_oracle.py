"""CPU oracle (oracle/trace_oracle.c) pinned against hand-derived known
answers and the committed golden fixtures; plus BVH-independence against a
brute-force scan of every triangle."""
import os

import numpy as np
import pytest

import kat
import mrt
import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("case", kat.cases(), ids=lambda c: c[0])
def test_known_answers(case):
    name, scene, rays, any_hit, expected = case
    nodes, woop, tri = scene()
    res, stats, _ = O.trace(np.stack(rays), nodes, woop, tri, any_hit=any_hit, stats=True)
    for (rid, rt), got in zip(expected, res):
        assert got[0] == rid, name
        assert got[1] == kat.f2i(rt), f"{name}: t={got[1:2].view(np.float32)[0]} want {rt}"
    assert (stats[:, 3] == 0).all()


def test_kat_woop_rows_match_the_product_woopify():
    """mrth_woopify (CudaBVH::woopifyTri restated, with the reference's
    cofactor-inverse quirk) equals the exact inverse on exactly representable triangles."""
    for v0, v1, v2 in [((0, 0, 0), (1, 0, 0), (0, 1, 0)), ((2, 0, -1), (4, 0, -1), (2, 2, -1)),
                       ((0, 0, -3), (1, 0, -3), (0, 1, -3))]:
        assert np.array_equal(mrt.woopify(v0, v1, v2), kat.woop_rows(v0, v1, v2))


def _golden_files():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))


@pytest.mark.parametrize("fname", _golden_files())
def test_oracle_reproduces_golden_fixture(fname):
    g = np.load(os.path.join(GOLDEN, fname))
    res, stats, _ = O.trace(g["rays"], g["nodes"], g["woop"], g["tri_index"], any_hit=bool(g["any_hit"]),
                            stats=True, threads=4)
    assert np.array_equal(res[:, :2], g["results"][:, :2])
    assert np.array_equal(stats[:, :3], g["stats"][:, :3])


@pytest.mark.parametrize("fname", _golden_files())
def test_builder_reproduces_golden_compact2(fname):
    """The SBVH + Compact2 bytes of the fixture scene are reproducible (determinism pin)."""
    g = np.load(os.path.join(GOLDEN, fname))
    scene = mrt.Scene.synthetic(str(g["scene"]), int(g["param"]), int(g["seed"]))
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    assert np.array_equal(nodes, g["nodes"]) and np.array_equal(woop, g["woop"]) and np.array_equal(tri, g["tri_index"])


@pytest.mark.parametrize("scene_name,param", [("sphere", 20), ("random", 2000), ("mori", 0)])
def test_closest_hit_equals_brute_force(scene_name, param):
    scene = mrt.Scene.synthetic(scene_name, param, 3)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 80, 60)
    res, _, _ = O.trace(rays, nodes, woop, tri, threads=4)
    bf = O.brute_force(rays, woop, tri)
    same = (res[:, 0] == bf[:, 0]) & (res[:, 1] == bf[:, 1])
    # Any difference must be an exact-t tie between two valid triangles.
    for i in np.nonzero(~same)[0]:
        assert res[i, 1] == bf[i, 1], f"ray {i}: BVH t differs from brute force"
    assert same.mean() > 0.999


def test_any_hit_agrees_with_closest_on_hit_or_miss():
    scene = mrt.Scene.synthetic("random", 3000, 5)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 64, 48)
    closest, _, _ = O.trace(rays, nodes, woop, tri)
    anyh, _, _ = O.trace(rays, nodes, woop, tri, any_hit=True)
    assert np.array_equal(closest[:, 0] == -1, anyh[:, 0] == -1)
    # an any-hit t is a real hit, never closer than the closest one
    hit = closest[:, 0] != -1
    assert (anyh[hit, 1].view(np.float32) >= closest[hit, 1].view(np.float32)).all()


def test_invalid_hits_accepts_genuine_results_and_rejects_altered_ones():
    """oracle_lib.invalid_hits (the batch valid-hit check of the GPU any-hit and fast-rcp
    tests): every result the oracle itself reports is genuine — closest and
    any hit, hits and misses — and one ulp on a hit's t, another triangle id, or a miss
    whose t is not tmax is not."""
    scene = mrt.Scene.synthetic("random", 3000, 5)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 64, 48)
    for any_hit in (False, True):
        res, _, _ = O.trace(rays, nodes, woop, tri, any_hit=any_hit)
        assert len(O.invalid_hits(rays, res, woop, tri)) == 0
    hits = np.nonzero(res[:, 0] != -1)[0][:50]
    misses = np.nonzero(res[:, 0] == -1)[0][:50]
    assert len(hits) == 50 and len(misses) == 50
    bad_t = res.copy()
    bad_t[hits, 1] += 1
    assert np.array_equal(O.invalid_hits(rays, bad_t, woop, tri, which=hits), hits)
    bad_id = res.copy()
    bad_id[hits, 0] += 1   # the neighbouring triangle (never the same t bits on these rays)
    assert len(O.invalid_hits(rays, bad_id, woop, tri, which=hits)) == 50
    bad_miss = res.copy()
    bad_miss[misses, 1] = np.float32(1.0).view(np.int32)
    assert np.array_equal(O.invalid_hits(rays, bad_miss, woop, tri, which=misses), misses)
    # with 1/Dz allowed one ulp off (the fast mode's bound) a one-ulp t may be genuine
    assert len(O.invalid_hits(rays, bad_t, woop, tri, which=hits, rcp_ulps=1)) < 50


def test_threads_do_not_change_results():
    scene = mrt.Scene.synthetic("mori", 0, 1)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 128, 96)
    a, sa, _ = O.trace(rays, nodes, woop, tri, stats=True, threads=1)
    b, sb, _ = O.trace(rays, nodes, woop, tri, stats=True, threads=8)
    assert np.array_equal(a, b) and np.array_equal(sa, sb)


def test_empty_batch():
    nodes, woop, tri = kat.scene_two_floors()
    res, _, _ = O.trace(np.zeros((0, 8), np.float32), nodes, woop, tri)
    assert res.shape == (0, 4)


@pytest.mark.parametrize("jx,jy", [(0.5, 0.5), (0.25, 0.875)])
def test_camera_matrix_export_reproduces_the_host_primary_rays(jx, jy):
    """mrth_camera_nscreen_to_world (the matrix the device generator takes) with the
    reference's per-ray formula (RayGenKernels.cu:88-110) gives the host rays, at the
    pixel centre (the reference) and at another sample position inside the pixel."""
    from mrt.raygen import nscreen_to_world
    scene = mrt.Scene.synthetic("bunny", 0, 1)
    cam, _ = scene.camera()
    w, h = 48, 40
    rays, slots = mrt.primary_rays(cam, w, h, subpixel=(jx, jy))
    m = nscreen_to_world(cam, w, h).reshape(4, 4).T   # column-major -> [row][col]
    f = np.float32
    px = slots.astype(np.int64)
    ns = np.stack([f(2) * ((px % w).astype(f) + f(jx)) / f(w) - f(1), f(2) * ((px // w).astype(f) + f(jy)) / f(h) - f(1),
                   np.zeros(len(px), f), np.ones(len(px), f)], 1).astype(f)
    wp4 = np.zeros((len(px), 4), f)
    for i in range(4):
        acc = np.zeros(len(px), f)
        for j in range(4):
            acc = (acc + m[i, j] * ns[:, j]).astype(f)
        wp4[:, i] = acc
    wp = wp4[:, :3] / wp4[:, 3:4]
    d = (wp - np.array(cam.position, f)).astype(f)
    dd = (f(0) + d[:, 0] * d[:, 0]).astype(f)
    dd = (dd + d[:, 1] * d[:, 1]).astype(f)
    dd = (dd + d[:, 2] * d[:, 2]).astype(f)
    inv = (f(1) * (f(1) / np.sqrt(dd))).astype(f)
    dirs = (d * inv[:, None]).astype(f)
    assert np.array_equal(dirs.view(np.uint32), rays[:, 4:7].view(np.uint32))


@pytest.mark.parametrize("scene_name,tris", [("mori", 12570), ("bunny", 144500), ("sponza", 121384),
                                             ("conference", 350949), ("dragon", 910348), ("fairy", 174117),
                                             ("sibenik", 75284)])
def test_stand_in_scenes_have_their_triangle_counts(scene_name, tris):
    """README.md:48-58 counts (fairy/sibenik: commonly distributed sizes, the README gives none)."""
    assert mrt.Scene.synthetic(scene_name, 0, 1).num_triangles == tris


def test_closed_nave_stand_in_hits_every_primary_ray():
    """The sibenik stand-in is a closed interior: diffuse rays from it never escape (README diffuse row)."""
    scene = mrt.Scene.synthetic("sibenik", 0, 1)
    nodes, woop, tri = mrt.Bvh.build(scene).buffers()
    cam, _ = scene.camera()
    rays, _ = mrt.primary_rays(cam, 48, 36)
    res, _, _ = O.trace(rays, nodes, woop, tri, threads=4)
    assert (res[:, 0] != -1).all()


@pytest.mark.parametrize("scene_name,digest", [("conference", "dfbbbfea18d11fba"), ("sponza", "c7e34a6a5c968e5e"),
                                               ("bunny", "a030c6170e26b859")])
def test_builder_output_is_pinned(scene_name, digest):
    """SHA-256 (prefix) of the Compact2 bytes of three stand-ins: the builder's output must not move when its
    internals do (the sort, the threading). Regression pin of this repo's builder, not a reference output."""
    import hashlib
    nodes, woop, tri = mrt.Bvh.build(mrt.Scene.synthetic(scene_name, 0, 1)).buffers()
    assert hashlib.sha256(nodes.tobytes() + woop.tobytes() + tri.tobytes()).hexdigest()[:16] == digest


def test_comb_stack_depth_known_answer():
    """kat.scene_comb: 40 pushes trace to the hand answer; 70 exceed the reference's
    64-entry stack and the oracle flags the overflow (stats[3]) like the kernel does."""
    for depth, overflow in ((40, 0), (63, 0), (64, 1), (70, 1)):
        bufs, r, (tid, t) = kat.scene_comb(depth)
        res, st, _ = O.trace(np.stack([r]), *bufs, stats=True)
        assert st[0, 3] == overflow, depth
        if not overflow:
            assert res[0, 0] == tid and res[0, 1] == kat.f2i(t)
            assert st[0, 0] == depth   # every inner node fetched once
