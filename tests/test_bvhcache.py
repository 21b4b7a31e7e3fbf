"""The reference's bvhcache naming (Renderer::getCudaBVH, Renderer.cc:157-217):
"<bvhCachePath>/%08x.dat" with hashBits(scene.hash(), platform.computeHash(),
buildParams.computeHash(), BVHLayout_Compact2). The framework hash
(src/framework/base/Hash.hh:181-201, Hash.cc:34-112) is restated independently
here and compared with the host library's.

Parity unpinned against the reference binary: its Hash.cc cannot be compiled here
(Defs.hh:188-190 includes <cuda.h> unconditionally, absent from this image), so the
pins are this restatement and the hand-derived values below.
"""
import ctypes as C
import os

import numpy as np
import pytest

import mrt

MAGIC = 0x9E3779B9
M32 = 0xFFFFFFFF


def mix(a, b, c):
    a = (a - b - c) & M32; a ^= c >> 13
    b = (b - c - a) & M32; b ^= (a << 8) & M32
    c = (c - a - b) & M32; c ^= b >> 13
    a = (a - b - c) & M32; a ^= c >> 12
    b = (b - c - a) & M32; b ^= (a << 16) & M32
    c = (c - a - b) & M32; c ^= b >> 5
    a = (a - b - c) & M32; a ^= c >> 3
    b = (b - c - a) & M32; b ^= (a << 10) & M32
    c = (c - a - b) & M32; c ^= b >> 15
    return a, b, c


def hash_buffer(data: bytes) -> int:
    a = b = c = MAGIC
    n = len(data)
    i = 0
    while n >= 12:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & M32
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & M32
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & M32
        a, b, c = mix(a, b, c)
        i += 12
        n -= 12
    tail = data[i:]
    # the reference's fall-through switch: bytes 0-3 into a, 4-7 into b, 8-10 into c, little end first
    for k in range(n):
        word, shift = divmod(k, 4)
        if word == 0:
            a = (a + (tail[k] << 8 * shift)) & M32
        elif word == 1:
            b = (b + (tail[k] << 8 * shift)) & M32
        else:
            c = (c + (tail[k] << 8 * shift)) & M32
    c = (c + n) & M32
    return mix(a, b, c)[2]


def hash_bits(a, b=MAGIC, c=0):
    return mix(a & M32, b & M32, (c + MAGIC) & M32)[2]


def hash_bits6(a, b, c, d, e=0, f=0):
    a, b, c = mix(a & M32, b & M32, (c + MAGIC) & M32)
    return mix((a + d) & M32, (b + e) & M32, (c + f) & M32)[2]


def fbits(x):
    return int(np.float32(x).view(np.uint32))


@pytest.mark.parametrize("n", list(range(0, 30)) + [1000, 4096])
def test_hash_buffer_matches_the_restatement(n):
    data = bytes((i * 37 + 11) & 0xFF for i in range(n))
    buf = C.create_string_buffer(data, max(n, 1))
    assert mrt._lib.host_lib().mrth_fw_hash_buffer(buf, n) == hash_buffer(data)


def test_hash_known_answers():
    """Hand-checkable corners of the hash: the tail length (not the total) enters c, so a
    12-byte and a 24-byte zero buffer hash alike after their block mixes differ only there."""
    assert hash_buffer(b"") == mix(MAGIC, MAGIC, MAGIC)[2]
    assert hash_bits(0) == mix(0, MAGIC, MAGIC)[2]
    assert hash_buffer(b"\x01") == mix(MAGIC + 1, MAGIC, MAGIC + 1)[2]


@pytest.mark.parametrize("name", ["mori", "sponza"])
def test_scene_hash_and_cache_name_match_the_restatement(name):
    scene = mrt.Scene.synthetic(name, 0, 1)
    v, t, n = scene.arrays()
    mat, sh = scene.tri_colors()
    want_scene = hash_bits6(hash_buffer(t.astype(np.int32).tobytes()), hash_buffer(n.astype(np.float32).tobytes()),
                            hash_buffer(mat.astype(np.uint32).tobytes()), hash_buffer(sh.astype(np.uint32).tobytes()),
                            hash_buffer(v.astype(np.float32).tobytes()))
    assert scene.hash() == want_scene
    platform = hash_bits6(hash_buffer(b"GPU"), fbits(1.0), fbits(1.0), hash_bits6(1, 1, 1, 8))
    params = hash_bits(fbits(1e-5))
    assert mrt.Bvh.cache_name(scene) == "%08x.dat" % hash_bits6(want_scene, platform, params, 5)
    # a different split alpha or leaf size names a different file
    assert mrt.Bvh.cache_name(scene, split_alpha=1e-6) != mrt.Bvh.cache_name(scene)
    assert mrt.Bvh.cache_name(scene, max_leaf=4) != mrt.Bvh.cache_name(scene)


def test_load_or_build_uses_the_cache(tmp_path):
    scene = mrt.Scene.synthetic("mori", 0, 1)
    d = str(tmp_path / "bvhcache")
    b1 = mrt.Bvh.load_or_build(scene, d)
    path = os.path.join(d, mrt.Bvh.cache_name(scene))
    assert os.path.exists(path)
    mtime = os.path.getmtime(path)
    b2 = mrt.Bvh.load_or_build(scene, d)
    assert os.path.getmtime(path) == mtime
    for x, y in zip(b1.buffers(), b2.buffers()):
        assert np.array_equal(x, y)


def test_obj_vertices_follow_the_reference_numbering(tmp_path):
    """MeshWavefrontIO.cc:317-348: one mesh vertex per distinct (position, texcoord, normal)
    triple, numbered in order of first use — position 1 used with two texcoords is two
    vertices — which is what Scene::hash sees."""
    p = tmp_path / "m.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvn 0 0 1\n"
                 "f 1/1/1 2/2/1 3/1/1\nf 1/2/1 2/2/1 3/1/1\nf 3 2 1\n")
    scene = mrt.Scene.from_obj(str(p))
    v, t, _ = scene.arrays()
    assert scene.num_vertices == 7
    assert t.tolist() == [[0, 1, 2], [3, 1, 2], [4, 5, 6]]
    assert v[t].tolist() == [[[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 0, 0], [1, 0, 0], [0, 1, 0]],
                             [[0, 1, 0], [1, 0, 0], [0, 0, 0]]]


def fw_parse_float(s: str) -> np.float32:
    """String.cc:452-509 for plain decimals: float32 accumulation, scale *= 0.1f."""
    f = np.float32
    neg = s.startswith("-")
    s = s.lstrip("+-")
    whole, _, frac = s.partition(".")
    v = f(0)
    for ch in whole:
        v = f(f(v * f(10)) + f(int(ch)))
    scale = f(1)
    for ch in frac:
        scale = f(scale * f(0.1))
        v = f(v + f(scale * f(int(ch))))
    return f(-v) if neg else v


def test_obj_numbers_use_the_framework_parser(tmp_path):
    """Vertex coordinates come out of the reference's own float parser (not strtof):
    0.123 accumulates as 0.1 + 0.01*2 + 0.001*3 in float32."""
    vals = ["0.123", "-7.3", "12.3456789", "0.7", "100.001", "3"]
    p = tmp_path / "n.obj"
    p.write_text("v " + " ".join(vals[:3]) + "\nv " + " ".join(vals[3:]) + "\nv 0 0 0\nf 1 2 3\n")
    v, _, _ = mrt.Scene.from_obj(str(p)).arrays()
    want = np.array([fw_parse_float(x) for x in vals], np.float32)
    assert np.array_equal(v[:2].reshape(-1).view(np.uint32), want.view(np.uint32))
    strtof = np.array([np.float32(float(x)) for x in vals], np.float32)
    assert not np.array_equal(want.view(np.uint32), strtof.view(np.uint32))   # the two parsers differ here
