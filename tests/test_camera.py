"""Camera signatures (CameraControls::decodeSignature, CameraControls.cc:374-419,
502-554) — every signature of the reference's benchmark command lines
(tests/golden/camera_signatures.txt, from grtcmdline.txt and test.txt) decoded by
the host library and checked against

  * an independent restatement here (6-bit characters, 6 characters per float
    little end first, direction faces normalised in float32 as
    VectorBase::normalized does), bit for bit; and
  * values derived by hand from the encoding: "///m10" + "0" ends every
    conference/sibenik/sponza signature, i.e. far = bits 50<<18 | 2<<24 | 1<<30
    = 0x42C80000 = 100.0 and keepAligned = 1; "///Uy2" + "0" (bunny/fairy/mori)
    is 36<<18 | 60<<24 | 1<<30 = 0x43FA0000 = 500.0.
"""
import os
import struct

import numpy as np
import pytest

import mrt

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "camera_signatures.txt")


def signatures():
    out = []
    for line in open(GOLDEN):
        if line.startswith("#") or not line.strip():
            continue
        scene, sig = line.rstrip("\n").split("\t")
        out.append((scene, sig))
    return out


def _bits(c):
    o = ord(c)
    if ord("/") <= o <= ord(":"):
        return o - ord("/")
    if ord("A") <= o <= ord("Z"):
        return o - ord("A") + 12
    if ord("a") <= o <= ord("z"):
        return o - ord("a") + 38
    raise ValueError(c)


def restated_decode(sig):
    """Independent decoder (float32 arithmetic through numpy in the reference's order)."""
    pos = [0]

    def bits():
        v = _bits(sig[pos[0]])
        pos[0] += 1
        return v

    def flt():
        u = 0
        for i in range(0, 32, 6):
            u |= bits() << i
        return np.float32(struct.unpack("<f", struct.pack("<I", u & 0xFFFFFFFF))[0])

    def direction():
        face = bits()
        x = np.float32(1.0 if not face & 4 else -1.0)
        y = flt() if not face & 8 else np.float32(0.0)
        z = flt() if not face & 8 else np.float32(0.0)
        len_sq = np.float32(np.float32(np.float32(np.float32(0) + x * x) + y * y) + z * z)
        k = np.float32(np.float32(1.0) * (np.float32(1.0) / np.sqrt(len_sq)))
        x, y, z = x * k, y * k, z * k
        return [(x, y, z), (z, x, y), (y, z, x), (y, z, x)][face & 3]

    p = (flt(), flt(), flt())
    fwd, up = direction(), direction()
    speed, fov, near, far = flt(), flt(), flt(), flt()
    keep = bits()
    assert pos[0] == len(sig)
    return p, fwd, up, speed, fov, near, far, keep


def f32bits(x):
    return int(np.float32(x).view(np.uint32))


@pytest.mark.parametrize("scene,sig", signatures(), ids=lambda v: v if len(v) < 20 else v[:12])
def test_signature_decodes_like_the_reference(scene, sig):
    cam = mrt.Camera.from_signature(sig)
    p, fwd, up, speed, fov, near, far, keep = restated_decode(sig)
    assert [f32bits(v) for v in cam.position] == [f32bits(v) for v in p]
    assert [f32bits(v) for v in cam.forward] == [f32bits(v) for v in fwd]
    assert [f32bits(v) for v in cam.up] == [f32bits(v) for v in up]
    assert f32bits(cam.fov) == f32bits(fov) and f32bits(cam.near) == f32bits(near)
    assert f32bits(cam.far) == f32bits(far) and f32bits(cam.speed) == f32bits(speed)
    assert cam.keep_aligned == bool(keep)
    # hand-derived from the encoding (module docstring)
    if sig.endswith("///m100"):
        assert f32bits(cam.far) == 0x42C80000 and cam.far == 100.0
    if sig.endswith("///Uy200"):
        assert f32bits(cam.far) == 0x43FA0000 and cam.far == 500.0
    assert cam.keep_aligned
    assert abs(np.linalg.norm(cam.forward) - 1.0) < 1e-6 and abs(np.linalg.norm(cam.up) - 1.0) < 1e-6
    assert 0 < cam.near < cam.far and 1.0 < cam.fov < 179.0


def test_all_reference_signatures_present():
    sigs = signatures()
    assert len(sigs) == 23
    # (sponza's, breakfast_room's, gallery's and test.txt's signatures repeat ones listed under earlier meshes)
    assert {s for s, _ in sigs} >= {"conference.obj", "bunny.obj", "hairball.obj", "dragon.obj", "sibenik.obj",
                                    "fairyforest.obj", "sanmiguel.obj", "testObj.obj"}


def test_axis_aligned_direction_faces():
    """Face bit 3 set = an axis-aligned direction with no components (CameraControls.cc:540-554):
    the conference up vector '9' = face 10 = 8 | 2 -> axis 2, positive: (0, 0, 1); 'B' = face 13 =
    8 | 4 | 1 -> axis 1, negative: tuv = (-1, 0, 0) rotated to (tuv.z, tuv.x, tuv.y) = (0, -1, 0);
    '8' = face 9 -> (0, 1, 0)."""
    cam = mrt.Camera.from_signature("6omr/04j3200bR6Z/0/3ZEAz/x4smy19///c/05frY109Qx7w////m100")
    assert cam.up == (0.0, 0.0, 1.0)
    # hand-built: position 0, forward face 13 (-y), up face 9 (+y), four zero floats, keepAligned 1
    zero = "//////"
    sig = zero * 3 + "B" + "8" + zero * 4 + "0"
    c = mrt.Camera.from_signature(sig)
    assert c.position == (0.0, 0.0, 0.0)
    assert c.forward == (0.0, -1.0, 0.0) and c.up == (0.0, 1.0, 0.0)


@pytest.mark.parametrize("bad", ["", "6omr", "6omr/04j3200bR6Z/0/3ZEAz/x4smy19///c/05frY109Qx7w////m100x",
                                 "6omr/04j3200bR6Z/0/3ZEAz/x4smy19///c/05frY109Qx7w////m10!"])
def test_invalid_signatures_fail(bad):
    with pytest.raises(mrt._lib.MrtError):
        mrt.Camera.from_signature(bad)


def test_quotes_comma_and_whitespace_are_accepted():
    sig = "6omr/04j3200bR6Z/0/3ZEAz/x4smy19///c/05frY109Qx7w////m100"
    a = mrt.Camera.from_signature(sig)
    b = mrt.Camera.from_signature(f'  \t"{sig}",\n')
    assert a == b


def test_signature_camera_drives_primary_rays():
    """A decoded reference camera feeds the primary generator (RayGen.cc:50-72 via
    Renderer.cc:126-129): the centre ray of a frame points along the camera's forward."""
    cam = mrt.Camera.from_signature("ShGMy/wx6Zz/Ypn8/05TJTmx1ljevx18///m007toC10AnAHx///Uy200")
    rays, slot_to_id = mrt.primary_rays(cam, 64, 48)
    centre = rays[np.argmax(slot_to_id == 24 * 64 + 32)]
    assert np.allclose(centre[0:3], cam.position)
    assert np.dot(centre[4:7], cam.forward) > 0.999
    assert (rays[:, 7] == np.float32(cam.far)).all()
