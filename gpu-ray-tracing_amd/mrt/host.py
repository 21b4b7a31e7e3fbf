"""Host-side producers of the trace inputs (scenes, SBVH/Compact2, rays).

Thin wrappers over lib/libmrt_host.so (include/mrt_host.h); every array is a
numpy array in the reference's binary layout:
  rays     float32 [n, 8]  (orig.xyz, tmin, dir.xyz, tmax)     src/rt/Util.hh:64-73
  results  int32   [n, 4]  (id, t bits, pad, pad)              src/rt/Util.hh:79-89
  nodes    int32   [k*16]  Compact2 inner nodes (64 B each)    src/rt/cuda/CudaBVH.hh:40-55
  woop     int32   [m*4]   Woop rows + (-0,-0,-0,-0) terminators
  triIndex int32   [m]     original triangle id per woop float4 slot
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib

# glibc's first rand() with the default seed: the reference's AO seed (RayGen.cc:106).
AO_SEED = 1804289383


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


@dataclass
class Camera:
    position: tuple
    forward: tuple
    up: tuple
    fov: float
    near: float
    far: float

    @classmethod
    def from_signature(cls, sig: str) -> "Camera":
        """CameraControls::decodeSignature (CameraControls.cc:374-419): the reference App's
        --camera text, e.g. the signatures of grtcmdline.txt. The signature's speed and
        keepAligned are kept as attributes."""
        c = _lib.HostCamera()
        speed, keep = C.c_float(), C.c_int32()
        _lib.check_host(_lib.host_lib().mrth_camera_decode_signature(sig.encode(), C.byref(c), C.byref(speed),
                                                                     C.byref(keep)))
        cam = cls(tuple(c.position), tuple(c.forward), tuple(c.up), c.fov_deg, c.near_dist, c.far_dist)
        cam.speed, cam.keep_aligned = float(speed.value), bool(keep.value)
        return cam

    def to_c(self) -> _lib.HostCamera:
        c = _lib.HostCamera()
        for i in range(3):
            c.position[i] = self.position[i]
            c.forward[i] = self.forward[i]
            c.up[i] = self.up[i]
        c.fov_deg, c.near_dist, c.far_dist = self.fov, self.near, self.far
        return c


class Scene:
    """A flattened triangle scene (reference src/rt/Scene.cc:35-83)."""

    def __init__(self, handle: int, name: str):
        self._h = C.c_void_p(handle)
        self.name = name
        # bound now: at interpreter exit the module's globals may already be gone when __del__ runs
        self._destroy = _lib.host_lib().mrth_scene_destroy

    @classmethod
    def synthetic(cls, name: str, param: int = 0, seed: int = 1) -> "Scene":
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_scene_synthetic(name.encode(), param, seed, C.byref(h)))
        return cls(h.value, name)

    @classmethod
    def from_obj(cls, path: str) -> "Scene":
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_scene_load_obj(path.encode(), C.byref(h)))
        return cls(h.value, path)

    @classmethod
    def from_arrays(cls, vertices, triangles, name: str = "arrays") -> "Scene":
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        t = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 3)
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_scene_from_arrays(_ptr(v), len(v), _ptr(t), len(t), C.byref(h)))
        return cls(h.value, name)

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._destroy(self._h)
            self._h = C.c_void_p()

    @property
    def handle(self):
        return self._h

    @property
    def num_triangles(self) -> int:
        return int(_lib.host_lib().mrth_scene_num_triangles(self._h))

    @property
    def num_vertices(self) -> int:
        return int(_lib.host_lib().mrth_scene_num_vertices(self._h))

    def arrays(self):
        nv, nt = self.num_vertices, self.num_triangles
        v = np.empty((nv, 3), np.float32)
        t = np.empty((nt, 3), np.int32)
        n = np.empty((nt, 3), np.float32)
        _lib.check_host(_lib.host_lib().mrth_scene_copy_arrays(self._h, _ptr(v), _ptr(t), _ptr(n)))
        return v, t, n

    def hash(self) -> int:
        """Scene::hash (Scene.cc:93-101)."""
        return int(_lib.host_lib().mrth_scene_hash(self._h))

    def tri_colors(self):
        """(material, shaded) ABGR uint32 per triangle (Scene::Scene, reference Scene.cc:47-80)."""
        nt = self.num_triangles
        mat = np.empty(nt, np.uint32)
        sh = np.empty(nt, np.uint32)
        _lib.check_host(_lib.host_lib().mrth_scene_tri_colors(self._h, _ptr(mat), _ptr(sh)))
        return mat, sh

    def camera(self):
        c = _lib.HostCamera()
        ao = C.c_float()
        _lib.check_host(_lib.host_lib().mrth_scene_camera(self._h, C.byref(c), C.byref(ao)))
        cam = Camera(tuple(c.position), tuple(c.forward), tuple(c.up), c.fov_deg, c.near_dist, c.far_dist)
        return cam, float(ao.value)


class Bvh:
    """Compact2 BVH buffers on the host (reference CudaBVH, BVHLayout_Compact2)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)
        self._destroy = _lib.host_lib().mrth_bvh_destroy   # bound now, as in Scene

    @classmethod
    def build(cls, scene: Scene, max_leaf: int = 8, min_leaf: int = 1, split_alpha: float = 1e-5,
              threads: int = 0) -> "Bvh":
        p = _lib.BuildParams()
        _lib.host_lib().mrth_default_build_params(C.byref(p))
        p.max_leaf_size, p.min_leaf_size, p.split_alpha, p.threads = max_leaf, min_leaf, split_alpha, threads
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_bvh_build(scene.handle, C.byref(p), C.byref(h)))
        return cls(h.value)

    @staticmethod
    def _params(max_leaf=8, min_leaf=1, split_alpha=1e-5, threads=0):
        p = _lib.BuildParams()
        _lib.host_lib().mrth_default_build_params(C.byref(p))
        p.max_leaf_size, p.min_leaf_size, p.split_alpha, p.threads = max_leaf, min_leaf, split_alpha, threads
        return p

    @classmethod
    def cache_name(cls, scene: Scene, max_leaf: int = 8, min_leaf: int = 1, split_alpha: float = 1e-5) -> str:
        """The reference's bvhcache file name for this scene and build, "%08x.dat" of
        hashBits(scene, platform, build params, layout) (Renderer.cc:178-186)."""
        buf = C.create_string_buffer(16)
        _lib.check_host(_lib.host_lib().mrth_bvh_cache_name(scene.handle, C.byref(cls._params(max_leaf, min_leaf,
                                                                                              split_alpha)), buf))
        return buf.value.decode()

    @classmethod
    def load_or_build(cls, scene: Scene, cache_dir: str = "bvhcache", **build) -> "Bvh":
        """Renderer::getCudaBVH (Renderer.cc:157-217): read <cache_dir>/<cache_name>.dat when it
        exists, otherwise build the SBVH and write it there (creating the directory)."""
        import os
        build_keys = {k: build[k] for k in ("max_leaf", "min_leaf", "split_alpha") if k in build}
        path = os.path.join(cache_dir, cls.cache_name(scene, **build_keys))
        if os.path.exists(path):
            return cls.load(path)
        bvh = cls.build(scene, **build)
        os.makedirs(cache_dir, exist_ok=True)
        bvh.save(path)
        return bvh

    @classmethod
    def load(cls, path: str) -> "Bvh":
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_bvh_load(path.encode(), C.byref(h)))
        return cls(h.value)

    @classmethod
    def from_buffers(cls, nodes: np.ndarray, woop: np.ndarray, tri_index: np.ndarray) -> "Bvh":
        n = np.ascontiguousarray(nodes).view(np.int32)
        w = np.ascontiguousarray(woop).view(np.int32)
        t = np.ascontiguousarray(tri_index, dtype=np.int32)
        h = C.c_void_p()
        _lib.check_host(_lib.host_lib().mrth_bvh_from_buffers(_ptr(n), n.nbytes, _ptr(w), w.nbytes, _ptr(t),
                                                               t.nbytes, C.byref(h)))
        return cls(h.value)

    def save(self, path: str) -> None:
        _lib.check_host(_lib.host_lib().mrth_bvh_save(self._h, path.encode()))

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._destroy(self._h)
            self._h = C.c_void_p()

    def buffers(self):
        """(nodes, woop, triIndex) as int32 numpy copies."""
        pn, pw, pt = C.c_void_p(), C.c_void_p(), C.c_void_p()
        nb, wb, tb = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check_host(_lib.host_lib().mrth_bvh_buffers(self._h, C.byref(pn), C.byref(nb), C.byref(pw),
                                                         C.byref(wb), C.byref(pt), C.byref(tb)))

        def grab(p, nbytes):
            if nbytes == 0:
                return np.zeros(0, np.int32)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(nbytes // 4,)).copy()

        return grab(pn, nb.value), grab(pw, wb.value), grab(pt, tb.value)

    def stats(self) -> dict:
        s = _lib.BvhStats()
        _lib.check_host(_lib.host_lib().mrth_bvh_get_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in s._fields_}


def woopify(v0, v1, v2) -> np.ndarray:
    a = [(C.c_float * 3)(*map(float, v)) for v in (v0, v1, v2)]
    out = (C.c_float * 12)()
    _lib.host_lib().mrth_woopify(a[0], a[1], a[2], out)
    return np.array(out, np.float32).reshape(3, 4)


def pixel_table(w: int, h: int) -> np.ndarray:
    out = np.empty(w * h, np.int32)
    _lib.check_host(_lib.host_lib().mrth_pixel_table(w, h, _ptr(out)))
    return out


def primary_rays(cam: Camera, w: int, h: int, subpixel=(0.5, 0.5)):
    """RayGen::primary (RayGen.cc:50-72): w*h rays in Morton pixel order + slot->pixel ids.
    subpixel: sample position inside each pixel (the reference's is the centre)."""
    rays = np.empty((w * h, 8), np.float32)
    slot_to_id = np.empty(w * h, np.int32)
    c = cam.to_c()
    if tuple(subpixel) == (0.5, 0.5):
        _lib.check_host(_lib.host_lib().mrth_primary_rays(C.byref(c), w, h, _ptr(rays), _ptr(slot_to_id)))
    else:
        _lib.check_host(_lib.host_lib().mrth_primary_rays_subpixel(C.byref(c), w, h, float(subpixel[0]),
                                                                   float(subpixel[1]), _ptr(rays), _ptr(slot_to_id)))
    return rays, slot_to_id


def ao_rays(primary: np.ndarray, primary_results: np.ndarray, scene: Scene, max_dist: float,
            num_samples: int = 1, seed: int = AO_SEED) -> np.ndarray:
    p = np.ascontiguousarray(primary, np.float32)
    r = np.ascontiguousarray(primary_results).view(np.int32).reshape(-1, 4)
    out = np.empty((len(p) * num_samples, 8), np.float32)
    _lib.check_host(_lib.host_lib().mrth_ao_rays(_ptr(p), _ptr(r), len(p), scene.handle, num_samples,
                                                 float(max_dist), seed & 0xFFFFFFFF, _ptr(out)))
    return out


def count_hits(results: np.ndarray) -> int:
    r = np.ascontiguousarray(results).view(np.int32).reshape(-1, 4)
    return int(_lib.host_lib().mrth_count_hits(_ptr(r), len(r)))


def write_ppm(path: str, pixels: np.ndarray, w: int, h: int, flip: bool = True) -> None:
    """Binary PPM (P6) of w*h ABGR uint32 pixels indexed y*w + x (the reference's
    PBO, Renderer.cc:221-238). flip=True writes row h-1 first: the reference drew
    the PBO with GL, whose row 0 is the bottom of the window."""
    px = np.ascontiguousarray(pixels, np.uint32).reshape(h, w)
    if flip:
        px = px[::-1]
    rgb = np.stack([px & 0xFF, (px >> 8) & 0xFF, (px >> 16) & 0xFF], axis=-1).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(rgb.tobytes())
