"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product
package. See oracle/oracle.cpp for what is restated from which reference file, and for the parity
status (unpinned: the reference ships no outputs to pin against).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: the sanitizer build (oracle/Makefile asan, scripts/asan_cpu_suite.sh)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

_lib = None
F = C.POINTER(C.c_float)
U8 = C.POINTER(C.c_uint8)
U32 = C.POINTER(C.c_uint32)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.or_scene_create.restype = C.c_void_p
        L.or_scene_create.argtypes = [C.c_int, F, F, F, C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_int32), C.c_int,
                                      C.POINTER(C.c_int32), C.POINTER(F), C.c_int, F, F]
        L.or_scene_destroy.argtypes = [C.c_void_p]
        L.or_scene_params.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.or_scene_segments.restype = C.c_ulonglong
        L.or_scene_segments.argtypes = [C.c_void_p, C.c_int]
        L.or_closest.argtypes = [C.c_void_p, C.c_int, F, F, C.c_int]
        L.or_tea16.restype = C.c_uint32
        L.or_tea16.argtypes = [C.c_uint32, C.c_uint32]
        L.or_rnd_seq.argtypes = [C.c_uint32, C.c_int, F]
        L.or_tonemap.argtypes = [C.c_int, F, F]
        L.or_gbuffer.argtypes = [C.c_void_p, F, F, F, C.c_int, C.c_int, C.c_uint32, F, F, F, F, F]
        L.or_sampling.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, F, F, F, F, F, F, F, F, F, U8]
        L.or_warp_sort.restype = C.c_uint32
        L.or_warp_sort.argtypes = [C.c_int, C.c_int, U8, U32]
        L.or_shading.argtypes = [C.c_void_p, F, F, C.c_int, C.c_int, C.c_uint32, C.c_int, U8, F, F, F, F]
        L.or_jfa.argtypes = [C.c_int, C.c_int, F, F, F]
        L.or_sibson.argtypes = [C.c_int, C.c_int, F, F, F]
        L.or_pullpush.argtypes = [C.c_int, C.c_int, F, F, F, F]
        L.or_atrous.argtypes = [C.c_int, C.c_int, C.c_int, F, F, F, F]
        L.or_logpolar.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, F, F, F]
        L.or_ptx_site.restype = C.c_int
        L.or_ptx_site.argtypes = [C.c_int, C.c_int, F, F]
        _lib = L
    return _lib


def fp(a):
    return a.ctypes.data_as(F)


# or_ptx_site: site ids -> (input row width, output row width); the row layouts are oracle.cpp's
PTX_SITES = {"intersect": (0, 17, 7), "attributes": (1, 20, 8), "refine": (2, 13, 6), "camera0": (3, 23, 3),
             "camera3": (4, 26, 3), "faceforward": (5, 6, 1), "reproject": (6, 21, 2), "gbuffer_light": (7, 18, 6),
             "is_valid": (8, 7, 1), "gaze_dist": (9, 6, 1), "atanf": (10, 1, 1), "atan2f": (11, 2, 1),
             "acosf": (12, 1, 1), "sinf": (13, 1, 1), "cosf": (14, 1, 1), "hemisphere": (15, 2, 3), "onb": (16, 6, 3),
             "diffuse_light": (17, 20, 6), "refract": (18, 7, 5), "reflect": (19, 6, 3), "fresnel": (20, 3, 1),
             "luminance": (21, 3, 1), "tonemap_rational": (22, 1, 1), "envmap_uv": (23, 3, 2), "saliency": (24, 7, 1),
             "velocity_arg": (25, 4, 1), "velocity_sal": (26, 1, 1), "depth_sal": (27, 9, 2), "normal_enc": (28, 1, 1)}


def ptx_site(name, rows):
    """The oracle's own function at one PTX site (or_ptx_site) on the rows of `rows` (n x in-width)."""
    sid, ni, no = PTX_SITES[name]
    a = _c(rows, np.float32).reshape(-1, ni)
    out = np.zeros((a.shape[0], no), np.float32)
    rc = lib().or_ptx_site(sid, a.shape[0], fp(a), fp(out))
    assert rc == no, (name, rc)
    return out


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class OracleScene:
    """Wraps a scene dict (fovrt.Scene.arrays() / PathTracer.scene_arrays())."""

    def __init__(self, arrays: dict, refraction_max_depth=16, diffuse_max_depth=1):
        L = lib()
        self.a = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in arrays.items()}
        a = self.a
        self._keep = [_c(a["pos"], np.float32), _c(a["nrm"], np.float32), _c(a["uv"], np.float32),
                      _c(a["flags"], np.int32), _c(a["materials"], np.int32)]
        self._tex = [_c(t, np.float32) for t in a["textures"]]
        dims = np.array([[t.shape[1], t.shape[0]] for t in self._tex], np.int32)
        self._dims = dims
        ptrs = (F * len(self._tex))(*[fp(t) for t in self._tex])
        self._ptrs = ptrs
        self._light = _c(a["light"], np.float32)
        self._bbox = _c(a["bbox"], np.float32)
        pos, nrm, uv, flags, mats = self._keep
        self.h = L.or_scene_create(len(flags), fp(pos), fp(nrm), fp(uv), flags.ctypes.data_as(C.POINTER(C.c_int32)),
                                   len(mats), mats.ctypes.data_as(C.POINTER(C.c_int32)), len(self._tex),
                                   dims.ctypes.data_as(C.POINTER(C.c_int32)), ptrs, int(a["envmap"]), fp(self._light),
                                   fp(self._bbox))
        L.or_scene_params(self.h, int(refraction_max_depth), int(diffuse_max_depth))

    def set_params(self, refraction_max_depth, diffuse_max_depth):
        lib().or_scene_params(self.h, int(refraction_max_depth), int(diffuse_max_depth))

    def segments(self, reset=True):
        return int(lib().or_scene_segments(self.h, 1 if reset else 0))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_scene_destroy(self.h)
            self.h = None

    def closest(self, rays: np.ndarray, brute=False):
        rays = _c(rays, np.float32)
        out = np.empty((rays.shape[0], 4), np.float32)
        lib().or_closest(self.h, rays.shape[0], fp(rays), fp(out), 1 if brute else 0)
        return out


def tea16(a, b):
    return int(lib().or_tea16(a, b))


def rnd_seq(seed, n):
    out = np.empty(n, np.float32)
    lib().or_rnd_seq(seed, n, fp(out))
    return out


def tonemap(rgb):
    rgb = _c(rgb, np.float32).reshape(-1, 3)
    out = np.empty_like(rgb)
    lib().or_tonemap(rgb.shape[0], fp(rgb), fp(out))
    return out


def gbuffer(scene: OracleScene, cam, W, H, frame):
    out = [np.zeros((H, W, 4), np.float32) for _ in range(5)]
    inv_vp = _c(cam.inv_vp[:], np.float32)
    prev_vp = _c(cam.prev_vp[:], np.float32)
    eye = _c(cam.eye[:], np.float32)
    lib().or_gbuffer(scene.h, fp(inv_vp), fp(prev_vp), fp(eye), W, H, frame, *[fp(o) for o in out])
    return dict(zip(["position", "normal", "depth", "diffuse", "weight"], out))


def sampling(scene: OracleScene, cam, W, H, mask_mode, position, depth, depth_cache, weight, normal, diffuse):
    weight = _c(weight, np.float32).copy()
    extra = np.zeros((H, W, 4), np.float32)
    mask = np.zeros((H, W), np.uint8)
    gaze = _c(cam.gaze[:], np.float32)
    prev_eye = _c(cam.prev_eye[:], np.float32)
    args = [_c(x, np.float32) for x in (position, depth, depth_cache)]
    normal, diffuse = _c(normal, np.float32), _c(diffuse, np.float32)
    lib().or_sampling(scene.h, W, H, mask_mode, fp(gaze), fp(prev_eye), fp(args[0]), fp(args[1]), fp(args[2]),
                      fp(weight), fp(normal), fp(diffuse), fp(extra), mask.ctypes.data_as(U8))
    return {"weight": weight, "extra": extra, "mask": mask}


def warp_sort(mask):
    mask = _c(mask, np.uint8)
    H, W = mask.shape
    tb = np.zeros((H, W, 3), np.uint32)
    n = lib().or_warp_sort(W, H, mask.ctypes.data_as(U8), tb.ctypes.data_as(U32))
    return int(n), tb


def shading(scene: OracleScene, cam, W, H, frame, spp, mask, weight, history_cache):
    hb = np.zeros((H, W, 4), np.float32)
    sh = np.zeros((H, W, 4), np.float32)
    inv_vp = _c(cam.inv_vp[:], np.float32)
    eye = _c(cam.eye[:], np.float32)
    mask, weight, history_cache = _c(mask, np.uint8), _c(weight, np.float32), _c(history_cache, np.float32)
    lib().or_shading(scene.h, fp(inv_vp), fp(eye), W, H, frame, spp, mask.ctypes.data_as(U8), fp(weight),
                     fp(history_cache), fp(hb), fp(sh))
    return {"history": hb, "shading": sh}


def jfa(shading_img):
    s = _c(shading_img, np.float32)
    H, W = s.shape[:2]
    coord = np.empty_like(s)
    color = np.empty_like(s)
    lib().or_jfa(W, H, fp(s), fp(coord), fp(color))
    return coord, color


def sibson(coord, color):
    coord, color = _c(coord, np.float32), _c(color, np.float32)
    H, W = coord.shape[:2]
    out = np.empty_like(coord)
    lib().or_sibson(W, H, fp(coord), fp(color), fp(out))
    return out


class PullPushState:
    """The two persistent 1.5S x S atlases of PullPushInterpolation (push carries across frames)."""

    def __init__(self, W, H):
        S = 1
        while S < W or S < H:
            S *= 2
        self.W, self.H, self.S = W, H, S
        self.pull = np.zeros((S, S + S // 2, 4), np.float32)
        self.push = np.zeros((S, S + S // 2, 4), np.float32)

    def render(self, shading_img):
        s = _c(shading_img, np.float32)
        out = np.empty((self.H, self.W, 4), np.float32)
        lib().or_pullpush(self.W, self.H, fp(s), fp(self.pull), fp(self.push), fp(out))
        return out


def atrous(count, pos, nrm, col):
    pos, nrm, col = _c(pos, np.float32), _c(nrm, np.float32), _c(col, np.float32)
    H, W = pos.shape[:2]
    out = np.empty_like(col)
    lib().or_atrous(W, H, count, fp(pos), fp(nrm), fp(col), fp(out))
    return out


def logpolar(img, gaze, fwd=None, inv=None):
    """LogPolarTransform::render of img around gaze = (x, y) (kernel coordinates); fwd / inv are the
    persistent output textures (zeros if None). Returns (fwd, inv)."""
    img = _c(img, np.float32)
    H, W = img.shape[:2]
    fwd = np.zeros((H, W, 4), np.float32) if fwd is None else _c(fwd, np.float32).copy()
    inv = np.zeros((H, W, 4), np.float32) if inv is None else _c(inv, np.float32).copy()
    lib().or_logpolar(W, H, float(gaze[0]), float(gaze[1]), fp(img), fp(fwd), fp(inv))
    return fwd, inv
