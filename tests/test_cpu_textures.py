"""Packed texture storage (csrc/context.cpp pack_texture, csrc/k_trace.hip tex_texel), checked on the CPU:
the 8-bit textures (PPM / PNG, every channel b / 255.0f) are stored as RGBA8 and the Radiance environment map
(load_hdr: m * 2^(e - 136)) as RGBE, and both decode to the RGBA32F texels bit for bit, so every lookup is
unchanged. The device's byte decode is the reciprocal product with one fma correction, checked here for all
256 bytes. The GPU suite's bit-exact G-buffer and shading tests run over the packed textures."""
import ctypes as C

import numpy as np
import pytest

from helpers import ASSET_DIR, ASSETS_PRESENT, TEXTURE_MODE

f = np.float32
F32, UNORM8, RGBE = 0, 1, 2


def _unorm8_device(b):
    """k_trace.hip unorm8: r = b * fl(1/255); fma(fma(-r, 255, b), fl(1/255), r), each fma one rounding."""
    inv = f(f(1) / f(255))
    x = f(b)
    r = f(x * inv)
    e = f(np.float64(x) - np.float64(r) * 255.0)
    return f(np.float64(e) * np.float64(inv) + np.float64(r))


def test_unorm8_decode_is_exact_for_every_byte():
    for b in range(256):
        assert _unorm8_device(b) == f(f(b) / f(255)), b


def _decode(words, kind):
    w = np.asarray(words, np.uint32)
    ch = np.stack([(w >> (8 * c)) & 255 for c in range(4)], -1)
    if kind == UNORM8:
        return np.array([[_unorm8_device(int(b)) for b in t] for t in ch], np.float32)
    e = ch[:, 3].astype(np.int64)
    fct = np.where(e > 0, np.ldexp(np.float32(1), (e - 136).astype(np.int32)).astype(np.float32), np.float32(0))
    rgb = (ch[:, :3].astype(np.float32) * fct[:, None]).astype(np.float32)
    return np.concatenate([rgb, np.ones((len(w), 1), np.float32)], 1)


def _pack(lib, texels):
    t = np.ascontiguousarray(texels, np.float32).reshape(-1, 4)
    out = np.zeros(len(t), np.uint32)
    fn = lib.fr__pack_texture
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_uint32)]
    kind = fn(t.ctypes.data_as(C.POINTER(C.c_float)), len(t), out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return kind, out, t


def test_pack_kinds_and_round_trip(fovrt_mod):
    lib = fovrt_mod.load_library()
    rng = np.random.default_rng(2)
    b = rng.integers(0, 256, (500, 4))
    k, w, t = _pack(lib, (b.astype(np.float32) / f(255)).astype(np.float32))
    assert k == UNORM8 and np.array_equal(_decode(w, k), t)
    m = rng.integers(0, 256, (500, 3)).astype(np.float32)
    e = rng.integers(100, 160, 500)
    rgbe = np.concatenate([(m * np.ldexp(np.float32(1), e - 136)[:, None].astype(np.float32)).astype(np.float32),
                           np.ones((500, 1), np.float32)], 1)
    rgbe[0, :3] = 0
    k, w, t = _pack(lib, rgbe)
    assert k == RGBE and np.array_equal(_decode(w, k), t)
    k, _, _ = _pack(lib, rng.random((50, 4)).astype(np.float32))  # arbitrary floats stay RGBA32F
    assert k == F32


@pytest.mark.skipif(not ASSETS_PRESENT, reason="the reference's texture assets are not in assets/")
def test_scene_textures_pack(fovrt_mod):
    """bunny.PPM and grid.ppm pack as RGBA8, CedarCity.hdr as RGBE, and both round-trip bit for bit."""
    lib = fovrt_mod.load_library()
    a = fovrt_mod.Scene(fovrt_mod.Config(scene=fovrt_mod.SCENE_BUNNY, texture_mode=TEXTURE_MODE,
                                         asset_dir=ASSET_DIR, detail=1)).arrays()
    kinds = []
    for i, tex in enumerate(a["textures"]):
        k, w, t = _pack(lib, tex)
        kinds.append(k)
        if k != F32 and t.shape[0] <= 1 << 20:
            sel = np.random.default_rng(i).integers(0, len(t), 20000)
            assert np.array_equal(_decode(w[sel], k), t[sel]), i
    assert kinds[a["envmap"]] == RGBE
    assert kinds.count(UNORM8) >= 2
