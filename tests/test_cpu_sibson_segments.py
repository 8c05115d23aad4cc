"""The exactness argument of k_sibson_wide's tap tables (csrc/k_image.hip, sib_axis_build), restated in numpy
float32 and checked on the CPU: the reference's positions v_{k+1} = fl(v_k + 1/W) from min_box while v < max_box
(sibsonFS.glsl:30-31) equal the segment table's v_s + (k - k_s) delta for every tap, over random boxes that
cross binade edges, zero and the image border. The GPU tests check the kernel itself against the oracle."""
import struct

import numpy as np

f = np.float32


def _bits(x):
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def _from_bits(b):
    return f(struct.unpack("<f", struct.pack("<I", b & 0xFFFFFFFF))[0])


def _fma(j, d, v):  # exact here: the product and sum fit in f64, one rounding to f32
    return f(np.float64(j) * np.float64(d) + np.float64(v))


def _same_binade(a, b):
    return (_bits(a) >> 23) == (_bits(b) >> 23)


def _binade_steps(v, d):
    b = _bits(v)
    edge = _from_bits(((b >> 23) + 1) << 23) if v > 0 else _from_bits(b & 0xFF800000)
    m = int(min(max(np.floor(f(f(edge - v) / d)), 0), 1e8))
    while m > 0 and not _same_binade(_fma(m, d, v), v):
        m -= 1
    while _same_binade(_fma(m + 1, d, v), v):
        m += 1
    return m


def _count_below(v, d, lim):
    j = int(min(max(np.ceil(f(f(lim - v) / d)), 1), 1e8))
    while j > 1 and not (_fma(j - 1, d, v) < lim):
        j -= 1
    while _fma(j, d, v) < lim:
        j += 1
    return j


def _build(v0, vmax, inc):
    k, segs, v = 0, [], v0
    while v < vmax:
        v1 = f(v + inc)
        v2 = f(v1 + inc)
        delta = f(v1 - v)
        m = 0
        if v != 0 and _same_binade(v, v2) and f(v2 - v1) == delta and delta > 0:
            m = min(_binade_steps(v, delta), _count_below(v, delta, vmax) - 1)
            if m >= 1 and f(_fma(m - 1, delta, v) + inc) != _fma(m, delta, v):
                m -= 1
        segs.append((k, v, delta))
        k += m + 1
        v = f(_fma(m, delta, v) + inc)
    return segs, k


def _sequence(v0, vmax, inc):
    out, v = [], v0
    while v < vmax:
        out.append(v)
        v = f(v + inc)
    return out


def test_tap_tables_equal_the_shader_sequence():
    rng = np.random.default_rng(1)
    most = 0
    for trial in range(400):
        W = int(rng.choice([61, 97, 130, 144, 160, 256, 1080, 1920, 2160, 3000, 3840, 4096]))
        x = int(rng.integers(0, W))
        fx = f(f(f(x) + f(0.5)) / f(W))
        d = f(rng.random() * (0.6 if trial % 2 else 0.05))
        inc = f(f(1) / f(W))
        segs, K = _build(f(fx - d), f(fx + d), inc)
        ref = _sequence(f(fx - d), f(fx + d), inc)
        assert K == len(ref)
        ks = [s[0] for s in segs] + [K]
        for s, (k0, v, dl) in enumerate(segs):
            for k in range(k0, ks[s + 1]):
                assert _fma(k - k0, dl, v) == ref[k], (W, x, float(d), k)
        most = max(most, len(segs))
    assert most <= 64  # SIBW_SEGS
