"""The closed-form row run of k_sibson_runs (csrc/k_image.hip, sib_rows_setup / sib_row_run), restated in numpy
float32 and checked against a brute-force walk of the reference's taps (sibsonFS.glsl:26-45: w from min_box.x in
steps of 1/W, tap inside when dx^2 + dy^2 <= the bound of d) on the CPU.

sib_row_run trusts that its fp32 chord estimate puts each end of a row's run within one tap of the true end and
settles each end with two exact tests, with no walk. The estimate is worst on the disc's top and bottom rows,
where r2max - dy2 cancels. This test walks every row of discs of 0.5 to 700 pixels at 1080p and 4K and checks the
settled run against the brute force, with the hardware's approximate sqrt and reciprocal modelled as the correctly
rounded values moved by up to two ulps either way (v_sqrt_f32 and v_rcp_f32 are within one ulp)."""
import numpy as np

f = np.float32


def _ulp_moves(x, n=2):
    out = [f(x)]
    lo = hi = f(x)
    for _ in range(n):
        lo = np.nextafter(lo, f(-np.inf), dtype=np.float32)
        hi = np.nextafter(hi, f(np.inf), dtype=np.float32)
        out += [lo, hi]
    return out


def _sqrt_le_bound(s):
    if s == 0:
        return f(0)
    up = np.nextafter(f(s), f(np.inf), dtype=np.float32)
    m = np.float64(s) + 0.5 * (np.float64(up) - np.float64(s))
    U = m * m
    u = f(U)
    if np.float64(u) >= U:
        u = np.nextafter(u, f(-np.inf), dtype=np.float32)
    return u


def _setup(fx, w0, wmax, inc):
    """sib_rows_setup: None when the pixel has no closed form."""
    if not (w0 > 0) or not (wmax < 1):
        return None
    if (w0.view(np.uint32) >> 23) != (wmax.view(np.uint32) >> 23):
        return None
    w1 = f(w0 + inc)
    delta = f(w1 - w0)
    if f(f(w1 + inc) - w1) != delta:
        return None
    wk = lambda k: f(np.float64(k) * np.float64(delta) + np.float64(w0))  # fma, one rounding
    inv = f(f(1) / delta)
    K = max(int(np.ceil(f(f(wmax - w0) * inv))), 0)
    while wk(K) < wmax:
        K += 1
    while K > 0 and not (wk(K - 1) < wmax):
        K -= 1
    if K == 0:
        return dict(K=0)
    kc = min(max(int(np.floor(f(f(fx - w0) * inv))), 0), K - 1)
    best, kbest = np.inf, 0
    for k in range(max(kc - 1, 0), min(kc + 2, K - 1) + 1):
        dx = f(fx - wk(k))
        if f(dx * dx) < best:
            best, kbest = f(dx * dx), k
    return dict(K=K, kbest=kbest, delta=delta, w0=w0, inv=inv, wk=wk)


def _row_runs(r, fx, dy2s, r2max, inv, sqrt_move):
    """sib_row_run for every row at once; returns (has, k0, k1)."""
    K, kb, w0 = r["K"], r["kbest"], r["w0"]
    ks = np.arange(K)
    wks = (ks.astype(np.float64) * np.float64(r["delta"]) + np.float64(w0)).astype(np.float32)
    dxs = (f(fx) - wks).astype(np.float32)
    dx2 = (dxs * dxs).astype(np.float32)

    def inside(k, dy2):
        k = np.clip(k, 0, K - 1)
        return (dx2[k] + dy2).astype(np.float32) <= r2max

    has = inside(np.full(dy2s.shape, kb), dy2s)
    chord = np.sqrt(np.maximum((r2max - dy2s).astype(np.float32), f(0))).astype(np.float32)
    chord = np.array([_ulp_moves(c, 2)[sqrt_move] for c in chord], np.float32)
    c = f(fx - w0)
    a = np.minimum(np.maximum(np.ceil(((c - chord).astype(np.float32) * inv).astype(np.float32)), 0), kb).astype(int)
    b = np.maximum(np.minimum(np.floor(((c + chord).astype(np.float32) * inv).astype(np.float32)), K - 1), kb).astype(int)
    k0 = np.where((a > 0) & inside(a - 1, dy2s), a - 1, np.where(inside(a, dy2s), a, a + 1))
    k1 = np.where((b < K - 1) & inside(b + 1, dy2s), b + 1, np.where(inside(b, dy2s), b, b - 1))
    return has, k0, k1, dx2


def test_row_run_estimate_settles_every_row():
    rng = np.random.default_rng(7)
    checked = 0
    for trial in range(400):
        W, H = [(1920, 1080), (3840, 2160)][trial % 2]
        x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
        # a seed texel at a random offset: d = distance of two texel centres, as k_sibson_runs forms it
        rad = [0.5, 1.5, 3, 8, 24, 90, 300, 700][trial % 8] * (0.7 + 0.6 * rng.random())
        ang = rng.random() * 2 * np.pi
        sx = int(np.clip(round(x + rad * np.cos(ang)), 0, W - 1))
        sy = int(np.clip(round(y + rad * np.sin(ang)), 0, H - 1))
        fx, fy = f(f(f(x) + f(0.5)) / f(W)), f(f(f(y) + f(0.5)) / f(H))
        cx, cy = f(f(f(sx) + f(0.5)) / f(W)), f(f(f(sy) + f(0.5)) / f(H))
        cdx, cdy = f(cx - fx), f(cy - fy)
        d = np.sqrt(f(f(cdx * cdx) + f(cdy * cdy))).astype(np.float32)
        if d == 0:
            continue
        inc_x, inc_y = f(f(1) / f(W)), f(f(1) / f(H))
        r = _setup(fx, f(fx - d), f(fx + d), inc_x)
        if r is None or r["K"] == 0:
            continue
        r2max = _sqrt_le_bound(d)
        hs, h = [], f(fy - d)
        while h < f(fy + d):
            hs.append(h)
            h = f(h + inc_y)
        dy = (f(fy) - np.array(hs, np.float32)).astype(np.float32)
        dy2s = (dy * dy).astype(np.float32)
        for inv in _ulp_moves(r["inv"], 2):
            for sm in range(5):
                has, k0, k1, dx2 = _row_runs(r, fx, dy2s, r2max, inv, sm)
                ins = ((dx2[None, :] + dy2s[:, None]).astype(np.float32) <= r2max)
                assert np.array_equal(has, ins.any(axis=1)), (W, x, y, float(d))
                for j in np.nonzero(has)[0]:
                    idx = np.nonzero(ins[j])[0]
                    # the run is contiguous, and the settled ends are its ends
                    assert idx[-1] - idx[0] + 1 == idx.size
                    assert (k0[j], k1[j]) == (idx[0], idx[-1]), (W, x, y, float(d), int(j), int(sm))
                    checked += 1
    assert checked > 10000
