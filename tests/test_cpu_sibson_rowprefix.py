"""k_sibson_rowp's whole-row prefix sums (csrc/k_image.hip), restated in numpy float32, against float64 sums.

k_sibson_strip sums a row's run as G[e] - G[s] with G = P + the row's block totals before it (k_jfa_final_prefix:
P is the 64-column block-local exclusive prefix, T the block totals, both fp32 warp scans). Those sums carry an
ulp of the row's running total rather than of a block's, which the strip kernel accepts because it only takes
discs of more than 2 x 64 rows (SIBS_HALF), whose average divides the error by thousands of taps. This checks
that claim on the colour range the path tracer produces (tone-mapped, HDR-ish up to 8): the averages of such
discs stay within 1e-5 of the float64 average, against the Sibson parity tolerance of 4e-3."""
import numpy as np

f = np.float32


def _block_scan(row):
    """P and T of one row as k_jfa_final_prefix forms them: per 64-column block, a Hillis-Steele inclusive
    scan in fp32 (shuffle-up by 1, 2, 4, ... 32), P = inclusive - value (exclusive), T = the block's total."""
    W = row.shape[0]
    NB = (W + 1 + 63) // 64
    P = np.zeros((NB * 64, 3), f)
    T = np.zeros((NB, 3), f)
    v = np.zeros((NB * 64, 3), f)
    v[:W] = row
    for B in range(NB):
        x = v[B * 64:(B + 1) * 64].copy()
        incl = x.copy()
        o = 1
        while o < 64:
            sh = np.zeros_like(incl)
            sh[o:] = incl[:-o]
            incl = (incl + sh).astype(f)
            o *= 2
        P[B * 64:(B + 1) * 64] = (incl - x).astype(f)
        T[B] = incl[63]
    return P[:W + 1], T


def _row_prefix(P, T):
    """k_sibson_rowp: the exclusive prefix of the block totals (64 at a time, carried), added to P."""
    NB = T.shape[0]
    tt = np.zeros((NB, 3), f)
    carry = np.zeros(3, f)
    for B0 in range(0, NB, 64):
        x = T[B0:B0 + 64]
        incl = x.copy()
        o = 1
        while o < len(x):
            sh = np.zeros_like(incl)
            sh[o:] = incl[:-o]
            incl = (incl + sh).astype(f)
            o *= 2
        tt[B0:B0 + len(x)] = (carry + (incl - x)).astype(f)
        carry = (carry + incl[-1]).astype(f)
    cols = np.arange(P.shape[0]) >> 6
    return (P + tt[cols]).astype(f)


def test_whole_row_prefix_big_disc_average():
    rng = np.random.default_rng(3)
    W = 3840
    rows = 260  # a disc of more than 2 x SIBS_HALF rows
    img = (rng.random((rows, W, 3)) ** 3 * 8.0).astype(f)  # mostly dark, a few bright texels (tone-mapped HDR)
    worst = 0.0
    for trial in range(20):
        cx = int(rng.integers(300, W - 300))
        half = int(rng.integers(64, 280))
        acc32 = np.zeros(3, np.float64)
        acc64 = np.zeros(3, np.float64)
        n = 0
        for j in range(rows):
            P, T = _block_scan(img[j])
            G = _row_prefix(P, T)
            dy = (j - rows / 2) / (rows / 2)
            c = int(half * np.sqrt(max(0.0, 1.0 - dy * dy)))
            s, e = max(cx - c, 0), min(cx + c + 1, W)
            if e <= s:
                continue
            acc32 += (G[e] - G[s]).astype(f)
            acc64 += img[j, s:e].astype(np.float64).sum(axis=0)
            n += e - s
        err = np.abs(acc32 / n - acc64 / n).max()
        worst = max(worst, err)
        assert err < 1e-5, (trial, err)
    assert worst > 0.0  # the restatement is not trivially exact


def test_row_prefix_equals_block_form_within_row_total_ulps():
    """G[e] - G[s] against the block form P[e] - P[s] + the block totals between, per run: they differ by
    rounding only, at most a few ulps of the row total."""
    rng = np.random.default_rng(4)
    W = 3840
    row = (rng.random((W, 3)) * 4.0).astype(f)
    P, T = _block_scan(row)
    G = _row_prefix(P, T)
    total = float(row.astype(np.float64).sum(axis=0).max())
    for _ in range(500):
        s = int(rng.integers(0, W - 1))
        e = int(rng.integers(s + 1, W + 1))
        blk = (P[e] - P[s]).astype(f)
        for B in range(s >> 6, e >> 6):
            blk = (blk + T[B]).astype(f)
        d = np.abs((G[e] - G[s]).astype(np.float64) - blk.astype(np.float64)).max()
        assert d <= 8 * np.spacing(f(total)), (s, e, d)
