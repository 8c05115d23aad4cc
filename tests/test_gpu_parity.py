"""GPU parity suite: every hot-path stage of libfovrt (HIP, gfx950) against the CPU oracle.

Integer / index work and the fp32 image passes that contain no transcendental are held to bit
equality; stages whose arithmetic goes through the platform fp32 libm (the materials' powf/cosf
..., A-Trous expf) are held to the north-star tolerance (per-channel RMSE <= 1e-3) plus a tighter
max-error bound. Each stage is fed the GPU's own upstream buffers, so a tolerance in one stage
never leaks into the next stage's comparison.
"""
import copy

import numpy as np
import pytest

from helpers import (GOLDEN, TEXTURE_MODE, ASSET_DIR, PullPushNp, _gl_linear_repeat, atrous_np, equal_nan,
                     logpolar_mask_np, rmse_per_channel, sparse_image)

pytestmark = pytest.mark.gpu

TN = None


@pytest.fixture(scope="module", autouse=True)
def _tn(fovrt_mod):
    global TN
    TN = fovrt_mod.TextureName


def make_tracer(fovrt, W, H, scene=1, mask=1, spp=1, dmd=1, refr=16, **kw):
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=scene, mask_mode=mask, spp=spp,
                                      diffuse_max_depth=dmd, refraction_max_depth=refr,
                                      texture_mode=TEXTURE_MODE, asset_dir=ASSET_DIR, **kw))
    assert t.initialize()
    return t


def ref_gaze(H, xpos, ypos, fullscreen=False):
    """The gaze the kernels see after cursorPosCallback (FR/gui.cpp:48-66): g_gaze = (LONG(xpos),
    LONG(ypos * adjust_scale)) with adjust_scale 1.25 in a window, 1 in full screen, then
    (g_gaze.x, H - g_gaze.y) (FR/PathTracer.cpp:795)."""
    gx = int(np.trunc(xpos))
    gy = int(np.trunc(ypos * (1.0 if fullscreen else 1.25)))
    return np.float32(gx), np.float32(H - gy)


def mismatch_report(a, b):
    bad = ~np.isclose(a, b, rtol=0, atol=0, equal_nan=True)
    if not bad.any():
        return "equal"
    idx = np.argwhere(bad)[:5]
    return f"{bad.sum()} of {bad.size} differ; first {idx.tolist()}: gpu {a[tuple(idx[0])]} oracle {b[tuple(idx[0])]}"


# ---------------------------------------------------------------------------------------------
# entry 0 — G-buffer (bit-exact)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene,W,H", [(0, 96, 64), (1, 96, 64), (2, 96, 64), (1, 100, 70)])
def test_gbuffer_bit_exact(fovrt_mod, oracle, scene, W, H):
    t = make_tracer(fovrt_mod, W, H, scene=scene)
    uni = fovrt_mod.Camera.preset(scene, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    t.geometry_launch()
    osc = oracle.OracleScene(t.scene_arrays())
    ref = oracle.gbuffer(osc, uni, W, H, 0)
    for name, tid in [("position", TN.POSITION), ("normal", TN.NORMAL), ("depth", TN.DEPTH),
                      ("diffuse", TN.DIFFUSE), ("weight", TN.WEIGHT)]:
        got = t.read(tid)
        assert equal_nan(got, ref[name]), (name, mismatch_report(got, ref[name]))
    assert t.stats()["gbuffer_primary"] == W * H


# ---------------------------------------------------------------------------------------------
# entries 1 + 2 — sampling mask (bit-exact), compaction / ray_count (bit-exact)
# ---------------------------------------------------------------------------------------------
# (W, H) = (100, 70): partial 16x16 blocks in k_sampling, the ballot publication and k_scatter, as
# at 1920x1080 (BASELINE configs[1]). gaze_window: a cursor (window coordinates, y down) passed to
# set_gaze: on the top edge (gaze.y = H) and off the window (k_sampling clamps its focal-depth read).
SAMPLING_CASES = ([(scene, m, 128, 96, None) for scene in (1, 2) for m in (0, 1, 2, 3, 4)]
                  + [(1, m, 100, 70, None) for m in (0, 4)]
                  # W % 16 == 0 with a partial last block row: k_sampling's 16-byte mask rows, the rows below H skipped
                  + [(1, m, 160, 72, None) for m in (0, 4)]
                  + [(2, 0, 100, 70, (50.0, 0.0)), (2, 0, 128, 96, (-30.0, 500.0)), (1, 4, 100, 70, (99.5, 0.0)),
                     (1, 0, 128, 96, (1e6, -1e6))]
                  # fractional cursors (glfw reports doubles, FR/gui.cpp:48-66): inexact gaze_dist products,
                  # the fma.rn sites of samplingStep.ptx decide the ring and isValid pixels
                  + [(1, 0, 128, 96, (37.3, 41.7)), (2, 4, 128, 96, (70.6, 52.35)), (2, 1, 100, 70, (33.33, 20.9)),
                     (1, 2, 128, 96, (90.17, 13.71))])


@pytest.mark.parametrize("mask_mode", [0, 1, 2, 3, 4])
def test_sampling_without_extra_bit_exact(fovrt_mod, oracle, mask_mode):
    """write_extra = 0: k_sampling skips the saliency features unless the saliency mask reads them; the
    mask and WEIGHT stay the oracle's, and EXTRA is left untouched."""
    W, H = 100, 70
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=mask_mode, write_extra=0)
    uni = fovrt_mod.Camera.preset(1, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    osc = oracle.OracleScene(t.scene_arrays())
    before = t.read(TN.EXTRA)
    for frame in range(2):
        t.geometry_launch()
        inp = [t.read(v) for v in (TN.POSITION, TN.DEPTH, TN.DEPTH_CACHE, TN.WEIGHT, TN.NORMAL, TN.DIFFUSE)]
        t.sampling_launch()
        ref = oracle.sampling(osc, uni, W, H, mask_mode, *inp)
        assert np.array_equal(t.read(TN.MASK), ref["mask"]), (frame, mismatch_report(t.read(TN.MASK), ref["mask"]))
        assert equal_nan(t.read(TN.WEIGHT), ref["weight"]), frame
        t.optimize_launch()
        t.shading_launch()
    assert equal_nan(t.read(TN.EXTRA), before)


@pytest.mark.parametrize("scene,mask_mode,W,H,gaze_window", SAMPLING_CASES)
def test_sampling_and_compaction_bit_exact(fovrt_mod, oracle, scene, mask_mode, W, H, gaze_window):
    t = make_tracer(fovrt_mod, W, H, scene=scene, mask=mask_mode)
    uni = fovrt_mod.Camera.preset(scene, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    if gaze_window is not None:
        t.set_gaze(*gaze_window)
        uni.gaze[0], uni.gaze[1] = ref_gaze(H, *gaze_window)
    osc = oracle.OracleScene(t.scene_arrays())
    for frame in range(2):  # frame 1 has a valid depth cache -> isValid / reprojection paths
        t.geometry_launch()
        inp = {k: t.read(v) for k, v in [("position", TN.POSITION), ("depth", TN.DEPTH), ("depth_cache", TN.DEPTH_CACHE),
                                         ("weight", TN.WEIGHT), ("normal", TN.NORMAL), ("diffuse", TN.DIFFUSE)]}
        t.sampling_launch()
        ref = oracle.sampling(osc, uni, W, H, mask_mode, inp["position"], inp["depth"], inp["depth_cache"],
                              inp["weight"], inp["normal"], inp["diffuse"])
        mask = t.read(TN.MASK)
        assert np.array_equal(mask, ref["mask"]), mismatch_report(mask, ref["mask"])
        assert equal_nan(t.read(TN.WEIGHT), ref["weight"])
        assert equal_nan(t.read(TN.EXTRA), ref["extra"]), mismatch_report(t.read(TN.EXTRA), ref["extra"])
        t.optimize_launch()
        n = t.ray_count()
        n_ref, _ = oracle.warp_sort(mask)
        assert n == n_ref == int(mask.sum())
        lst = t.read(TN.THREAD)[:n]
        assert np.array_equal(np.sort(lst), np.flatnonzero(mask.reshape(-1)))
        t.shading_launch()
    if mask_mode in (1, 4):
        assert np.array_equal(mask, logpolar_mask_np(W, H, uni.gaze[0], uni.gaze[1], signed=mask_mode == 4))
    if gaze_window is not None:  # the gaze-target read-back clamps to the screen like the focal-depth read
        gx = min(max(int(np.float32(uni.gaze[0])), 0), W - 1) if uni.gaze[0] > 0 else 0
        gy = min(max(int(np.float32(uni.gaze[1])), 0), H - 1) if uni.gaze[1] > 0 else 0
        assert np.array_equal(np.float32(t.gaze_target()), t.read(TN.POSITION)[gy, gx, :3])


# ---------------------------------------------------------------------------------------------
# entry 3 — foveated shading (north-star tolerance: per-channel RMSE <= 1e-3)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene,spp,dmd,mask_mode,W,H", [(0, 1, 1, 3, 64, 48), (1, 1, 1, 1, 64, 48), (1, 4, 3, 1, 64, 48),
                                                         (1, 4, 3, 3, 64, 48), (2, 2, 3, 0, 64, 48), (2, 8, 1, 1, 64, 48),
                                                         (1, 4, 3, 4, 100, 70)])
def test_shading_within_tolerance(fovrt_mod, oracle, scene, spp, dmd, mask_mode, W, H):
    t = make_tracer(fovrt_mod, W, H, scene=scene, mask=mask_mode, spp=spp, dmd=dmd)
    uni = fovrt_mod.Camera.preset(scene, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    osc = oracle.OracleScene(t.scene_arrays(), refraction_max_depth=16, diffuse_max_depth=dmd)
    for _ in range(3):
        frame = t.m_accumFrame
        t.geometry_launch()
        t.sampling_launch()
        t.optimize_launch()
        mask, weight, hist_in = t.read(TN.MASK), t.read(TN.WEIGHT), t.read(TN.HISTORY_CACHE)
        gcls = t.read(TN.GCLASS)
        t.shading_launch()
        got_sh, got_hist = t.read(TN.SHADING), t.read(TN.HISTORY_CACHE)  # swapped: cache = just written
        ref = oracle.shading(osc, uni, W, H, frame, spp, mask, weight, hist_in)
        rm = rmse_per_channel(got_sh, ref["shading"])
        assert (rm <= 1e-3).all(), (frame, rm, mismatch_report(got_sh, ref["shading"]))
        assert np.abs(np.nan_to_num(got_sh - ref["shading"], nan=1.0)).max() < 5e-2
        exact = np.mean(np.all(got_sh == ref["shading"], axis=-1))
        assert exact > 0.5, exact
        # per primary-hit class of the traced pixels: each class's RMSE on its own, so a
        # systematic error confined to one class (the refraction trees) cannot hide behind the others; misses
        # differ only by the platform libm in the environment lookup
        for c in range(4):
            sel = (mask == 1) & (gcls == c)
            if sel.sum() < 16:
                continue
            d = np.nan_to_num(got_sh[sel] - ref["shading"][sel], nan=1.0)
            crm = np.sqrt(np.mean(d[:, :3] ** 2, 0))
            assert (crm <= 1e-3).all(), (frame, c, crm)
            if c == 3:
                assert np.abs(d).max() <= 2e-3, (frame, np.abs(d).max())
        # inactive pixels carry history exactly; alpha is exactly 0 or 1 (App. A #14)
        inactive = mask == 0
        assert equal_nan(got_hist[inactive], ref["history"][inactive])
        assert set(np.unique(got_sh[..., 3]).tolist()) <= {0.0, 1.0}
    st = t.stats()
    assert st["overflow"] == 0 and st["primary"] > 0


@pytest.mark.parametrize("kind", ["empty", "last_pixel", "full", "one_row"])
def test_shading_host_mask_edge_cases(fovrt_mod, oracle, kind):
    """Entry 3 on a host-written mask (fr_write_buffer rebuilds the wave ballots): no active pixel (an empty
    megakernel launch: every pixel carries its history), the last pixel alone (one partial wave, the end of
    the active list), every pixel (the largest launch of the size) and one ragged row; two frames each, so
    the second reprojects the first one's history. Against the oracle at the north-star tolerance."""
    W, H, spp = 64, 48, 4
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=spp, dmd=3)
    uni = fovrt_mod.Camera.preset(1, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    osc = oracle.OracleScene(t.scene_arrays(), refraction_max_depth=16, diffuse_max_depth=3)
    m = np.zeros((H, W), np.uint8)
    if kind == "last_pixel":
        m[H - 1, W - 1] = 1
    elif kind == "full":
        m[:] = 1
    elif kind == "one_row":
        m[H // 2, 3:W - 5] = 1
    for _ in range(2):
        frame = t.m_accumFrame
        t.geometry_launch()
        t.sampling_launch()
        t.write(TN.MASK, m)
        t.optimize_launch()
        assert t.ray_count() == int(m.sum())
        weight, hist_in = t.read(TN.WEIGHT), t.read(TN.HISTORY_CACHE)
        t.shading_launch()
        got = t.read(TN.SHADING)
        ref = oracle.shading(osc, uni, W, H, frame, spp, m, weight, hist_in)
        rm = rmse_per_channel(got, ref["shading"])
        assert (rm <= 1e-3).all(), (kind, frame, rm, mismatch_report(got, ref["shading"]))
        inactive = m == 0
        assert equal_nan(t.read(TN.HISTORY_CACHE)[inactive], ref["history"][inactive])
    st = t.stats()
    assert st["overflow"] == 0 and (st["primary"] > 0) == (kind != "empty")


@pytest.mark.parametrize("refr", [0, 1, 3])
def test_shading_refraction_depth_cap(fovrt_mod, oracle, refr):
    """Glass bunny with the refraction recursion cut short (fr_config.refraction_max_depth): the
    truncation path and refraction nodes that keep one child or none, against the oracle at the same cap."""
    W, H, spp = 64, 48, 4
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=3, spp=spp, dmd=3, refr=refr)
    uni = fovrt_mod.Camera.preset(1, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    osc = oracle.OracleScene(t.scene_arrays(), refraction_max_depth=refr, diffuse_max_depth=3)
    frame = t.m_accumFrame
    t.geometry_launch(); t.sampling_launch(); t.optimize_launch()
    mask, weight, hist_in = t.read(TN.MASK), t.read(TN.WEIGHT), t.read(TN.HISTORY_CACHE)
    t.shading_launch()
    got = t.read(TN.SHADING)
    ref = oracle.shading(osc, uni, W, H, frame, spp, mask, weight, hist_in)
    rm = rmse_per_channel(got, ref["shading"])
    assert (rm <= 1e-3).all(), (rm, mismatch_report(got, ref["shading"]))
    st = t.stats()
    assert st["truncated"] > 0 and st["overflow"] == 0
    if refr == 0:
        assert st["refraction"] == 0 and st["reflection"] == 0


# ---------------------------------------------------------------------------------------------
# JumpFlooding / Sibson / PullPush — bit-exact; A-Trous — tolerance
# ---------------------------------------------------------------------------------------------
def _box_tracer(fovrt_mod, W, H):
    return make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=1)


# Sibson run form (sibson_mode 0) against the per-tap form: the taps are the same; a run uses its
# first tap's 8-bit GL_LINEAR weight for all its taps, and the f32 tap positions of the per-tap form
# put a weight on the other side of a 1/256 rounding step on a few taps of some rows (the position
# noise is ~1e-4 texel). One flipped step moves a tap by (1/256) |c1 - c0|, so a pixel's colour by
# at most 1/256 of a colour difference spread over its taps. Measured at 1080p (10 % log-polar):
# RMSE 1.35e-5, 99th percentile 1.1e-4, max 6.2e-4. The reference's texture unit rounds its own
# fixed-point positions, so it is not pinned at this level either.
SIB_RUN_MAX = 4e-3     # one 1/256 weight step of a full colour difference
SIB_RUN_RMSE = 5e-5    # per channel; the north-star image tolerance is 1e-3

JFA_CASES = [(64, 48, "logpolar"), (512, 512, "logpolar"), (1920, 1080, "logpolar"), (33, 17, 0.1),
             (40, 40, 0.0), (40, 40, 1.0), (1, 1, 1.0), (7, 5, "single"), (256, 64, 0.003)]


def _mask(W, H, kind, rng):
    if kind == "logpolar":
        return logpolar_mask_np(W, H, W // 2, H - H // 2)
    if kind == "single":
        m = np.zeros((H, W), np.uint8)
        m[H // 3, W - 1] = 1
        return m
    return (rng.random((H, W)) < kind).astype(np.uint8)


@pytest.mark.parametrize("W,H,kind", JFA_CASES)
def test_jfa_and_sibson_bit_exact(fovrt_mod, oracle, W, H, kind):
    rng = np.random.default_rng(W * 131 + H)
    img = sparse_image(W, H, _mask(W, H, kind, rng), seed=W + H)
    t = _box_tracer(fovrt_mod, W, H)
    t.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(t).render(TN.SHADING)
    coord, color = t.read(TN.JFA_COORD), t.read(TN.JFA_COLOR)
    rc, rcol = oracle.jfa(img)
    assert equal_nan(coord, rc), mismatch_report(coord, rc)
    assert equal_nan(color, rcol), mismatch_report(color, rcol)
    if W * H <= 512 * 512:
        rs = oracle.sibson(rc, rcol)
        # sibson_mode 1: per tap, the shader's order -> bit-exact
        fovrt_mod.SibsonInterpolation(t).render()
        si = t.read(TN.SIBSON)
        assert equal_nan(si, rs), mismatch_report(si, rs)
        # sibson_mode 0 (default): run form over prefix sums -> the same taps, rounding-level differences
        tf = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
        tf.write(TN.JFA_COORD, coord)
        tf.write(TN.JFA_COLOR, color)
        fovrt_mod.SibsonInterpolation(tf).render()
        sf = tf.read(TN.SIBSON)
        assert np.isfinite(sf).all() and np.array_equal(sf[..., 3], rs[..., 3])
        assert np.abs(sf - rs).max() <= SIB_RUN_MAX, np.abs(sf - rs).max()
        assert (rmse_per_channel(sf, rs) <= SIB_RUN_RMSE).all(), rmse_per_channel(sf, rs)


@pytest.mark.parametrize("W,H", [(1920, 1080), (3840, 2160)])
def test_sibson_run_form_full_size(fovrt_mod, W, H):
    """BASELINE sizes (the oracle's per-tap Sibson takes minutes there): the default run form against
    the per-tap form (bit-exact with the oracle at every size the suite runs it) on the same JFA output
    of a 10 % log-polar image: same tap sets (alpha, coverage), rounding-level colour differences."""
    mask = logpolar_mask_np(W, H, W // 2, H - H // 2, signed=True)
    img = sparse_image(W, H, mask, seed=3)
    ex = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=1)
    ru = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
    ex.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(ex).render(TN.SHADING)
    fovrt_mod.SibsonInterpolation(ex).render()
    ru.write(TN.JFA_COORD, ex.read(TN.JFA_COORD))
    ru.write(TN.JFA_COLOR, ex.read(TN.JFA_COLOR))
    fovrt_mod.SibsonInterpolation(ru).render()
    a, b = ex.read(TN.SIBSON), ru.read(TN.SIBSON)
    assert np.isfinite(b).all() and np.array_equal(a[..., 3], b[..., 3])
    assert np.abs(a - b).max() <= SIB_RUN_MAX, np.abs(a - b).max()
    assert (rmse_per_channel(a, b) <= SIB_RUN_RMSE).all(), rmse_per_channel(a, b)


def _jfa_then_run_form(fovrt_mod, img, W, H):
    """JFA on the image (per-tap context), then the default run-form Sibson on its output."""
    ex = _box_tracer(fovrt_mod, W, H)
    ex.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(ex).render(TN.SHADING)
    coord, color = ex.read(TN.JFA_COORD), ex.read(TN.JFA_COLOR)
    ru = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
    ru.write(TN.JFA_COORD, coord)
    ru.write(TN.JFA_COLOR, color)
    si = fovrt_mod.SibsonInterpolation(ru)
    ns = min(si.render() for _ in range(2))  # (the first call also loads the kernels)
    return coord, color, ru.read(TN.SIBSON), ns


@pytest.mark.parametrize("W,H,kind", [(160, 120, "few"), (97, 61, "corner"), (256, 144, "few"), (130, 70, "edge")])
def test_sibson_run_form_wide_discs(fovrt_mod, oracle, W, H, kind):
    """Discs spanning most of the image (a handful of seeds: the holes an off-centre log-polar gaze
    leaves, scripts/gaze_probe.py). Their boxes cross the binade edges of the tap positions and the
    image border, so the pixels take k_sibson_wide's segment tables; against the oracle's per-tap
    Sibson (sibsonFS.glsl:16-49)."""
    rng = np.random.default_rng(W * 7 + H)
    m = np.zeros((H, W), np.uint8)
    if kind == "few":
        m[rng.integers(0, H, 5), rng.integers(0, W, 5)] = 1
    elif kind == "corner":
        m[0, 0] = m[2, 1] = 1
    else:  # seeds along the right border only: discs reach across the left border
        m[::17, W - 1] = 1
    img = sparse_image(W, H, m, seed=W + H)
    coord, color, sf, _ = _jfa_then_run_form(fovrt_mod, img, W, H)
    rs = oracle.sibson(coord, color)
    assert np.isfinite(sf).all() and np.array_equal(sf[..., 3], rs[..., 3])
    assert np.abs(sf - rs).max() <= SIB_RUN_MAX, np.abs(sf - rs).max()
    # The shader's own f32 running sum over ~3e4 taps per pixel is off by up to ~2e-4 from the exact
    # average (256x144 "few": oracle against an f64 sum, max 1.85e-4, mean 8.4e-5 over 40 pixels), so
    # the RMSE bound here is that of the reference's rounding, not of the run form's (5e-5).
    assert (rmse_per_channel(sf, rs) <= 2e-4).all(), rmse_per_channel(sf, rs)
    for p in np.random.default_rng(3).choice(W * H, 16, replace=False):
        y, x = divmod(int(p), W)
        ref = _sibson_pixel_np(coord, color, x, y)
        assert np.abs(sf[y, x, :3] - ref).max() <= SIB_RUN_RMSE, (x, y, sf[y, x, :3], ref)


def _sibson_counts(fovrt_mod, t):
    """fr__sibson_counts: the last Sibson pass's list lengths (strips, wide[0], wide[1])."""
    import ctypes as C
    cnt = (C.c_uint32 * 3)()
    assert fovrt_mod.load_library().fr__sibson_counts(t._ctx, cnt) == 0
    return [int(v) for v in cnt]


@pytest.mark.parametrize("W,H,kind", [(640, 360, "logpolar180"), (512, 288, "few"), (256, 160, "corner")])
def test_sibson_strip_kernel_whole_image(fovrt_mod, oracle, W, H, kind, monkeypatch):
    """k_sibson_strip (the default for discs over 2 x 24 rows) on whole images against the oracle's per-tap
    Sibson (sibsonFS.glsl:16-49), every pixel: an off-centre signed log-polar mask (bench.py --gaze-path's
    cursor at 180 degrees, scaled to 640 x 360), a few-seed frame and two corner seeds. The pass must list
    strips (fr__sibson_counts), and the k_sibson_wide form (FOVRT_SIB_STRIP=0) of the same JFA output must
    agree with it within one GL_LINEAR weight step."""
    rng = np.random.default_rng(W + 3 * H)
    if kind == "logpolar180":
        m = logpolar_mask_np(W, H, W / 2 - 0.25 * H, H / 2, signed=True)
    else:
        m = np.zeros((H, W), np.uint8)
        if kind == "few":
            m[rng.integers(0, H, 5), rng.integers(0, W, 5)] = 1
        else:
            m[1, 2] = m[H - 3, W - 1] = 1
    img = sparse_image(W, H, m, seed=W + H)
    ex = _box_tracer(fovrt_mod, W, H)
    ex.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(ex).render(TN.SHADING)
    coord, color = ex.read(TN.JFA_COORD), ex.read(TN.JFA_COLOR)
    outs = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("FOVRT_SIB_STRIP", strip)
        ru = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
        ru.write(TN.JFA_COORD, coord)
        ru.write(TN.JFA_COLOR, color)
        fovrt_mod.SibsonInterpolation(ru).render()
        outs[strip] = ru.read(TN.SIBSON)
        counts = _sibson_counts(fovrt_mod, ru)
        if strip == "1":
            assert counts[0] > 0, counts  # the strip kernel ran
        else:
            assert counts[0] == 0 and counts[1] + counts[2] > 0, counts
        ru.destroy()
    rs = oracle.sibson(coord, color)
    sf = outs["1"]
    assert np.isfinite(sf).all() and np.array_equal(sf[..., 3], rs[..., 3])
    assert np.abs(sf - rs).max() <= SIB_RUN_MAX, np.abs(sf - rs).max()
    # the reference's own f32 running sums over 10^4-10^5 taps per pixel (test_sibson_run_form_wide_discs)
    assert (rmse_per_channel(sf, rs) <= 2e-4).all(), rmse_per_channel(sf, rs)
    assert np.array_equal(outs["0"][..., 3], sf[..., 3])
    assert np.abs(outs["0"] - sf).max() <= SIB_RUN_MAX, np.abs(outs["0"] - sf).max()


@pytest.mark.parametrize("W,H,kind", [(201, 400, "rightedge"), (329, 250, "rightedge"), (640, 360, "logpolar180"),
                                      (1920, 1080, "logpolar")])
def test_sibson_seeds_from_jfa_state(fovrt_mod, oracle, W, H, kind):
    """The run form right after its own JumpFlooding reads each pixel's seed from the final 8-byte JFA state
    (k_sibson_runs<true>); after the JFA outputs were written (or handed out) it reads JFA_COORD instead. Both
    must give the same image bit for bit. The right-edge cases put big discs (over 2 x 24 rows) in the last,
    partial 16-pixel tile column (W % 16 = 9 and 9) away from the top and bottom rows, where lanes past the
    tile's pixel count take part in the wave's row-range reduction."""
    if kind == "rightedge":
        m = np.zeros((H, W), np.uint8)
        m[::16, ::16] = 1  # seeds everywhere (small discs) but in a hole at the right border's middle
        m[H // 2 - 75:H // 2 + 75, W - 90:] = 0
        m[H // 2 - 70, W - 1] = m[H // 2 + 70, W - 1] = 1
    elif kind == "logpolar180":
        m = logpolar_mask_np(W, H, W / 2 - 0.25 * H, H / 2, signed=True)
    else:
        m = logpolar_mask_np(W, H, W // 2, H - H // 2, signed=True)
    img = sparse_image(W, H, m, seed=W * 5 + H)
    t = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
    t.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(t).render(TN.SHADING)
    fovrt_mod.SibsonInterpolation(t).render()  # seeds from the JFA state
    a = t.read(TN.SIBSON)
    coord, color = t.read(TN.JFA_COORD), t.read(TN.JFA_COLOR)
    if kind == "rightedge":
        assert _sibson_counts(fovrt_mod, t)[0] > 0  # big discs went to the strip kernel
    t.write(TN.JFA_COORD, coord)  # (the same values: now from JFA_COORD)
    fovrt_mod.SibsonInterpolation(t).render()
    b = t.read(TN.SIBSON)
    assert equal_nan(a, b), mismatch_report(a, b)
    if W * H <= 640 * 360:
        rs = oracle.sibson(coord, color)
        assert np.isfinite(a).all() and np.array_equal(a[..., 3], rs[..., 3])
        assert np.abs(a - rs).max() <= SIB_RUN_MAX, np.abs(a - rs).max()
        assert (rmse_per_channel(a, rs) <= 2e-4).all(), rmse_per_channel(a, rs)
    t.destroy()


@pytest.mark.parametrize("side", ["right", "left"])
def test_sibson_strip_kernel_binade_classes(fovrt_mod, side, monkeypatch):
    """k_sibson_strip on discs that span the whole row: seeds in one border column of a 3000 x 96 frame (W not a
    power of two, so the tap step differs from 1/W by a different rounding in every binade of x = 2^-k). Seeds on
    the right: the big discs sit at the left, and their rows cross a dozen segments near x = 0 (the class tables,
    the merged runs, the left border tap). Seeds on the left: the discs run into the right border (the right
    border tap) inside one binade. Against the shader's per-pixel loops on sampled pixels, and every pixel against
    the k_sibson_wide form (FOVRT_SIB_STRIP=0) within one GL_LINEAR weight step."""
    W, H = 3000, 96
    m = np.zeros((H, W), np.uint8)
    m[::6, W - 1 if side == "right" else 0] = 1
    img = sparse_image(W, H, m, seed=17 if side == "right" else 19)
    ex = _box_tracer(fovrt_mod, W, H)
    ex.write(TN.SHADING, img)
    fovrt_mod.JumpFlooding(ex).render(TN.SHADING)
    coord, color = ex.read(TN.JFA_COORD), ex.read(TN.JFA_COLOR)
    outs = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("FOVRT_SIB_STRIP", strip)
        ru = make_tracer(fovrt_mod, W, H, scene=0, mask=3, sibson_mode=0)
        ru.write(TN.JFA_COORD, coord)
        ru.write(TN.JFA_COLOR, color)
        fovrt_mod.SibsonInterpolation(ru).render()
        outs[strip] = ru.read(TN.SIBSON)
        if strip == "1":
            assert _sibson_counts(fovrt_mod, ru)[0] > 0  # the strip kernel ran
        ru.destroy()
    sf = outs["1"]
    assert np.isfinite(sf).all() and np.array_equal(outs["0"][..., 3], sf[..., 3])
    assert np.abs(outs["0"] - sf).max() <= SIB_RUN_MAX, np.abs(outs["0"] - sf).max()
    assert (rmse_per_channel(outs["0"], sf) <= SIB_RUN_RMSE).all(), rmse_per_channel(outs["0"], sf)
    yy, xx = np.mgrid[0:H, 0:W]
    d = np.hypot(coord[..., 0] - (xx + 0.5) / W, coord[..., 1] - (yy + 0.5) / H)
    big = np.flatnonzero(d.ravel() * H > 64)
    assert big.size > 1000
    for p in np.random.default_rng(7).choice(big, 12, replace=False):
        y, x = divmod(int(p), W)
        ref = _sibson_pixel_np(coord, color, x, y)
        assert ref is not None and sf[y, x, 3] == 1.0
        assert np.abs(sf[y, x, :3] - ref).max() <= SIB_RUN_MAX, (x, y, sf[y, x, :3], ref)


def _sibson_pixel_np(coord, color, x, y):
    """One pixel of sibsonFS.glsl:16-49 in numpy: the shader's f32 position sequences (h, w += 1/size)
    walked in order, the taps outside [0, 1) or the disc dropped, GL_LINEAR + REPEAT at each tap
    (8-bit weights), summed in f64 (any order: the run form's own order differs)."""
    f = np.float32
    H, W = coord.shape[:2]
    fx, fy = f((f(x) + f(0.5)) / f(W)), f((f(y) + f(0.5)) / f(H))
    cs, ct = coord[y, x, 0], coord[y, x, 1]
    dx, dy = f(cs - fx), f(ct - fy)
    d = f(np.sqrt(f(f(dx * dx) + f(dy * dy))))

    def seq(lo, hi, inc):
        out, v = [], lo
        while v < hi:
            out.append(v)
            v = f(v + inc)
        return np.array(out, f)

    ws = seq(f(fx - d), f(fx + d), f(f(1) / f(W)))
    hs = seq(f(fy - d), f(fy + d), f(f(1) / f(H)))
    ww, hh = np.meshgrid(ws, hs)
    r = np.sqrt(f(f(f(fx - ww) ** 2) + f(f(fy - hh) ** 2)), dtype=f)
    on = (ww >= 0) & (ww < 1) & (hh >= 0) & (hh < 1) & ~(r > d)
    if not on.any():
        return None
    c = _gl_linear_repeat(color, ww[on], hh[on]).astype(np.float64)
    return c[:, :3].sum(0) / on.sum()


def test_sibson_run_form_offcentre_gaze_4k(fovrt_mod):
    """The 4K log-polar mask of bench.py --gaze-path's cursor at 180 degrees (gaze (1380, 1080)) leaves
    holes whose discs reach ~1,100 rows: the widest pixels (k_sibson_wide) and a sample of the rest
    against the shader's per-pixel loops. The seeds are the mask alone (no carried history), so the
    holes are wider than in the bench's frames (mean disc 103 rows): the pass takes ~28 ms here with
    k_sibson_strip (41 ms with k_sibson_wide alone, FOVRT_SIB_STRIP=0; ~96 ms before the border runs' split,
    round 4); the bound is a regression guard against per-tap walks."""
    W, H = 3840, 2160
    mask = logpolar_mask_np(W, H, 1380, 1080, signed=True)
    img = sparse_image(W, H, mask, seed=11)
    coord, color, sf, ns = _jfa_then_run_form(fovrt_mod, img, W, H)
    assert np.isfinite(sf).all()
    yy, xx = np.mgrid[0:H, 0:W]
    d = np.hypot(coord[..., 0] - (xx + 0.5) / W, coord[..., 1] - (yy + 0.5) / H)
    rng = np.random.default_rng(5)
    wide = np.argsort(d.ravel())[-400:]
    pick = np.concatenate([rng.choice(wide, 12, replace=False), rng.choice(np.flatnonzero(d > 0), 12, replace=False),
                           [int(np.argmax(d))]])
    for i, p in enumerate(pick):
        y, x = divmod(int(p), W)
        ref = _sibson_pixel_np(coord, color, x, y)
        if ref is None:  # a disc narrower than the tap spacing may hold no tap: the seed colour
            assert 12 <= i < 24, (x, y)
            continue
        assert sf[y, x, 3] == 1.0, (x, y)
        assert np.abs(sf[y, x, :3] - ref).max() <= SIB_RUN_MAX, (x, y, d[y, x] * H, sf[y, x, :3], ref)
    assert ns / 1e6 < 80.0, ns / 1e6


@pytest.mark.parametrize("W,H", [(64, 64), (96, 64), (256, 256), (130, 70)])
def test_pullpush_bit_exact_across_frames(fovrt_mod, oracle, W, H):
    rng = np.random.default_rng(W + 7 * H)
    t = _box_tracer(fovrt_mod, W, H)
    st = oracle.PullPushState(W, H)
    npst = PullPushNp(W, H)  # the independent numpy restatement of the shaders as well
    for k, p in enumerate((0.1, 0.01, 0.3, 0.0)):
        img = sparse_image(W, H, (rng.random((H, W)) < p).astype(np.uint8), seed=k)
        t.write(TN.SHADING, img)
        fovrt_mod.PullPushInterpolation(t).render(TN.SHADING)
        got = t.read(TN.PULLPUSH)
        ref = st.render(img)
        assert equal_nan(got, ref), (k, mismatch_report(got, ref))
        assert equal_nan(got, npst.render(img)), k


@pytest.mark.parametrize("W,H", [(80, 60), (203, 77)])  # the second: ragged 16x16 blocks, interior and edge
@pytest.mark.parametrize("count", [1, 2, 3])
def test_atrous_within_tolerance(fovrt_mod, oracle, count, W, H):
    rng = np.random.default_rng(count + W)
    t = _box_tracer(fovrt_mod, W, H)
    pos, nrm, col = (rng.random((H, W, 4), dtype=np.float32) for _ in range(3))
    t.write(TN.POSITION, pos)
    t.write(TN.NORMAL, nrm)
    t.write(TN.PULLPUSH, col)
    fovrt_mod.ATrous(t).render(count, TN.POSITION, TN.NORMAL, TN.PULLPUSH)
    got = t.read(TN.ATROUS)
    ref = oracle.atrous(count, pos, nrm, col)
    assert np.abs(got - ref).max() < 2e-6
    assert np.abs(got - atrous_np(count, pos, nrm, col)).max() < 4e-6  # the numpy restatement of atFS


def test_golden_vectors_on_gpu(fovrt_mod):
    import os
    g = np.load(os.path.join(GOLDEN, "jfa_64x48.npz"))
    t = _box_tracer(fovrt_mod, 64, 48)
    t.write(TN.SHADING, g["input"])
    fovrt_mod.JumpFlooding(t).render()
    assert equal_nan(t.read(TN.JFA_COORD), g["coord"]) and equal_nan(t.read(TN.JFA_COLOR), g["color"])
    s = np.load(os.path.join(GOLDEN, "sibson_64x48.npz"))
    fovrt_mod.SibsonInterpolation(t).render()
    assert equal_nan(t.read(TN.SIBSON), s["output"])
    p = np.load(os.path.join(GOLDEN, "pullpush_64.npz"))
    t2 = _box_tracer(fovrt_mod, 64, 64)
    for k in range(p["inputs"].shape[0]):
        t2.write(TN.SHADING, p["inputs"][k])
        fovrt_mod.PullPushInterpolation(t2).render()
        assert equal_nan(t2.read(TN.PULLPUSH), p["outputs"][k]), k


# ---------------------------------------------------------------------------------------------
# Whole frame: fr_frame == the reference's stage-by-stage call sequence; full-size properties
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("timing", [True, False])  # False: frames pipelined (reconstruction || next trace)
def test_frame_driver_equals_stage_calls(fovrt_mod, timing):
    W, H = 128, 128
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    for _ in range(4):
        a.frame(timing=timing)
        b.geometry_launch(); b.sampling_launch(); b.optimize_launch(); b.shading_launch()
        fovrt_mod.JumpFlooding(b).render(TN.SHADING)
        fovrt_mod.SibsonInterpolation(b).render()
        fovrt_mod.PullPushInterpolation(b).render(TN.SHADING)
        fovrt_mod.ATrous(b).render(1, TN.POSITION, TN.NORMAL, TN.PULLPUSH)
    for tid in (TN.SHADING, TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS, TN.HISTORY_CACHE, TN.POSITION,
                TN.NORMAL, TN.DEPTH_CACHE):
        assert equal_nan(a.read(tid), b.read(tid)), tid


@pytest.mark.parametrize("chunk,bands", [("64", "1"), ("4", "1"), ("0", "0"), ("64", "0")])
def test_megakernel_schedule_does_not_change_samples(fovrt_mod, monkeypatch, chunk, bands):
    """The megakernel's work queue (k_shade_paths): at 1080p the launch has between 1 and 8 samples per
    lane, so the refraction class is handed out in small chunks spread over all waves (the adaptive
    policy), and each XCD takes one band of every primary-hit class. Fixed 64-slot and 4-slot chunks
    (FOVRT_SHADE_CHUNK_REFR) and chunks interleaved over the XCDs (FOVRT_SHADE_XCD_BANDS=0), both read at
    fr_create, schedule the same samples differently: every slot must still be traced exactly once,
    and a sample's value does not depend on the lane or the time it runs, so SHADING and the history
    are bit-identical."""
    W, H = 1920, 1080
    monkeypatch.delenv("FOVRT_SHADE_CHUNK_REFR", raising=False)
    monkeypatch.delenv("FOVRT_SHADE_XCD_BANDS", raising=False)
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=1)
    monkeypatch.setenv("FOVRT_SHADE_CHUNK_REFR", chunk)
    monkeypatch.setenv("FOVRT_SHADE_XCD_BANDS", bands)
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=1)
    for t in (a, b):
        t.update_optix_variables(fovrt_mod.Camera.preset(1, W, H))
    for _ in range(2):
        for t in (a, b):
            t.geometry_launch(); t.sampling_launch(); t.optimize_launch(); t.shading_launch()
    assert a.ray_count() == b.ray_count() and a.ray_count() * 4 > 1536 * 128  # >= 1 sample per lane
    for tid in (TN.SHADING, TN.HISTORY_CACHE):
        assert equal_nan(a.read(tid), b.read(tid)), tid
    st_a, st_b = a.stats(), b.stats()
    for k in ("primary", "shadow", "mirror", "refraction", "reflection"):
        assert st_a[k] == st_b[k], k
    a.destroy(); b.destroy()


@pytest.mark.parametrize("W,H,spp", [(1920, 1080, 4), (256, 256, 8)])
def test_megakernel_tail_handoff(fovrt_mod, monkeypatch, W, H, spp):
    """The small-launch form of k_shade_paths (SampleSum): fixed-point sample sums, and idle lanes of a
    dry wave take pending refraction/reflection items of their busy neighbours. FOVRT_SHADE_HANDOFF=1 (the
    default) uses it for frames below 64 pixel-samples (W H spp) per lane of the grid, which covers 1080p
    at 4 spp and 256x256; 2 forces it, 0 turns it off (fp32 running sums, the oracle's order). The default and the forced form are bit-identical
    (the same form; which lanes run an item does not change the integer sums); the fp32 form differs only
    by the rounding of the sums: per channel RMSE <= 1e-6, max 1e-4 on the tone-mapped colour."""
    monkeypatch.delenv("FOVRT_SHADE_CHUNK_REFR", raising=False)
    monkeypatch.delenv("FOVRT_SHADE_XCD_BANDS", raising=False)
    tracers = {}
    for mode in ("1", "2", "0"):
        monkeypatch.setenv("FOVRT_SHADE_HANDOFF", mode)
        t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=spp, dmd=3)
        t.update_optix_variables(fovrt_mod.Camera.preset(1, W, H))
        for _ in range(2):
            t.geometry_launch(); t.sampling_launch(); t.optimize_launch(); t.shading_launch()
        tracers[mode] = t
    a, b, c = tracers["1"], tracers["2"], tracers["0"]
    for tid in (TN.SHADING, TN.HISTORY_CACHE):
        assert equal_nan(a.read(tid), b.read(tid)), tid
    sa, sc = a.read(TN.SHADING), c.read(TN.SHADING)
    assert np.array_equal(np.isnan(sa), np.isnan(sc))
    assert (rmse_per_channel(sa, sc) <= 1e-6).all(), rmse_per_channel(sa, sc)
    assert np.nanmax(np.abs(sa - sc)) <= 1e-4, mismatch_report(sa, sc)
    st = [t.stats() for t in (a, b, c)]
    for k in ("primary", "shadow", "mirror", "refraction", "reflection", "truncated"):
        assert st[0][k] == st[1][k] == st[2][k], k
    for t in (a, b, c):
        t.destroy()


@pytest.mark.parametrize("slots", ["3", "2"])
def test_pipelined_frames_panning_equal_stage_calls(fovrt_mod, monkeypatch, slots):
    """fr_frame pipelining (front stages of frame N+1 beside entry 3 of frame N, reconstruction inputs and
    the trace tail's WEIGHT / mask / active list rotating over FOVRT_SLOTS frame slots) against the
    synchronous stage calls: 8 frames (the slots wrap around more than twice), the camera panning every
    frame, so every frame's shading reprojects the previous history; all outputs bit-identical."""
    monkeypatch.setenv("FOVRT_SLOTS", slots)
    W, H = 320, 192
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    cam = fovrt_mod.Camera.preset(1, W, H)
    for f in range(8):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
        a.update_optix_variables(cam)
        b.update_optix_variables(cam)
        a.frame(timing=False)
        b.geometry_launch(); b.sampling_launch(); b.optimize_launch(); b.shading_launch()
        fovrt_mod.JumpFlooding(b).render(TN.SHADING)
        fovrt_mod.SibsonInterpolation(b).render()
        fovrt_mod.PullPushInterpolation(b).render(TN.SHADING)
        fovrt_mod.ATrous(b).render(1, TN.POSITION, TN.NORMAL, TN.PULLPUSH)
    for tid in (TN.SHADING, TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS, TN.HISTORY_CACHE, TN.POSITION,
                TN.NORMAL, TN.DEPTH_CACHE, TN.WEIGHT, TN.MASK):
        assert equal_nan(a.read(tid), b.read(tid)), tid
    assert a.ray_count() == b.ray_count()


def test_early_sample_setup_equals_setup_after_resolve(fovrt_mod, monkeypatch):
    """The early sample setup of latency mode (a frame's k_sample_setup on the front stream with its front stages,
    from the history validity bits the previous frame's k_carry_history wrote) against the setup after the previous
    resolve on the context stream (FOVRT_EARLY_SETUP=0): 12 frames, the camera panning and the gaze
    moving every frame (the seeds' validity comes from reprojected pixels), a light change (the accumulation
    restarts at frame 0, which clears the history), a timed frame, and a host write of HISTORY_CACHE that leaves
    part of the history invalid (the next frame must not use the bits of the history before the write). Bit for
    bit, frame by frame at the checkpoints."""
    W, H = 320, 192
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    monkeypatch.setenv("FOVRT_EARLY_SETUP", "0")
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    monkeypatch.delenv("FOVRT_EARLY_SETUP")
    for t in (a, b):
        t.set_pipeline_mode(fovrt_mod.PIPELINE_LATENCY)
    cam = fovrt_mod.Camera.preset(1, W, H)
    hist = np.zeros((H, W, 4), np.float32)
    hist[:, : W // 2] = (0.25, 0.5, 0.75, 1.0)  # the right half's history invalid (.w = 0)
    outs = (TN.SHADING, TN.HISTORY_CACHE, TN.SIBSON, TN.ATROUS, TN.MASK, TN.WEIGHT)
    for f in range(12):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
        for t in (a, b):
            t.update_optix_variables(cam)
            t.set_gaze(W / 2 + 30 * np.cos(f), (H / 2 + 30 * np.sin(f)) / 1.25)
            if f == 4:
                t.set_light_power(0.8)
            if f == 7:
                t.write(TN.HISTORY_CACHE, hist)
            t.frame(timing=f == 9)
        if f in (3, 8, 11):
            for tid in outs:
                assert equal_nan(a.read(tid), b.read(tid)), (f, tid)
    assert a.ray_count() == b.ray_count()
    for t in (a, b):
        t.destroy()


def test_latency_pipeline_mode_equals_throughput_mode(fovrt_mod):
    """fr_set_pipeline_mode(FR_PIPELINE_LATENCY) (one trace half in flight; the host waits for the previous
    frame's path trace) renders the same frames as the default throughput pipelining, bit for bit, with
    the camera panning and the gaze moving every frame; the frame clock covers every frame."""
    W, H = 320, 192
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    a.set_pipeline_mode(fovrt_mod.PIPELINE_LATENCY)
    a.frame_clock(True)
    cam = fovrt_mod.Camera.preset(1, W, H)
    for f in range(7):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
        for t in (a, b):
            t.update_optix_variables(cam)
            t.set_gaze(W / 2 + 20 * np.cos(f), (H / 2 + 20 * np.sin(f)) / 1.25)
            t.frame(timing=False)
    lat, itv = a.frame_clock_read()
    a.frame_clock(False)
    assert len(lat) == 7 and len(itv) == 6 and (lat > 0).all()
    for tid in (TN.SHADING, TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS, TN.HISTORY_CACHE, TN.MASK):
        assert equal_nan(a.read(tid), b.read(tid)), tid
    with pytest.raises(fovrt_mod.FovrtError):
        a.set_pipeline_mode(2)


def test_kernel_timing_counts_frames_and_leaves_results_unchanged(fovrt_mod):
    """fr_kernel_timing: live HIP events around entry 3 of pipelined frames (what bench.py reports)."""
    W, H, K = 128, 128, 40  # more frames than the 32-slot event ring: slots are harvested on reuse
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=1, spp=4, dmd=3)
    a.kernel_timing(True)
    for _ in range(K):
        a.frame(timing=False)
        b.frame(timing=False)
    kt = a.kernel_times()
    a.kernel_timing(False)
    assert kt["frames"] == K
    assert kt["shading_ms"] >= kt["shade_paths_ms"] > 0
    for tid in (TN.SHADING, TN.SIBSON, TN.ATROUS, TN.HISTORY_CACHE):
        assert equal_nan(a.read(tid), b.read(tid)), tid


@pytest.mark.parametrize("scene,W,H", [(1, 3840, 2160), (2, 3840, 2160), (1, 7680, 4320)])
def test_full_size_frame_properties(fovrt_mod, scene, W, H):
    """BASELINE configs[2] (bunny) and the scene of configs[3] (vokselia) at full size (3840x2160, 4 spp,
    GI 3, 10% log-polar mask), and 8K (within the compaction scan's limit of 64 M pixels): size-independent
    invariants of every stage."""
    t = make_tracer(fovrt_mod, W, H, scene=scene, mask=4, spp=4, dmd=3)
    for _ in range(2):
        tm = t.frame(timing=True)
    mask = t.read(TN.MASK)
    n = t.ray_count()
    assert n == tm["ray_count"] == int(mask.sum())
    assert 0.08 < n / (W * H) < 0.12  # ~9.5% at 4K
    assert np.array_equal(mask, logpolar_mask_np(W, H, W // 2, H - H // 2, signed=True))
    sh = t.read(TN.SHADING)
    assert np.all(sh[..., 3][mask == 1] == 1.0)
    coord = t.read(TN.JFA_COORD)
    assert np.all(coord[..., 3] == 1.0)  # every pixel found a seed
    at = t.read(TN.ATROUS)
    assert np.isfinite(at).mean() > 0.999
    st = t.stats()
    assert st["overflow"] == 0
    assert st["primary"] == 2 * n * 4
    assert st["gbuffer_primary"] == 2 * W * H


# ---------------------------------------------------------------------------------------------
# The C++ facades (include/fovrt.hpp): the headless main.cpp-shaped driver gives the same images
# as the Python mirror driving the same C ABI calls
# ---------------------------------------------------------------------------------------------
def test_cpp_facade_driver_matches_python(fovrt_mod, tmp_path):
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(fovrt_mod.LIB_PATH), "fovrt_run")
    assert os.path.exists(exe), "build with make -C foveated-rendering-using-ray-tracing_amd"
    W, H, frames = 96, 64, 2
    out = tmp_path / "atrous.pfm"
    args = [exe, str(W), str(H), "--scene", "bunny", "--mask", "logpolar10", "--spp", "4", "--dmd", "3",
            "--frames", str(frames), "--dump", "ATROUS", str(out), "--assets", ASSET_DIR]
    if TEXTURE_MODE == 1:
        args.append("--procedural")
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("ray count") == frames
    with open(out, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        assert (w, h) == (W, H) and float(f.readline()) < 0
        img = np.frombuffer(f.read(), dtype="<f4").reshape(H, W, 3)
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    for _ in range(frames):
        t.geometry_launch(); t.sampling_launch(); t.optimize_launch(); t.shading_launch()
        fovrt_mod.JumpFlooding(t).render(TN.SHADING)
        fovrt_mod.SibsonInterpolation(t).render()
        fovrt_mod.PullPushInterpolation(t).render(TN.SHADING)
        fovrt_mod.ATrous(t).render(1, TN.POSITION, TN.NORMAL, TN.PULLPUSH)
    assert equal_nan(img, t.read(TN.ATROUS)[..., :3])


# ---------------------------------------------------------------------------------------------
# Tile sharding (BASELINE configs[3]): ranks trace their own screen tiles, the root
# unpacks the others' shading tiles and reconstructs; the composite equals the one-GPU frame.
# Rehearsed here with three contexts on one device (one process), slabs in torch device memory.
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("nranks,tile,first,sparse,W,H", [(2, 64, 0, False, 200, 136), (3, 32, 0, False, 200, 136),
                                                         (2, 64, 1, False, 200, 136), (3, 32, 1, False, 200, 136),
                                                         (4, 16, 1, False, 200, 136), (3, 32, 0, True, 200, 136),
                                                         (2, 64, 1, True, 200, 136), (4, 16, 1, True, 200, 136),
                                                         (4, 128, 1, True, 3840, 2160)])
def test_tile_shards_composite_equals_full_frame(fovrt_mod, nranks, tile, first, sparse, W, H):
    """first = 1 (fr_set_shard_ex, the bench default): the compositing rank traces no tiles. sparse: the
    gather sends only the traced pixels (fr_shard_pack_active / fr_shard_unpack_active) instead of the
    ranks' tile slabs of SHADING. 200x136 is not a multiple of the tiles (clipped border tiles); 4K is the
    bench's tiling, where each tracer's launch is small but the frame is not: the sample-sum form follows
    the frame size (SampleSum), so the ranks and the one-GPU frame still agree bit for bit."""
    import torch
    full = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    ranks = [make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3) for _ in range(nranks)]
    for r, t in enumerate(ranks):
        t.set_shard(r, nranks, tile, first)
    n = ranks[0].shard_texels()
    assert all(t.shard_texels() == n for t in ranks)
    slabs = [torch.zeros(n * 4, dtype=torch.float32, device="cuda") for _ in range(nranks)]
    root = ranks[0]
    for _ in range(3):
        full.frame(timing=False)
        counts = [t.trace_frame(timing=True)["ray_count"] for t in ranks]
        if sparse:
            cap = max(counts)
            act = [torch.zeros(cap * 5 + 1, dtype=torch.float32, device="cuda") for _ in range(nranks)]
            packed = [t.shard_pack_active(act[r].data_ptr(), cap) for r, t in enumerate(ranks)]
            assert packed == counts
            for r in range(1, nranks):
                root.shard_unpack_active(act[r].data_ptr(), cap, packed[r])
        else:
            for r, t in enumerate(ranks):
                t.shard_pack(TN.SHADING, slabs[r].data_ptr(), n * 16)
            for r in range(1, nranks):
                root.shard_unpack(TN.SHADING, r, slabs[r].data_ptr(), n * 16)
        root.reconstruct_frame(timing=False)
        assert sum(counts) == full.ray_count()
        assert first == 0 or counts[0] == 0
        assert equal_nan(root.read(TN.SHADING), full.read(TN.SHADING))
    for tid in (TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS):
        assert equal_nan(root.read(tid), full.read(tid)), tid
    masks = sum(t.read(TN.MASK).astype(np.int32) for t in ranks)
    assert np.array_equal(masks, full.read(TN.MASK))  # the ranks' masks partition the full mask


@pytest.mark.parametrize("scene,mask", [(0, 0), (0, 4), (1, 4)])
def test_tile_shards_moving_camera_with_history_exchange(fovrt_mod, scene, mask):
    """Moving camera: reprojection reads the previous frame's history at other ranks' tiles, so every
    rank all-gathers HISTORY_CACHE after its trace half (bench.py exchange_history). With that exchange
    the composite equals the single-context frame bit for bit; without it, it does not."""
    import torch
    W, H, nranks, tile = 160, 112, 2, 16
    mk = lambda: make_tracer(fovrt_mod, W, H, scene=scene, mask=mask, spp=2, dmd=2)
    full, ranks, stale = mk(), [mk() for _ in range(nranks)], [mk() for _ in range(nranks)]
    for group in (ranks, stale):
        for r, t in enumerate(group):
            t.set_shard(r, nranks, tile)
    n = ranks[0].shard_texels()
    slabs = [torch.zeros(n * 4, dtype=torch.float32, device="cuda") for _ in range(nranks)]
    cam = fovrt_mod.Camera.preset(scene, W, H)
    diverged, cross = False, 0
    for f in range(5):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.03, 0.02, 0.0], np.float32))  # pan: the eye stays
        for t in [full] + ranks + stale:
            t.update_optix_variables(cam)
        full.frame(timing=False)
        for group, exchange in ((ranks, True), (stale, False)):
            for t in group:
                t.trace_frame(timing=False)
            if exchange:  # all-gather of HISTORY_CACHE (the buffer the next frame reprojects from)
                for r, t in enumerate(group):
                    t.shard_pack(TN.HISTORY_CACHE, slabs[r].data_ptr(), n * 16)
                for r, t in enumerate(group):
                    for s in range(nranks):
                        if s != r:
                            t.shard_unpack(TN.HISTORY_CACHE, s, slabs[s].data_ptr(), n * 16)
            for r, t in enumerate(group):
                t.shard_pack(TN.SHADING, slabs[r].data_ptr(), n * 16)
            for r in range(1, nranks):
                group[0].shard_unpack(TN.SHADING, r, slabs[r].data_ptr(), n * 16)
            group[0].reconstruct_frame(timing=False)
        for tid in (TN.SHADING, TN.ATROUS):
            assert equal_nan(ranks[0].read(tid), full.read(tid)), (f, tid)
        assert equal_nan(ranks[1].read(TN.HISTORY_CACHE), full.read(TN.HISTORY_CACHE)), f
        # valid reprojections whose source texel lies in a tile of the other rank
        wgt = full.read(TN.WEIGHT)
        ys, xs = np.nonzero(wgt[..., 2] > 0)
        qx = np.floor(wgt[ys, xs, 0] + np.float32(0.5)).astype(np.int64)
        qy = np.floor(wgt[ys, xs, 1] + np.float32(0.5)).astype(np.int64)
        tiles_x = (W + tile - 1) // tile
        owner = lambda x, y: ((y // tile) * tiles_x + x // tile) % nranks
        cross += int(np.count_nonzero(owner(xs, ys) != owner(qx, qy)))
        diverged |= not equal_nan(stale[0].read(TN.SHADING), full.read(TN.SHADING))
    print("valid:", len(xs), "cross-tile:", cross, "stale diverged:", diverged)
    assert cross > 0  # the camera motion makes ranks read each other's history
    assert diverged  # ... and the exchange is what keeps the tiles exact


# ---------------------------------------------------------------------------------------------
# LogPolarTransform (FR/Log_Polar_Transform.cpp:40-106) and the gaze input (FR/gui.cpp:48-66)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("W,H", [(128, 96), (200, 136)])
def test_logpolar_transform_bit_exact(fovrt_mod, oracle, W, H):
    t = _box_tracer(fovrt_mod, W, H)
    rs = np.random.RandomState(W)
    lp = fovrt_mod.LogPolarTransform(t)
    fwd = inv = None
    for k, gaze_window in enumerate([None, (W * 0.3, H * 0.2), (W - 5.0, 7.0)]):
        img = rs.rand(H, W, 4).astype(np.float32)
        t.write(TN.SHADING, img)
        if gaze_window is None:
            gaze = (W // 2, H - H // 2)  # the default gaze (FR/gui.cpp:34-35, kernels use H - y)
        else:
            t.set_gaze(*gaze_window)
            gaze = ref_gaze(H, *gaze_window)
        lp.render(TN.SHADING)
        fwd, inv = oracle.logpolar(img, gaze, fwd, inv)  # outputs persist across calls, as GL textures do
        assert equal_nan(t.read(TN.LOGPOLAR), fwd), k
        assert equal_nan(t.read(TN.LOGPOLAR_INVERSE), inv), k


def test_set_gaze_follows_the_cursor_mapping(fovrt_mod):
    """fr_set_gaze = cursorPosCallback: windowed cursors are scaled by adjust_scale = 1.25 in y and
    truncated to the Win32 POINT; full screen uses 1; fr_reset_gaze = framebufferSizeCallback's
    (W / 2, H / 2). Checked through the gaze the log-polar mask is built around."""
    W, H = 160, 96
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=1, dmd=1)
    cases = [((40.7, 30.9), False), ((40.7, 30.9), True), ((-3.5, 70.2), False), ((159.9, 0.0), False)]
    for (x, y), fs in cases:
        t.set_gaze(x, y, fullscreen=fs)
        t.frame(timing=False)
        g = ref_gaze(H, x, y, fs)
        assert np.array_equal(t.read(TN.MASK), logpolar_mask_np(W, H, g[0], g[1], signed=True)), (x, y, fs)
    # windowed 30.9 * 1.25 = 38.625 -> 38, full screen 30 : the two masks differ
    assert ref_gaze(H, 40.7, 30.9)[1] == H - 38 and ref_gaze(H, 40.7, 30.9, True)[1] == H - 30
    t.reset_gaze()
    t.frame(timing=False)
    assert np.array_equal(t.read(TN.MASK), logpolar_mask_np(W, H, W // 2, H - H // 2, signed=True))


def test_composite_views_side_by_side(fovrt_mod):
    import torch
    W, H = 96, 64
    eyes = [make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=1, dmd=1) for _ in range(2)]
    for k, t in enumerate(eyes):
        cam = fovrt_mod.Camera.preset(1, W, H)
        cam.setPosition(np.asarray(cam.pos) + np.array([0.064 * (k - 0.5), 0, 0], np.float32))
        cam.lookAt(cam.target)
        t.update_optix_variables(cam)
        t.frame(timing=False)
    stack = torch.empty(2 * W * H * 4, dtype=torch.float32, device="cuda")
    for k, t in enumerate(eyes):
        t.copy_buffer(TN.ATROUS, stack[k * W * H * 4:].data_ptr(), W * H * 16)
    out = torch.empty_like(stack)
    eyes[0].composite_views(stack.data_ptr(), 2, out.data_ptr(), out.numel() * 4)
    img = out.cpu().numpy().reshape(H, 2 * W, 4)
    assert equal_nan(img[:, :W], eyes[0].read(TN.ATROUS)) and equal_nan(img[:, W:], eyes[1].read(TN.ATROUS))
    assert not equal_nan(img[:, :W], img[:, W:])  # two different eyes


def test_logpolar_mask_cache_follows_the_gaze(fovrt_mod):
    """The log-polar sampling mask is cached between frames and recomputed when the gaze moves."""
    W, H = 160, 96
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=1, dmd=1)
    for gaze_window in (None, None, (40.0, 30.0), (40.0, 30.0), (150.0, 90.0)):
        if gaze_window is not None:
            t.set_gaze(*gaze_window)
            g = ref_gaze(H, *gaze_window)
        else:
            g = (W // 2, H - H // 2)
        t.frame(timing=False)
        assert np.array_equal(t.read(TN.MASK), logpolar_mask_np(W, H, g[0], g[1], signed=True)), gaze_window


# ---------------------------------------------------------------------------------------------
# GPU BVH builder (k_bvh.hip): traversal results do not depend on the tree, so
# frames over the device-built LBVH equal the host-built binned-SAH ones bit for bit.
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene", [0, 1, 2])
def test_gpu_bvh_builder_frames_equal_host_built(fovrt_mod, scene):
    W, H = 160, 96
    host = make_tracer(fovrt_mod, W, H, scene=scene, mask=4, spp=2, dmd=2)
    dev = make_tracer(fovrt_mod, W, H, scene=scene, mask=4, spp=2, dmd=2, bvh_builder=1)
    for _ in range(3):
        host.frame(timing=False)
        dev.frame(timing=False)
    for tid in (TN.POSITION, TN.NORMAL, TN.DEPTH, TN.DIFFUSE, TN.SHADING, TN.ATROUS):
        assert equal_nan(dev.read(tid), host.read(tid)), tid
    assert dev.stats()["segments"] == host.stats()["segments"]
    a = dev.scene_arrays()
    assert 0 < a["bvh_nodes"] and a["bvh_max_stack"] <= 24
    ms = dev.rebuild_bvh()
    assert ms > 0.0
    dev.frame(timing=False)
    host.frame(timing=False)
    assert equal_nan(dev.read(TN.SHADING), host.read(TN.SHADING))


def test_gpu_bvh_follows_moved_triangles(fovrt_mod, oracle):
    """fr_set_positions: new vertex positions, device rebuild; the G-buffer equals the oracle's over
    the moved triangles (the oracle traces the exported soup)."""
    W, H = 96, 64
    t = make_tracer(fovrt_mod, W, H, scene=1, bvh_builder=1)
    pos = t.scene_arrays()["pos"].reshape(-1, 3, 3).copy()
    pos[..., 1] += np.float32(0.05) * np.sin(np.float32(3.0) * pos[..., 0]).astype(np.float32)
    t.set_positions(pos)
    uni = fovrt_mod.Camera.preset(1, W, H).uniforms(W, H)
    t.set_camera_uniforms(uni)
    t.geometry_launch()
    arrays = t.scene_arrays()
    assert np.array_equal(arrays["pos"].reshape(-1, 3, 3), pos)
    ref = oracle.gbuffer(oracle.OracleScene(arrays), uni, W, H, 0)
    for name, tid in [("position", TN.POSITION), ("normal", TN.NORMAL), ("depth", TN.DEPTH),
                      ("diffuse", TN.DIFFUSE)]:
        got = t.read(tid)
        assert equal_nan(got, ref[name]), (name, mismatch_report(got, ref[name]))
    # the bounding box (depth-saliency theta) follows the geometry; the tree depth is reported
    flat = pos.reshape(-1, 3)
    assert np.array_equal(arrays["bbox"], np.concatenate([flat.min(0), flat.max(0)]).astype(np.float32))
    assert arrays["bvh_depth"] > 0
    inp = {k: t.read(v) for k, v in [("position", TN.POSITION), ("depth", TN.DEPTH), ("depth_cache", TN.DEPTH_CACHE),
                                     ("weight", TN.WEIGHT), ("normal", TN.NORMAL), ("diffuse", TN.DIFFUSE)]}
    t.sampling_launch()
    sref = oracle.sampling(oracle.OracleScene(arrays), uni, W, H, 1, inp["position"], inp["depth"],
                           inp["depth_cache"], inp["weight"], inp["normal"], inp["diffuse"])
    assert np.array_equal(t.read(TN.EXTRA), sref["extra"])
    # a rejected update leaves the scene as it was
    bad = pos.copy()
    bad[0, 0, 0] = np.nan
    with pytest.raises(RuntimeError):
        t.set_positions(bad)
    assert np.array_equal(t.scene_arrays()["pos"].reshape(-1, 3, 3), pos)
    t.geometry_launch()
    assert equal_nan(t.read(TN.POSITION), ref["position"])


# ---------------------------------------------------------------------------------------------
# Multi-GPU groups through the C ABI (fr_group_*): ranks as contexts of this process on the one GPU
# of the box (device-to-device copies), and a one-rank RCCL communicator. The group runs the same
# frame as the reference's loop on one GPU, so every output equals the single-context frame.
# ---------------------------------------------------------------------------------------------
def foreign_history(weight, own):
    """Pixels whose carried history (k_carry_history / history_of: texel f2u_sat(roundf(.x)), f2u_sat(roundf(.y))
    of the previous history when .z > 0) comes from outside `own`, directly or through a chain of such
    sources (a still camera maps each pixel to the same source every frame)."""
    H, W = own.shape
    w = weight.astype(np.float64)
    valid = w[..., 2] > 0
    rnd = lambda a: np.clip(np.trunc(a + np.copysign(0.5, a)), 0, 2.0 ** 32 - 1)  # roundf, then f2u_sat
    src = np.clip(rnd(w[..., 1]) * W + rnd(w[..., 0]), 0, W * H - 1).astype(np.int64).ravel()
    own_f, valid_f = own.ravel(), valid.ravel()
    bad = valid_f & ~own_f[src]
    for _ in range(16):
        nxt = bad | (valid_f & bad[src])
        if np.array_equal(nxt, bad):
            break
        bad = nxt
    return bad.reshape(H, W)


GROUP_CASES = [  # (ranks, views, tile, split, moving, W, H, mask, jfa_ranks)
    (2, 1, 64, True, False, 200, 136, 4, 0), (3, 1, 32, True, False, 200, 136, 4, 0), (4, 1, 16, True, False, 200, 136, 0, 0),
    (3, 1, 32, False, False, 200, 136, 4, 0), (4, 2, 32, True, False, 200, 136, 4, 0), (2, 1, 32, True, True, 160, 112, 0, 0),
    (3, 1, 16, True, True, 160, 112, 4, 0), (4, 1, 128, True, False, 3840, 2160, 4, 0),
    (4, 1, 32, True, False, 200, 136, 4, 2), (6, 2, 32, True, True, 160, 112, 4, 2), (4, 1, 16, True, False, 200, 136, 0, 3),
    (8, 1, 128, True, False, 3840, 2160, 4, 0),
    # "drift": the camera turns by under a pixel per frame while the group keeps its still-camera mode
    # (tile-local front, no traced pixels to the tracers): reprojections round into the neighbouring
    # tiles, whose history validity the pure tracer takes from the rings (k_vring_pack)
    (3, 1, 32, True, "drift", 200, 136, 4, 0), (4, 1, 16, True, "drift", 200, 136, 0, 0)]
GROUP_SCENE = (1, 4, 3)  # bunny, 4 spp, diffuse_max_depth 3 (configs[2])
# BASELINE.json configs[3] and [4] as their own group shapes (scene, spp, diffuse_max_depth appended):
#   C4 vokselia 4K, 8 spp, saliency mask, one view tiled over 4 ranks;
#   C5 vokselia 4K, 8 spp GI 3, saliency mask, two eyes of 4 ranks each with the stereo composite.
# A still camera, so the tracers run the tile-local front with the saliency stencil's 4-px halo
# (FR/cuda/samplingStep.cu:186-199); the two chains as FR/main.cpp:336-355.
GROUP_CASES_CONFIGS = [
    pytest.param(4, 1, 128, True, False, 3840, 2160, 0, 0, (2, 8, 1), id="C4-vokselia-4K-8spp-saliency-4ranks",
                 marks=pytest.mark.timeout(600)),
    pytest.param(8, 2, 128, True, False, 3840, 2160, 0, 0, (2, 8, 3), id="C5-vokselia-stereo-4K-8spp-gi3-2x4ranks",
                 marks=pytest.mark.timeout(600)),
]


@pytest.mark.parametrize("R,V,tile,split,moving,W,H,mask,jfa,scn",
                         [c + (GROUP_SCENE,) for c in GROUP_CASES] + GROUP_CASES_CONFIGS)
def test_group_frames_equal_single_context(fovrt_mod, R, V, tile, split, moving, W, H, mask, jfa, scn):
    """fr_group_frame over R in-process ranks (V views of G = R / V): pipelined frames (no host sync but
    each rank's own front stages); with moving=True the camera pans every frame and every rank receives
    every other rank's traced pixels. Each view's reconstruction ranks hold the single-context frame's
    SHADING and history, view rank 0 its JFA / Sibson and the output rank its pull-push / A-Trous; the
    composite on rank 0 is the views' A-Trous images side by side."""
    import torch
    G = R // V
    scene, spp, dmd = scn
    mk = lambda: make_tracer(fovrt_mod, W, H, scene=scene, mask=mask, spp=spp, dmd=dmd)
    ranks = [mk() for _ in range(R)]
    fulls = [mk() for _ in range(V)]
    if G > 1:  # the group sums samples in fixed point (fr_group_config.sample_sum 2): the references too
        for f in fulls:
            f.set_sample_sum(2)
    cams = []
    for v in range(V):
        cam = fovrt_mod.Camera.preset(scene, W, H)
        cam.setPosition(np.asarray(cam.pos) + np.array([0.064 * (v - (V - 1) / 2), 0, 0], np.float32))
        cam.lookAt(cam.target)
        cams.append(cam)
    g = fovrt_mod.Group(ranks, views=V, tile=tile, split_recon=split, moving_camera=moving is True, composite=True,
                        jfa_ranks=jfa)
    info = [g.rank_info(i) for i in range(R)]
    assert sum(i["tiles"] for i in info[:G]) == ((W + tile - 1) // tile) * ((H + tile - 1) // tile)
    for f in range(4):
        for v in range(V):
            if moving:
                cams[v].setPrevState()
                step = [0.02, 0.01, 0.0] if moving is True else [0.025, 0.0, 0.0]
                cams[v].lookAt(np.asarray(cams[v].target) + np.array(step, np.float32))
            fulls[v].update_optix_variables(cams[v])
            for r in range(v * G, (v + 1) * G):
                ranks[r].update_optix_variables(cams[v])
            fulls[v].frame(timing=False)
        g.frame(timing=(f == 2))
    g.synchronize()
    out = torch.empty(V * W * H * 4, dtype=torch.float32, device="cuda")
    g.composite(out.data_ptr(), out.numel() * 4)
    comp = out.cpu().numpy().reshape(H, V * W, 4)
    owners = g.tile_owners(W, H)
    own_px = np.repeat(np.repeat(owners, tile, 0), tile, 1)[:H, :W]
    n_foreign_src = 0  # tracers' own pixels whose history source lies in another rank's tiles
    for v in range(V):
        full = fulls[v]
        jfa_rank, at_rank = g.output_ranks(v)
        m = jfa if jfa else (2 if split and G >= 6 else 1)  # the turns: view rank 0, 2, 3, ... one frame each
        assert jfa_rank == v * G + (0 if 3 % m == 0 else 3 % m + 1) and at_rank == v * G + (1 if split and G > 1 else 0)
        for r in range(v * G, (v + 1) * G):
            ch = info[r]["chains"]
            if ch or moving is True:
                for tid in (TN.SHADING, TN.HISTORY_CACHE):
                    assert equal_nan(ranks[r].read(tid), full.read(tid)), (v, r, tid)
            else:  # a still camera's tracer runs a tile-local front: its own tiles equal the full frame
                sel = own_px == r - v * G
                assert equal_nan(ranks[r].read(TN.MASK)[sel], full.read(TN.MASK)[sel]), (v, r)
                assert equal_nan(ranks[r].read(TN.WEIGHT)[sel], full.read(TN.WEIGHT)[sel]), (v, r)
                # ... except the pixels whose history comes (reprojection rounded across a tile edge, possibly
                # through a chain of such pixels) from another rank's tiles: the receivers add that history
                # themselves (k_shard_unpack_active), nothing reads the tracer's value there
                # the history validity (.w > 0, which picks a traced pixel's seed) of the ring around its
                # tiles comes from the owners (k_vring_pack / unpack, FR_VRING = 2 pixels inside every tile)
                yy, xx = np.mgrid[0:H, 0:W]
                ring = ((xx % tile < 2) | (xx % tile >= tile - 2) | (yy % tile < 2) | (yy % tile >= tile - 2)) & ~sel
                vt, vf = ranks[r].read(TN.HISTORY_CACHE)[..., 3] > 0, full.read(TN.HISTORY_CACHE)[..., 3] > 0
                assert np.array_equal(vt[ring], vf[ring]), (v, r, int((vt[ring] != vf[ring]).sum()))
                # ... so every own pixel sees the one-GPU validity at its (still camera: adjacent) source
                wf = full.read(TN.WEIGHT).astype(np.float64)
                rnd = lambda a: np.clip(np.trunc(a + np.copysign(0.5, a)), 0, 2.0 ** 32 - 1)
                sx, sy = np.clip(rnd(wf[..., 0]), 0, W - 1).astype(int), np.clip(rnd(wf[..., 1]), 0, H - 1).astype(int)
                src_ok = sel & (wf[..., 2] > 0)
                assert (np.abs(sx - xx)[src_ok] <= 1).all() and (np.abs(sy - yy)[src_ok] <= 1).all()  # within the ring
                assert np.array_equal(vt[sy, sx][src_ok], vf[sy, sx][src_ok]), (v, r)
                n_foreign_src += int((src_ok & ~sel[sy, sx]).sum())
                if moving is False:  # (a drifting camera's history chains cross tiles frame after frame)
                    hsel = sel & ~foreign_history(full.read(TN.WEIGHT), sel)
                    assert hsel.sum() >= 0.99 * sel.sum()
                    for tid in (TN.SHADING, TN.HISTORY_CACHE):
                        assert equal_nan(ranks[r].read(tid)[hsel], full.read(tid)[hsel]), (v, r, tid)
                assert ranks[r].stats()["gbuffer_primary"] < full.stats()["gbuffer_primary"]
            if r == jfa_rank:
                for tid in (TN.JFA_COLOR, TN.SIBSON):
                    assert equal_nan(ranks[r].read(tid), full.read(tid)), (v, r, tid)
            if r == at_rank:
                for tid in (TN.PULLPUSH, TN.ATROUS):
                    assert equal_nan(ranks[r].read(tid), full.read(tid)), (v, r, tid)
        assert equal_nan(comp[:, v * W:(v + 1) * W], full.read(TN.ATROUS)), v
        chains = [info[r]["chains"] for r in range(v * G, (v + 1) * G)]
        assert chains[0] & 1 and any(c & 2 for c in chains)
    print("tracer pixels with a foreign history source:", n_foreign_src)
    if moving == "drift":  # reprojections round across tile edges: the case the rings exist for
        assert n_foreign_src > 0
    g.destroy()
    for t in ranks + fulls:
        t.destroy()


def test_group_one_rank_rccl(fovrt_mod):
    """A one-rank RCCL communicator (fr_rccl_unique_id / fr_rccl_comm_init) driving a group with the
    composite: the group frame equals fr_frame and the composite is the A-Trous image."""
    import torch
    W, H = 128, 96
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    full = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    uid = fovrt_mod.rccl_unique_id()
    assert len(uid) == 128
    g = fovrt_mod.Group.rccl(t, uid, 1, 0, composite=True)
    assert g.rank_info(0) == {"view": 0, "view_rank": 0, "chains": 3, "tiles": ((W + 127) // 128) * ((H + 127) // 128)}
    for _ in range(3):
        g.frame()
        full.frame(timing=False)
    out = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
    g.composite(out.data_ptr(), out.numel() * 4)
    for tid in (TN.SHADING, TN.SIBSON, TN.ATROUS):
        assert equal_nan(t.read(tid), full.read(tid)), tid
    assert equal_nan(out.cpu().numpy().reshape(H, W, 4), full.read(TN.ATROUS))
    g.destroy()


def test_frame_clock_and_shard_count_state(fovrt_mod):
    """fr_frame_clock: one latency per pipelined frame and one interval per pair of consecutive frames,
    all positive, the latency at least the serial frame's G-buffer-to-A-Trous span's order; more frames
    than the event ring (16) are harvested in order. fr_shard_counts refuses before a front stage has run
    under the current shard plan (no stale or uninitialised counts), and answers after one."""
    W, H = 128, 96
    t = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    t.frame_clock(True)
    for _ in range(40):
        t.frame(timing=False)
    lat, itv = t.frame_clock_read()
    assert lat.size == 40 and itv.size == 39
    assert (lat > 0).all() and (itv > 0).all() and np.isfinite(lat).all()
    t.frame_clock(False)
    lat, itv = t.frame_clock_read()
    assert lat.size == 0 and itv.size == 0
    t.set_shard(0, 2, 32)
    with pytest.raises(fovrt_mod.FovrtError) as e:
        t.shard_counts(2)
    assert e.value.code == fovrt_mod.FR_E_STATE
    t.frame(timing=False)
    t.synchronize()
    n = t.shard_counts(2)
    assert int(n[0]) == int(t.read(TN.MASK).sum()) and int(n[1]) > 0  # rank 0's own tiles are its mask
    t.set_shard(0, 3, 32)  # a new plan: the counts of the old one are gone
    with pytest.raises(fovrt_mod.FovrtError):
        t.shard_counts(3)
    t.destroy()


def test_snapshot_restore_reproduces_next_frame(fovrt_mod):
    """fr_snapshot / fr_restore: the temporal state a frame hands to the next (history and depth
    ping-pong, FR/PathTracer.cpp:226-238; the pull-push atlases the push reads across frames,
    FR/PullPushInterpolation.cpp:57-58; m_accumFrame; the camera) restored mid-sequence, into a fresh context
    and into the same one after it ran on, reproduces the next frame bit for bit: camera panning, gaze moving."""
    W, H = 320, 192
    a = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    cam = fovrt_mod.Camera.preset(1, W, H)
    gazes = [(W / 2 + 25 * np.cos(f), (H / 2 + 25 * np.sin(f)) / 1.25) for f in range(8)]

    def advance(t, f):
        t.update_optix_variables(cams[f])
        t.set_gaze(*gazes[f])
        t.frame(timing=False)

    cams = []  # every frame's camera (with its previous pose), so a frame can be replayed
    for f in range(8):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
        cams.append(copy.deepcopy(cam))
    for f in range(4):
        advance(a, f)
    snap = a.snapshot()
    advance(a, 4)
    outs = (TN.SHADING, TN.HISTORY_CACHE, TN.DEPTH_CACHE, TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS, TN.MASK)
    want = {tid: a.read(tid) for tid in outs}
    # a fresh context restored from the snapshot
    b = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    b.restore(snap)
    advance(b, 4)
    for tid in outs:
        assert equal_nan(b.read(tid), want[tid]), ("fresh context", tid)
    # the same context, restored after two more frames
    advance(a, 5)
    advance(a, 6)
    a.restore(snap)
    advance(a, 4)
    for tid in outs:
        assert equal_nan(a.read(tid), want[tid]), ("same context", tid)
    # a snapshot of another configuration is refused
    c = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=2, dmd=3)
    with pytest.raises(fovrt_mod.FovrtError):
        c.restore(snap)
    for t in (a, b, c):
        t.destroy()


@pytest.mark.parametrize("W,H,gaze_deg", [(320, 192, None), (640, 360, 180.0)])
def test_jfa_outputs_written_on_demand(fovrt_mod, monkeypatch, W, H, gaze_deg):
    """JumpFlooding leaves JFA_COORD unwritten: Sibson's run form reads the seeds from the final JFA state, and
    the context writes the image (from that state and JFA_COLOR) when something asks for it. Against contexts that
    write it every time (FOVRT_JFA_LAZY_OUTPUTS=0), bit for bit: the outputs after pipelined frames (Sibson's wide and
    big discs included: an off-centre gaze at 640x360), after the caller overwrote the JFA's input, and after
    trace-only frames."""
    monkeypatch.setenv("FOVRT_JFA_LAZY_OUTPUTS", "0")
    eager = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    monkeypatch.delenv("FOVRT_JFA_LAZY_OUTPUTS")
    lazy = make_tracer(fovrt_mod, W, H, scene=1, mask=4, spp=4, dmd=3)
    cam = fovrt_mod.Camera.preset(1, W, H)
    outs = (TN.JFA_COORD, TN.JFA_COLOR, TN.SIBSON, TN.PULLPUSH, TN.ATROUS, TN.SHADING)
    for f in range(4):
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
        for t in (eager, lazy):
            t.update_optix_variables(cam)
            if gaze_deg is not None:
                a = np.deg2rad(gaze_deg)
                t.set_gaze(W / 2 + 0.25 * H * np.cos(a), (H / 2 + 0.25 * H * np.sin(a)) / 1.25)
            t.frame(timing=False)
    for tid in outs:
        assert equal_nan(lazy.read(tid), eager.read(tid)), ("after frames", tid)
    # the JFA input overwritten by the caller before the owed outputs were read
    for t in (eager, lazy):
        t.frame(timing=False)
        t.write(TN.SHADING, np.zeros((H, W, 4), np.float32))
    for tid in (TN.JFA_COORD, TN.JFA_COLOR):
        assert equal_nan(lazy.read(tid), eager.read(tid)), ("after a SHADING write", tid)
    # trace-only frames: the slot holding the JFA's input comes round again
    for t in (eager, lazy):
        t.frame(timing=False)
        for _ in range(4):
            t.trace_frame(timing=False)
    for tid in (TN.JFA_COORD, TN.JFA_COLOR):
        assert equal_nan(lazy.read(tid), eager.read(tid)), ("after trace-only frames", tid)
    eager.destroy()
    lazy.destroy()
