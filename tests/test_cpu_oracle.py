"""CPU suite: the oracle against independent restatements, known-answer tests and golden fixtures.

The reference ships no tests or fixtures and cannot run here, so the oracle is
pinned by (1) hand-derived known answers, (2) independent pure-Python / numpy restatements of the
same reference files, (3) brute-force ray casting, and (4) the committed golden vectors that the
GPU path is also held to (tests/golden/make_golden.py regenerates them).
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, equal_nan, jfa_np, logpolar_mask_np, rnd_py, sparse_image, tea16_py


def test_tea16_matches_python(oracle):
    for a, b in [(0, 0), (1, 0), (12345, 7), (0xFFFFFFFF, 0xFFFFFFFF), (3840 * 1080 + 1920, 41)]:
        assert oracle.tea16(a, b) == tea16_py(a, b)


def test_rnd_sequence_matches_python(oracle):
    for seed in (0, 1, 0xDEADBEEF, oracle.tea16(77, 3)):
        ref, _ = rnd_py(seed, 16)
        assert np.array_equal(oracle.rnd_seq(seed, 16), ref)
    # rnd = lcg / 2^24 lies in [0, 1) and hits exactly 0 for lcg == 0
    assert (oracle.rnd_seq(123, 1000) < 1.0).all()


def test_tonemap_known_answers(oracle):
    # Uncharted2ToneMapping (shared_helper_funcs.h:354-373): U(2c) / U(11.2), then pow 2.2.
    f = np.float32

    def U(x):
        A, B, C, D, E, F = f(0.15), f(0.5), f(0.1), f(0.2), f(0.02), f(0.3)
        return ((x * (A * x + C * B) + D * E) / (x * (A * x + B) + D * F)) - E / F

    vals = np.array([[0.0, 0.1, 1.0], [10.0, 0.5, 2.0], [5.0, 5.0, 5.0]], np.float32)
    ref = np.power(U(f(2.0) * vals) * (f(1.0) / U(f(11.2))), f(2.2), dtype=np.float32)
    got = oracle.tonemap(vals)
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-7, equal_nan=True)
    assert got[2, 0] == got[2, 1] == got[2, 2]
    assert got[1, 0] > got[0, 2] > got[0, 1]  # monotone in the input
    assert got[1, 0] > 1.0  # "gamma" is pow 2.2 (App. A #6): values above the white point exceed 1


def test_oracle_bvh_equals_brute_force(oracle, fovrt_mod):
    cfg = fovrt_mod.Config(scene=fovrt_mod.SCENE_BUNNY, texture_mode=1, detail=1)
    a = fovrt_mod.Scene(cfg).arrays()
    sc = oracle.OracleScene(a)
    rng = np.random.default_rng(3)
    n = 3000
    o = rng.uniform(-4, 4, (n, 3)); o[:, 1] = rng.uniform(0.05, 3, n)
    # aim half of the rays at the bunny / earth, half uniformly
    tgt = np.where(rng.random((n, 1)) < 0.5, np.array([[-1.5, 0.7, 1.2]]), np.array([[0.0, 1.0, 0.0]]))
    d = tgt + rng.normal(scale=0.3, size=(n, 3)) - o
    d[: n // 4] = rng.normal(size=(n // 4, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.full((n, 1), 1e-3), np.full((n, 1), np.inf)], 1).astype(np.float32)
    A, B = sc.closest(rays), sc.closest(rays, brute=True)
    assert (A[:, 1] >= 0).sum() > n // 3
    assert np.array_equal(A, B)


def test_oracle_jfa_matches_numpy_restatement(oracle):
    W, H = 48, 40
    rng = np.random.default_rng(5)
    for density in (0.0, 0.02, 0.1, 1.0):
        mask = (rng.random((H, W)) < density).astype(np.uint8)
        img = sparse_image(W, H, mask)
        c, col = oracle.jfa(img)
        c2, col2 = jfa_np(img)
        assert equal_nan(c, c2) and equal_nan(col, col2), density


def test_logpolar_mask_matches_numpy_restatement(oracle, fovrt_mod):
    W, H = 128, 96
    cfg = fovrt_mod.Config(scene=fovrt_mod.SCENE_BOX, texture_mode=1)
    sc = oracle.OracleScene(fovrt_mod.Scene(cfg).arrays())
    cam = fovrt_mod.Camera.preset(fovrt_mod.SCENE_BOX, W, H).uniforms(W, H)
    z = np.zeros((H, W, 4), np.float32)
    out = oracle.sampling(sc, cam, W, H, 1, z, z, z, z, z, z)
    ref = logpolar_mask_np(W, H, cam.gaze[0], cam.gaze[1])
    assert np.array_equal(out["mask"], ref)
    assert 0.03 < out["mask"].mean() < 0.08  # literal uint2 arithmetic: ~5% density
    out = oracle.sampling(sc, cam, W, H, 4, z, z, z, z, z, z)
    ref = logpolar_mask_np(W, H, cam.gaze[0], cam.gaze[1], signed=True)
    assert np.array_equal(out["mask"], ref)
    assert 0.09 < out["mask"].mean() < 0.13  # signed differences: the ~10% of SURVEY §8(a) row 5b


def test_warp_sort_permutation(oracle):
    rng = np.random.default_rng(9)
    for (W, H, p) in [(16, 8, 0.3), (33, 17, 0.05), (8, 8, 0.0), (8, 8, 1.0)]:
        mask = (rng.random((H, W)) < p).astype(np.uint8)
        n, tb = oracle.warp_sort(mask)
        assert n == int(mask.sum())  # ray_count (warpSort.cu:76-82)
        # a permutation of the pixels, with the active flag preserved (z > 0 <=> active)
        xy = tb[..., :2].reshape(-1, 2)
        assert len({(int(a), int(b)) for a, b in xy}) == W * H
        act = tb[..., 2].reshape(-1) > 0
        assert act.sum() == n
        assert all(mask[int(b), int(a)] == 1 for (a, b), f in zip(xy, act) if f)


@pytest.mark.parametrize("name", ["jfa_64x48", "pullpush_64", "sibson_64x48", "atrous_32", "logpolar_512", "kat"])
def test_oracle_matches_golden(oracle, name):
    path = os.path.join(GOLDEN, name + ".npz")
    g = np.load(path)
    if name.startswith("jfa"):
        c, col = oracle.jfa(g["input"])
        assert equal_nan(c, g["coord"]) and equal_nan(col, g["color"])
    elif name.startswith("pullpush"):
        st = oracle.PullPushState(g["inputs"].shape[2], g["inputs"].shape[1])
        for k in range(g["inputs"].shape[0]):
            assert equal_nan(st.render(g["inputs"][k]), g["outputs"][k]), k
    elif name.startswith("sibson"):
        assert equal_nan(oracle.sibson(g["coord"], g["color"]), g["output"])
    elif name.startswith("atrous"):
        out = oracle.atrous(int(g["count"]), g["pos"], g["nrm"], g["col"])
        assert np.allclose(out, g["output"], rtol=0, atol=1e-6)
    elif name.startswith("logpolar"):
        H, W = g["mask"].shape
        assert np.array_equal(logpolar_mask_np(W, H, float(g["gaze"][0]), float(g["gaze"][1])), g["mask"])
    else:
        assert [oracle.tea16(int(a), int(b)) for a, b in g["tea_in"]] == list(g["tea_out"])
        assert np.array_equal(oracle.rnd_seq(int(g["rnd_seed"]), len(g["rnd_out"])), g["rnd_out"])
        assert np.allclose(oracle.tonemap(g["tm_in"]), g["tm_out"], rtol=1e-6, atol=0)


def _sqrt_le_bound(d):
    """numpy mirror of k_image.hip sqrt_le_bound: the largest float32 x with sqrtf(x) <= d."""
    f32 = np.float32
    c = f32(d) * f32(d)
    while c > 0 and np.sqrt(c) > d:
        c = np.nextafter(c, f32(0))
    while True:
        n = np.nextafter(c, f32(np.inf))
        if not np.sqrt(n) <= d:
            return c
        c = n


def test_sqrt_free_disc_test_is_exact():
    """Sibson's disc test 'sqrtf(r2) > d' is replaced by 'r2 > sqrt_le_bound(d)' (k_image.hip):
    equivalent for every float32 r2 >= 0 because sqrtf is correctly rounded and monotone. Checked
    here on the ulps around d*d and on random values."""
    rs = np.random.RandomState(3)
    ds = np.concatenate([rs.rand(300).astype(np.float32) * np.float32(0.01),
                         np.float32([0.0, 1e-20, 2.6e-4, 1.0, 3.0])])
    for d in ds:
        d = np.float32(d)
        b = _sqrt_le_bound(d)
        c = np.float32(d * d)
        probe = [c, b] + [np.nextafter(c, np.float32(np.inf)) for _ in range(1)]
        x = c
        for _ in range(8):
            x = np.nextafter(x, np.float32(0)); probe.append(x)
        x = c
        for _ in range(8):
            x = np.nextafter(x, np.float32(np.inf)); probe.append(x)
        probe += list((rs.rand(50) * 4 * float(c) + 1e-30).astype(np.float32))
        for r2 in probe:
            r2 = np.float32(r2)
            assert (np.sqrt(r2) > d) == (r2 > b), (d, r2, b)


# ---------------------------------------------------------------------------------------------
# Pull-push and A-Trous: the oracle against independent numpy restatements written from the
# reference's GLSL (tests/helpers.py), so the GPU's bit-exact pull-push and its A-Trous tolerance
# rest on two restatements of the shaders, not on the oracle alone (parity is still unpinned
# against the reference itself: it cannot run here and ships no outputs).
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("W,H", [(16, 16), (32, 32), (24, 20), (1, 1), (64, 40)])
def test_pullpush_oracle_equals_numpy_restatement(oracle, W, H):
    from helpers import PullPushNp
    rng = np.random.default_rng(W * 7 + H)
    ref, mine = oracle.PullPushState(W, H), PullPushNp(W, H)
    for k, p in enumerate((0.1, 0.02, 0.4, 0.0, 1.0)):  # atlases carry state across frames
        img = sparse_image(W, H, (rng.random((H, W)) < p).astype(np.uint8), seed=k)
        a, b = ref.render(img), mine.render(img)
        assert equal_nan(a, b), (k, np.argwhere(~np.isclose(a, b, rtol=0, atol=0, equal_nan=True))[:4])
        assert equal_nan(ref.push, mine.push) and equal_nan(ref.pull, mine.pull)


@pytest.mark.parametrize("W,H,count", [(32, 24, 1), (40, 33, 2), (17, 9, 3)])
def test_atrous_oracle_matches_numpy_restatement(oracle, W, H, count):
    from helpers import atrous_np
    rng = np.random.default_rng(W + H + count)
    pos = rng.normal(size=(H, W, 4)).astype(np.float32) * np.float32(0.3)
    pos[..., 3] = 1.0
    nrm = rng.random((H, W, 4), dtype=np.float32)
    nrm[..., 3] = (rng.random((H, W)) < 0.5).astype(np.float32)
    col = rng.random((H, W, 4), dtype=np.float32)
    got = oracle.atrous(count, pos, nrm, col)
    ref = atrous_np(count, pos, nrm, col)
    assert np.abs(got - ref).max() <= 2e-6, np.abs(got - ref).max()


# ---------------------------------------------------------------------------------------------
# Second restatements (numpy float32, written from the reference text) of the stages only the oracle
# pinned before: sampling_step's saliency + masked_sampling, and Sibson. Bit-for-bit agreement.
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene,W,H,mask_mode,gaze_shift", [(1, 64, 64, 0, (0, 0)), (2, 96, 64, 0, (0, 0)),
                                                            (2, 128, 128, 0, (30, -20)), (1, 100, 70, 0, (-60, 25)),
                                                            (0, 64, 48, 0, (0, 0)), (2, 96, 64, 4, (5, 5)),
                                                            (1, 64, 64, 2, (0, 0))])
def test_sampling_matches_numpy_restatement(oracle, fovrt_mod, scene, W, H, mask_mode, gaze_shift):
    """oracle.sampling (the C++ restatement) against helpers.sampling_np (numpy, from samplingStep.cu and
    shared_helper_funcs.h) on the oracle's own G-buffer of two frames (the second has a depth cache, so
    the reprojection-validity path runs), with the reprojection uv perturbed on some pixels (velocity,
    off-screen and negative uv) and the gaze moved off centre: mask, weight and heat map bit-identical."""
    from helpers import sampling_np
    arrays = fovrt_mod.Scene(fovrt_mod.Config(scene=scene, texture_mode=1, detail=1)).arrays()
    osc = oracle.OracleScene(arrays)
    cam = fovrt_mod.Camera.preset(scene, W, H)
    uni = cam.uniforms(W, H)
    uni.gaze[0] += np.float32(gaze_shift[0])
    uni.gaze[1] += np.float32(gaze_shift[1])
    rng = np.random.default_rng(W + H + scene)
    g0 = oracle.gbuffer(osc, uni, W, H, 0)
    g1 = oracle.gbuffer(osc, uni, W, H, 1)
    weight = g1["weight"].copy()
    pick = rng.random((H, W)) < 0.2
    weight[pick, 0] += rng.normal(scale=3.0, size=pick.sum()).astype(np.float32)
    weight[pick, 1] += rng.normal(scale=3.0, size=pick.sum()).astype(np.float32)
    neg = rng.random((H, W)) < 0.03
    weight[neg, :2] = -1.0
    n_valid_total = 0
    for frame, g, dc in ((0, g0, np.zeros_like(g0["depth"])), (1, g1, g0["depth"])):
        w_in = weight if frame == 1 else g["weight"]
        ref = oracle.sampling(osc, uni, W, H, mask_mode, g["position"], g["depth"], dc, w_in, g["normal"],
                              g["diffuse"])
        prev_eye = np.array(uni.prev_eye[:], np.float32)
        m, w, e = sampling_np(W, H, mask_mode, (uni.gaze[0], uni.gaze[1]), prev_eye, arrays["bbox"], g["position"],
                              g["depth"], dc, w_in, g["normal"], g["diffuse"])
        assert np.array_equal(m, ref["mask"]), (frame, np.argwhere(m != ref["mask"])[:5])
        assert equal_nan(w, ref["weight"]), frame
        assert equal_nan(e, ref["extra"]), (frame, np.argwhere(~np.isclose(e, ref["extra"], rtol=0, atol=0,
                                                                             equal_nan=True))[:5])
        n_valid_total += int((w[..., 2] == 1).sum())
    assert n_valid_total > 0  # the cache-hit path ran
    if mask_mode == 0:
        assert 0 < ref["mask"].mean() < 1


@pytest.mark.parametrize("W,H,density", [(64, 64, 0.1), (96, 64, 0.03), (128, 128, 0.1), (40, 33, 0.5),
                                         (64, 48, "single")])
def test_sibson_matches_numpy_restatement(oracle, W, H, density):
    """oracle.sibson against helpers.sibson_np (numpy, from sibsonFS.glsl:16-49) on the oracle's JFA
    output of sparse images: bit-identical, including pixels whose disc wraps past the border (REPEAT)
    and seed pixels (radius 0: the seed colour itself)."""
    from helpers import sibson_np
    rng = np.random.default_rng(W * 7 + H)
    if density == "single":
        m = np.zeros((H, W), np.uint8)
        m[H // 3, W - 1] = 1
    else:
        m = (rng.random((H, W)) < density).astype(np.uint8)
    img = sparse_image(W, H, m, seed=W)
    coord, color = oracle.jfa(img)
    ref = oracle.sibson(coord, color)
    got = sibson_np(coord, color)
    assert equal_nan(got, ref), np.argwhere(~np.isclose(got, ref, rtol=0, atol=0, equal_nan=True))[:5]
