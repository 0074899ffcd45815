"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact for every integer/byte output (disparity int16, u8 maps, HOG histograms) and for
the float32 post-processing (identical op order, -ffp-contract=off); Harris within the
north_star tolerance 1e-4 (absolute).  Small sizes run the NumPy oracle, large sizes the C
oracle; full benchmark sizes add size-independent properties.
"""
import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair, to_bgr

pytestmark = pytest.mark.gpu

HARRIS_TOL = 1e-4


def _pair(H, W, D, seed, min_disp=0):
    L, R, _ = stereo_pair(H, W, max(16, D), seed, max(0, min_disp))
    return L, R


@pytest.mark.parametrize("cost", ["sad", "ssd"])
@pytest.mark.parametrize("D,win", [(16, 1), (32, 3), (48, 5), (64, 9), (96, 5), (128, 11),
                                   (160, 7), (256, 15), (320, 7)])
def test_disparity_matches_oracle(engine, cost, D, win):
    if cost == "ssd" and D > 256 and win >= 13:
        pytest.skip("SSD key range")
    H, W = 37, 400
    L, R = _pair(H, W, D, seed=D + win)
    got = engine.disparity(L, R, 0, D, win, cost)
    exp = C.disparity16(L, R, 0, D, win, 0 if cost == "sad" else 1)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("min_disp", [-16, -5, 3, 17])
def test_disparity_min_disp_offsets(engine, min_disp):
    L, R = _pair(29, 300, 64, seed=11)
    got = engine.disparity(L, R, min_disp, 64, 7)
    np.testing.assert_array_equal(got, O.disparity16(L, R, min_disp, 64, 7))


@pytest.mark.parametrize("H,W", [(1, 200), (2, 129), (5, 64), (7, 65), (64, 63), (3, 1000)])
def test_disparity_ragged_shapes(engine, H, W):
    rng = np.random.default_rng(H * 1000 + W)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    for D, win in [(16, 3), (64, 9)]:
        np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win),
                                      O.disparity16(L, R, 0, D, win))


@pytest.mark.parametrize("win", [5, 7, 9, 11, 13, 15])
@pytest.mark.parametrize("H", [1, 2, 3, 5, 6, 7, 13])
def test_four_row_kind_every_height_and_window(engine, win, H):
    """The 4-rows-per-wave SAD kind (win >= 5): heights that leave 1-3 rows in the last
    wave, every supported window radius, a negative min_disp."""
    rng = np.random.default_rng(win * 100 + H)
    W = 173
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    for min_disp, D in [(0, 48), (-5, 64)]:
        np.testing.assert_array_equal(engine.disparity(L, R, min_disp, D, win),
                                      O.disparity16(L, R, min_disp, D, win))


@pytest.mark.parametrize("win", [5, 7, 9, 11, 13, 15])
@pytest.mark.parametrize("D", [4, 50, 64, 100, 127, 128, 200, 256])
def test_ring_kind_disparity_counts(engine, D, win):
    """The cost-ring SAD kind (win 5..11, D <= 256; win 13/15 with D % 4 == 0 and a ring of
    16-bit packed column costs): lanes of 4 disparities with padding inside a lane
    (D % 4 != 0), padding lanes re-matching the last group (win 13/15), 16/32/64 lanes per
    group, several segments per row and a ragged last segment, negative min_disp."""
    rng = np.random.default_rng(D * 10 + win)
    H, W = 11, 1333
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = np.roll(L, -(D // 3), axis=1) ^ rng.integers(0, 8, (H, W), dtype=np.uint8)
    for min_disp in (0, -3):
        np.testing.assert_array_equal(engine.disparity(L, R, min_disp, D, win),
                                      C.disparity16(L, R, min_disp, D, win, 0))


def test_disparity_image_narrower_than_band(engine):
    L, R = _pair(20, 50, 64, seed=3)
    got = engine.disparity(L, R, 0, 64, 5)
    assert (got == -16).all()
    np.testing.assert_array_equal(got, O.disparity16(L, R, 0, 64, 5))


def test_flat_images_tie_to_min_disp(engine):
    L = np.full((40, 300), 77, np.uint8)
    got = engine.disparity(L, L.copy(), 4, 48, 9)
    exp = O.disparity16(L, L, 4, 48, 9)
    np.testing.assert_array_equal(got, exp)
    assert (got[:, 52:] == 4 * 16).all()


@pytest.mark.parametrize("D,win", [(200, 15), (68, 13), (256, 15)])
def test_ring_packed_ties_go_to_the_real_lowest_disparity(engine, D, win):
    # flat images: every disparity ties, including the padding lanes' re-matched group
    L = np.full((21, 700), 140, np.uint8)
    got = engine.disparity(L, L.copy(), -2, D, win)
    np.testing.assert_array_equal(got, O.disparity16(L, L, -2, D, win))
    valid = got != -3 * 16
    assert valid.sum() > 0 and (got[valid] == -2 * 16).all()


def test_extreme_contrast_no_overflow(engine):
    # alternating 0/255 columns make every SAD/SSD tap maximal
    L = np.tile(np.array([0, 255], np.uint8), (24, 160))
    R = np.roll(L, 1, axis=1)
    for cost, D, win in [("sad", 128, 15), ("sad", 256, 15), ("sad", 64, 13), ("ssd", 256, 15), ("ssd", 64, 15)]:
        np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win, cost),
                                      C.disparity16(L, R, 0, D, win, 0 if cost == "sad" else 1))


def test_integer_shift_recovered_exactly(engine):
    rng = np.random.default_rng(5)
    for shift in (0, 7, 31, 63):
        L = rng.integers(0, 256, (48, 320), dtype=np.uint8)
        R = np.roll(L, -shift, axis=1)
        got = engine.disparity(L, R, 0, 64, 9) // 16
        # away from the wrap-around seam every valid pixel recovers the shift
        assert (got[:, 64:320 - shift - 8] == shift).all()


@pytest.mark.parametrize("D,win", [(64, 9), (32, 15), (256, 15), (96, 5)])
def test_hog_cost_matches_oracle(engine, D, win):
    L, R = _pair(33, 330, D, seed=7 * D + win)
    got = engine.disparity(L, R, 0, D, win, "hog")
    np.testing.assert_array_equal(got, C.disparity16(L, R, 0, D, win, 2))


@pytest.mark.parametrize("win", [1, 3, 9, 15])
def test_hog_hist_matches_oracle(engine, win):
    L, _ = _pair(45, 150, 32, seed=win)
    np.testing.assert_array_equal(engine.hog_hist(L, win), O.hog_hist(L, win))


@pytest.mark.parametrize("H,W,win", [(1, 1, 3), (2, 70, 15), (150, 211, 15), (131, 64, 13), (97, 130, 5),
                                     (70, 51, 1), (65, 300, 7), (40, 1000, 15), (37, 993, 9), (70, 497, 3),
                                     (33, 1489, 7), (5, 2000, 1), (66, 1100, 11), (9, 496, 15), (3, 504, 13),
                                     (11, 241, 15), (12, 481, 11), (13, 249, 9), (7, 248, 5), (8, 257, 1)])
def test_hog_hist_strip_shapes(engine, H, W, win):
    """The column-run kernel: waves of 240 / 248 / 256 columns (4 columns per lane, 2 / 1 / 0
    halo lanes a side), 24-row strips, images narrower than a wave or than the window, widths
    one past a wave / ending in a halo lane, 1-pixel images (reflect-101 of size 1)."""
    rng = np.random.default_rng(H * 1000 + W + win)
    g = rng.integers(0, 256, (H, W), dtype=np.uint8)
    g[:, ::7] = 255                      # strong edges: large magnitudes in every bin
    np.testing.assert_array_equal(engine.hog_hist(g, win), O.hog_hist(g, win))


@pytest.mark.parametrize("win", [1, 3, 5, 7, 9, 11, 13, 15])
def test_hog_hist_dev_row_bands_every_radius(engine, win):
    """sv_hog_hist_dev over row bands [row0, row1) at every radius (0..7: 0, 1 and 2 halo
    lanes a side), an image 2.5 waves wide with a pitch > W: the band's rows bit-exact, the
    rows outside it untouched (sentinel)."""
    H, W, pitch = 75, 600, 616
    rng = np.random.default_rng(win)
    g = rng.integers(0, 256, (H, W), dtype=np.uint8)
    g[:, ::11] = 255
    img = np.zeros((H, pitch), np.uint8)
    img[:, :W] = g
    exp = O.hog_hist(g, win)                                   # [9, H, W]
    dimg = engine.dev_alloc(img.nbytes)
    dout = engine.dev_alloc(H * W * 20)
    try:
        engine.to_device(dimg, img)
        for row0, row1 in ((0, H), (17, 53), (74, 75), (0, 1)):
            engine.to_device(dout, np.full((H, W, 10), 0xBEEF, np.uint16))
            engine.hog_hist_dev(dimg, H, W, pitch, win, row0, row1, dout)
            engine.synchronize()
            got = engine.to_host(dout, (H, W, 10), np.uint16)
            np.testing.assert_array_equal(got[row0:row1, :, :9].transpose(2, 0, 1), exp[:, row0:row1])
            assert (got[row0:row1, :, 9] == 0).all()              # the pad bin
            assert (got[:row0] == 0xBEEF).all() and (got[row1:] == 0xBEEF).all()
    finally:
        engine.dev_free(dimg)
        engine.dev_free(dout)


def test_harris_within_tolerance(engine):
    for H, W, seed in [(50, 70, 0), (1, 40, 1), (17, 1, 2), (128, 300, 3)]:
        rng = np.random.default_rng(seed)
        g = rng.integers(0, 256, (H, W), dtype=np.uint8)
        got = engine.harris(g)
        exp = O.harris(g)
        assert np.abs(got - exp).max() <= HARRIS_TOL
    flat = np.full((32, 32), 9, np.uint8)
    assert np.abs(engine.harris(flat)).max() == 0.0


def test_harris_output_of_disparity_call(engine):
    L, R = _pair(40, 260, 64, seed=2)
    d16, hr = engine.disparity(L, R, 0, 64, 9, harris=True)
    np.testing.assert_array_equal(d16, O.disparity16(L, R, 0, 64, 9))
    assert np.abs(hr - O.harris(L)).max() <= HARRIS_TOL


def test_gray_matches_opencv_fixed_point(engine):
    rng = np.random.default_rng(1)
    bgr = rng.integers(0, 256, (31, 77, 3), dtype=np.uint8)
    np.testing.assert_array_equal(engine.gray(bgr), O.bgr_to_gray(bgr))


def test_median5_f32(engine):
    rng = np.random.default_rng(2)
    a = rng.normal(size=(23, 91)).astype(np.float32)
    np.testing.assert_array_equal(engine.median5(a), O.median5(a))


def test_posts_match_reference_numpy(engine):
    rng = np.random.default_rng(3)
    d = (rng.integers(-16, 64 * 16, (40, 50)) / 16).astype(np.float32)
    for lo, hi in [(0.3, 2.0), (0.2, 4.0), (0.1, 0.5)]:
        df, nm = engine.depth_post(d, lo, hi)
        edf, enm = O.depth_post(d, lo, hi)
        np.testing.assert_array_equal(df, edf)
        np.testing.assert_array_equal(nm, enm)
    dn, du, cf = engine.scaled_post(d, 0, 64)
    edn, edu, ecf = O.scaled_post(d, 0, 64)
    np.testing.assert_array_equal(dn, edn)
    np.testing.assert_array_equal(du, edu)
    np.testing.assert_array_equal(cf, ecf)


def test_depth_map_path_bgr(engine):
    L, R = _pair(60, 300, 64, seed=4)
    bl, br = to_bgr(L), to_bgr(R)
    depth, disp, norm = engine.depth_map(bl, br, 0, 64, 9, 0.3, 2.0)
    e_depth, e_disp, e_norm = O.create_depth_map(bl, br, 0, 64, 9, 0.3, 2.0)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


def test_stereo_scaled_path(engine):
    L, R = _pair(60, 300, 96, seed=5)
    dn, disp, du, cf = engine.stereo_scaled(to_bgr(L), to_bgr(R), 0, 96, 5)
    e = O.create_depth_map_stereo_scaled(to_bgr(L), to_bgr(R), 0, 96, 5)
    for got, exp in zip((dn, disp, du, cf), e):
        np.testing.assert_array_equal(got, exp)


def test_full_hd_metric_config_against_c_oracle(engine):
    """BASELINE metric config: 1920x1080, D=128, win=9 (bit-exact vs the C oracle)."""
    L, R, gt = stereo_pair(1080, 1920, 128, seed=0)
    got = engine.disparity(L, R, 0, 128, 9)
    exp = C.disparity16(L, R, 0, 128, 9, 0)
    np.testing.assert_array_equal(got, exp)
    # property: the background plane (d = D/4) is recovered exactly away from edges
    assert (got[20:250, 300:600] == 32 * 16).mean() > 0.99


def test_full_hd_c3_config_11x11(engine):
    L, R, _ = stereo_pair(1080, 1920, 128, seed=1)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, 128, 11),
                                  C.disparity16(L, R, 0, 128, 11, 0))


def test_vga_stream_config_with_harris(engine):
    """C2: 640x480 D=64 win=9 + Harris, several frames."""
    for seed in range(3):
        L, R, _ = stereo_pair(480, 640, 64, seed=seed)
        d16, hr = engine.disparity(L, R, 0, 64, 9, harris=True)
        np.testing.assert_array_equal(d16, C.disparity16(L, R, 0, 64, 9, 0))
        assert np.abs(hr - C.harris(L)).max() <= HARRIS_TOL


# ---- row tiling, device API, golden fixtures, torch-first runtime ------------------------
GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "golden_v1.npz")


def test_golden_fixtures_on_gpu(engine):
    g = np.load(GOLDEN)
    names = sorted({k.split("_")[0] for k in g.files if k.endswith("_params")})
    for n in names:
        L, R = g[f"{n}_left"], g[f"{n}_right"]
        mn, D, win = (int(v) for v in g[f"{n}_params"])
        for cname in ("sad", "ssd", "hog"):
            np.testing.assert_array_equal(engine.disparity(L, R, mn, D, win, cname), g[f"{n}_d16_{cname}"])
        depth, disp, norm = engine.depth_map(L, R, mn, D, win, 0.3, 2.0)
        np.testing.assert_array_equal(disp, g[f"{n}_disparity"])
        np.testing.assert_array_equal(depth, g[f"{n}_depth_final"])
        np.testing.assert_array_equal(norm, g[f"{n}_depth_norm"])
        assert np.abs(engine.harris(L) - g[f"{n}_harris"]).max() <= HARRIS_TOL
        np.testing.assert_array_equal(engine.hog_hist(L, win), g[f"{n}_hog"])
    np.testing.assert_array_equal(engine.gray(g["gray_bgr"]), g["gray_out"])


@pytest.mark.parametrize("cost,win", [("sad", 9), ("sad", 11), ("ssd", 7), ("hog", 15)])
def test_row_bands_reassemble_bit_exactly_on_gpu(engine, cost, win):
    L, R, _ = stereo_pair(131, 700, 128, seed=21)
    full = engine.disparity(L, R, 0, 128, win, cost)
    for world in (2, 3, 8):
        out = np.zeros_like(full)
        for k in range(world):
            r0, r1 = 131 * k // world, 131 * (k + 1) // world
            engine.disparity_rows(L, R, 0, 128, win, r0, r1, cost, out=out)
        np.testing.assert_array_equal(out, full)


def test_device_api_band_pipeline(engine):
    """sv_disparity_dev + sv_median_rows_dev over row bands == the host depth_map path."""
    H, W, D, win = 70, 400, 64, 9
    L, R, _ = stereo_pair(H, W, D, seed=5)
    e_depth, e_disp, e_norm = engine.depth_map(L, R, 0, D, win, 0.3, 2.0)
    dL, dR = engine.dev_alloc(H * W), engine.dev_alloc(H * W)
    d16 = engine.dev_alloc(H * W * 2)
    ddisp, ddepth, dnorm = engine.dev_alloc(H * W * 4), engine.dev_alloc(H * W * 4), engine.dev_alloc(H * W)
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        for k in range(3):
            r0, r1 = H * k // 3, H * (k + 1) // 3
            h0, h1 = max(0, r0 - 2), min(H, r1 + 2)
            engine.disparity_dev(dL, dR, H, W, W, 0, D, win, "sad", h0, h1, d16, W)
            engine.median_post_dev(d16, H, W, r0, r1, 1, ddisp, ddepth, dnorm,
                                   min_depth=0.3, max_depth=2.0, min_disp_global=0)
        np.testing.assert_array_equal(engine.to_host(ddisp, (H, W), np.float32), e_disp)
        np.testing.assert_array_equal(engine.to_host(ddepth, (H, W), np.float32), e_depth)
        np.testing.assert_array_equal(engine.to_host(dnorm, (H, W), np.uint8), e_norm)
        # whole device path in one call
        engine.depth_map_dev(dL, dR, H, W, W, 0, D, win, 0.3, 2.0, ddepth, ddisp, dnorm)
        np.testing.assert_array_equal(engine.to_host(ddepth, (H, W), np.float32), e_depth)
    finally:
        for p in (dL, dR, d16, ddisp, ddepth, dnorm):
            engine.dev_free(p)


@pytest.mark.parametrize("cost,win", [("sad", 9), ("sad", 11), ("ssd", 5), ("hog", 7), ("hog", 15), ("hog", 1)])
def test_frame_batch_matches_single_frames(engine, cost, win):
    """sv_*_batch_dev (one launch over grid.z) == the per-frame oracle, frame by frame,
    with a padded input frame stride and a padded output pitch."""
    nf, H, W, D = 3, 37, 300, 64
    pitch, fstride = W + 16, (W + 16) * H + 64
    pairs = [stereo_pair(H, W, D, seed=40 + z)[:2] for z in range(nf)]
    hL = np.zeros(nf * fstride, np.uint8)
    hR = np.zeros(nf * fstride, np.uint8)
    for z, (L, R) in enumerate(pairs):
        hL[z * fstride: z * fstride + pitch * H].reshape(H, pitch)[:, :W] = L
        hR[z * fstride: z * fstride + pitch * H].reshape(H, pitch)[:, :W] = R
    opitch, ofs = W + 8, (W + 8) * H + 40
    dL, dR = engine.dev_alloc(hL.nbytes), engine.dev_alloc(hR.nbytes)
    d16 = engine.dev_alloc(nf * ofs * 2)
    try:
        engine.to_device(dL, hL)
        engine.to_device(dR, hR)
        engine.disparity_batch_dev(dL, dR, nf, H, W, pitch, fstride, 0, D, win, cost, d16, opitch, ofs)
        out = engine.to_host(d16, (nf * ofs,), np.int16)
        for z, (L, R) in enumerate(pairs):
            got = out[z * ofs: z * ofs + opitch * H].reshape(H, opitch)[:, :W]
            ref = C.disparity16(L, R, 0, D, win, {"sad": 0, "ssd": 1, "hog": 2}[cost])
            np.testing.assert_array_equal(got, ref, err_msg=f"frame {z}")
    finally:
        for p in (dL, dR, d16):
            engine.dev_free(p)


def test_depth_map_batch_dev_and_scaled_batch(engine):
    nf, H, W, D, win = 4, 45, 320, 64, 9
    pairs = [stereo_pair(H, W, D, seed=60 + z)[:2] for z in range(nf)]
    hL = np.stack([p[0] for p in pairs])
    hR = np.stack([p[1] for p in pairs])
    n = nf * H * W
    dL, dR = engine.dev_alloc(n), engine.dev_alloc(n)
    ddepth, ddisp, dnorm, dconf = (engine.dev_alloc(n * 4), engine.dev_alloc(n * 4),
                                   engine.dev_alloc(n), engine.dev_alloc(n * 4))
    d16 = engine.dev_alloc(n * 2)
    try:
        engine.to_device(dL, hL)
        engine.to_device(dR, hR)
        engine.depth_map_batch_dev(dL, dR, nf, H, W, W, H * W, 0, D, win, 0.3, 2.0, ddepth, ddisp, dnorm)
        depth = engine.to_host(ddepth, (nf, H, W), np.float32)
        disp = engine.to_host(ddisp, (nf, H, W), np.float32)
        norm = engine.to_host(dnorm, (nf, H, W), np.uint8)
        for z, (L, R) in enumerate(pairs):
            e = O.create_depth_map(L, R, 0, D, win, 0.3, 2.0)
            np.testing.assert_array_equal(depth[z], e[0], err_msg=f"frame {z}")
            np.testing.assert_array_equal(disp[z], e[1], err_msg=f"frame {z}")
            np.testing.assert_array_equal(norm[z], e[2], err_msg=f"frame {z}")
        # scaled post over the same batch of int16 maps (app 2)
        engine.disparity_batch_dev(dL, dR, nf, H, W, W, H * W, 0, D, win, "sad", d16, W, H * W)
        engine.median_post_batch_dev(d16, nf, H, W, 2, ddisp, ddepth, dnorm, dconf, min_disp=0, num_disp=D)
        a = engine.to_host(ddepth, (nf, H, W), np.float32)
        u8 = engine.to_host(dnorm, (nf, H, W), np.uint8)
        conf = engine.to_host(dconf, (nf, H, W), np.float32)
        for z, (L, R) in enumerate(pairs):
            e = O.create_depth_map_stereo_scaled(L, R, 0, D, win)
            np.testing.assert_array_equal(a[z], e[0], err_msg=f"frame {z}")
            np.testing.assert_array_equal(u8[z], e[2], err_msg=f"frame {z}")
            np.testing.assert_array_equal(conf[z], e[3], err_msg=f"frame {z}")
    finally:
        for p in (dL, dR, ddepth, ddisp, dnorm, dconf, d16):
            engine.dev_free(p)


@pytest.mark.parametrize("H,W", [(1, 1), (1, 70), (2, 3), (3, 65), (5, 64), (17, 130), (33, 63), (70, 129)])
def test_median_post_ragged_maps_and_bands(engine, H, W):
    """k_median_i16 (4 rows per lane, shared-rank selection) on arbitrary int16 x16 maps:
    every ragged size, full frame and 3 row bands, depth and scaled post, vs the oracle."""
    rng = np.random.default_rng(H * 7919 + W)
    D = 64
    d16 = (rng.integers(-1, D, (H, W)) * 16).astype(np.int16)
    # runs of equal values to exercise ties
    d16[:, ::3] = d16[:, :1]
    disp = O.disparity_f32(d16)
    e_depth, e_norm = O.depth_post(disp, 0.3, 2.0, 0)
    e_sn, e_su8, e_conf = O.scaled_post(disp, 0, D)
    n = H * W
    d_in = engine.dev_alloc(n * 2)
    bufs = [engine.dev_alloc(n * 4) for _ in range(3)] + [engine.dev_alloc(n)]
    try:
        engine.to_device(d_in, d16)
        for bands in (1, 3):
            for k in range(bands):
                r0, r1 = H * k // bands, H * (k + 1) // bands
                engine.median_post_dev(d_in, H, W, r0, r1, 1, bufs[0], bufs[1], bufs[3],
                                       min_depth=0.3, max_depth=2.0, min_disp_global=0,
                                       min_disp=0, num_disp=D)
            np.testing.assert_array_equal(engine.to_host(bufs[0], (H, W), np.float32), disp)
            np.testing.assert_array_equal(engine.to_host(bufs[1], (H, W), np.float32), e_depth)
            np.testing.assert_array_equal(engine.to_host(bufs[3], (H, W), np.uint8), e_norm)
        engine.median_post_dev(d_in, H, W, 0, H, 2, bufs[0], bufs[1], bufs[3], bufs[2],
                               min_disp=0, num_disp=D)
        np.testing.assert_array_equal(engine.to_host(bufs[1], (H, W), np.float32), e_sn)
        np.testing.assert_array_equal(engine.to_host(bufs[3], (H, W), np.uint8), e_su8)
        np.testing.assert_array_equal(engine.to_host(bufs[2], (H, W), np.float32), e_conf)
    finally:
        for p in [d_in] + bufs:
            engine.dev_free(p)


def test_profiling_counters(engine):
    L, R = _pair(40, 300, 64, seed=1)
    engine.profile(True)
    engine.profile_reset()
    for _ in range(3):
        engine.depth_map(L, R, 0, 64, 9, 0.3, 2.0)
    engine.profile(False)
    ms, n = engine.profile_read("match")
    assert n == 3 and ms > 0
    ms, n = engine.profile_read("median")
    assert n == 3 and ms > 0


def test_thread_pool_usage_like_reference(engine):
    """fused_depth_map.py:2591-2598 submits the stereo call to a ThreadPoolExecutor."""
    from concurrent.futures import ThreadPoolExecutor
    from stereovision_amd import fused_depth_map as FDM
    L, R = _pair(60, 300, 96, seed=8)
    bl, br = to_bgr(L), to_bgr(R)
    exp = O.create_depth_map_stereo_scaled(bl, br, 0, 96, 5)
    with ThreadPoolExecutor(max_workers=2) as ex:
        futs = [ex.submit(FDM.create_depth_map_stereo_scaled, bl.copy(), br.copy(), 0, 96, 5)
                for _ in range(6)]
        for f in futs:
            dn, disp, cmap, conf = f.result(timeout=30)
            np.testing.assert_array_equal(disp, exp[1])
            np.testing.assert_array_equal(conf, exp[3])


def test_dropin_create_depth_map_end_to_end(engine, monkeypatch):
    from stereovision_amd import depth_map as DM
    monkeypatch.setattr(DM, "NUM_DISP", 64)
    monkeypatch.setattr(DM, "WINDOW_SIZE", 9)
    L, R = _pair(50, 320, 64, seed=9)
    depth, disp, cmap = DM.create_depth_map(to_bgr(L), to_bgr(R), None, 0.2, 4.0)
    e = O.create_depth_map(to_bgr(L), to_bgr(R), 0, 64, 9, 0.2, 4.0)
    np.testing.assert_array_equal(depth, e[0])
    np.testing.assert_array_equal(disp, e[1])
    assert cmap.shape == (50, 320, 3)
    # reference default globals (NUM_DISP=320, WINDOW_SIZE=7) on a frame wide enough
    monkeypatch.setattr(DM, "NUM_DISP", 320)
    monkeypatch.setattr(DM, "WINDOW_SIZE", 7)
    L, R = _pair(30, 700, 320, seed=10)
    depth, disp, cmap = DM.create_depth_map(L, R)
    np.testing.assert_array_equal(disp, O.disparity_f32(C.disparity16(L, R, 0, 320, 7, 0)))


def test_row_tiled_module_and_single_hip_runtime(engine):
    """RowTiledDepthMap (torch-free, device pointers) bands == the full-frame oracle for 1, 2
    and 4 emulated ranks, and the process maps exactly one HIP runtime: ROCm's (nothing in
    the product path or the tests' GPU process loads torch's bundled copy)."""
    import sys
    from stereovision_amd.distributed import RowTiledDepthMap
    H, W, D, win = 97, 500, 64, 9
    L, R, _ = stereo_pair(H, W, D, seed=3)
    dL, dR = engine.dev_alloc(H * W), engine.dev_alloc(H * W)
    engine.to_device(dL, L)
    engine.to_device(dR, R)
    ref = O.disparity_f32(C.disparity16(L, R, 0, D, win, 0))
    ref_depth, _ = O.depth_post(ref, 0.3, 2.0)
    try:
        for world in (1, 2, 4):
            disp = np.zeros((H, W), np.float32)
            depth = np.zeros((H, W), np.float32)
            for k in range(world):
                rt = RowTiledDepthMap(H, W, D, win, rank=k, world=world, engine=engine)
                rt.compute(dL, dR)
                engine.synchronize()
                disp[rt.r0:rt.r1] = engine.to_host(rt.disp, (H, W), np.float32)[rt.r0:rt.r1]
                depth[rt.r0:rt.r1] = engine.to_host(rt.out_a, (H, W), np.float32)[rt.r0:rt.r1]
                rt.close()
            np.testing.assert_array_equal(disp, ref, err_msg=str(world))
            np.testing.assert_array_equal(depth, ref_depth, err_msg=str(world))
    finally:
        engine.dev_free(dL)
        engine.dev_free(dR)
    hip = {ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln}
    assert len(hip) == 1 and "/torch/" not in next(iter(hip)), hip
    assert "torch" not in sys.modules


@pytest.mark.parametrize("H,W,nf,pad", [(45, 150, 3, 3), (16, 64, 2, 3), (33, 301, 3, 3), (7, 70, 2, 3),
                                        (120, 640, 4, 3), (9, 8, 1, 3), (48, 640, 2, 0), (37, 1000, 2, 4),
                                        (20, 256, 3, 0), (24, 260, 2, 0), (9, 300, 2, 0), (8, 257, 1, 1)])
def test_depth_map_harris_batch_dev_fused(engine, H, W, nf, pad):
    """sv_depth_map_batch_dev with out.harris (C2: Harris blocks inside the median launch) == the C
    oracle frame by frame: the create_depth_map outputs bit-exact and the Harris response of
    each left frame within 1e-4 (north_star; observed exact), with row pitches wider than the
    frame (unaligned) and equal to it (the 248-column waves' dword loads, W >= 256); frames
    under 8 px take the separate Harris launch."""
    D, win, pitch = 32, 7, W + pad
    rng = np.random.default_rng(H * W + nf)
    L = np.zeros((nf, H, pitch), np.uint8)
    R = np.zeros((nf, H, pitch), np.uint8)
    for z in range(nf):
        a, b = _pair(H, W, D, seed=40 + z)
        L[z, :, :W], R[z, :, :W] = a, b
        L[z, :, W:] = rng.integers(0, 256, (H, pitch - W))   # never read as data
    n = H * W
    dL, dR = engine.dev_alloc(L.nbytes), engine.dev_alloc(R.nbytes)
    outs = [engine.dev_alloc(4 * n * nf), engine.dev_alloc(4 * n * nf), engine.dev_alloc(n * nf),
            engine.dev_alloc(4 * n * nf)]
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        engine.depth_map_batch_dev(dL, dR, nf, H, W, pitch, H * pitch, 0, D, win, 0.3, 2.0, outs[0],
                                   outs[1], outs[2], d_harris=outs[3])
        depth = engine.to_host(outs[0], (nf, H, W), np.float32)
        disp = engine.to_host(outs[1], (nf, H, W), np.float32)
        norm = engine.to_host(outs[2], (nf, H, W), np.uint8)
        har = engine.to_host(outs[3], (nf, H, W), np.float32)
        for z in range(nf):
            Lz, Rz = np.ascontiguousarray(L[z, :, :W]), np.ascontiguousarray(R[z, :, :W])
            e_depth, e_disp, e_norm = C.depth_map(Lz, Rz, 0, D, win)
            np.testing.assert_array_equal(disp[z], e_disp, err_msg=f"frame {z}")
            np.testing.assert_array_equal(depth[z], e_depth, err_msg=f"frame {z}")
            np.testing.assert_array_equal(norm[z], e_norm, err_msg=f"frame {z}")
            np.testing.assert_allclose(har[z], C.harris(Lz), rtol=0, atol=1e-4, err_msg=f"frame {z}")
    finally:
        for p_ in (dL, dR, *outs):
            engine.dev_free(p_)


@pytest.mark.parametrize("H,W", [(45, 150), (16, 64), (33, 130), (2, 70), (17, 3)])
def test_harris_batch_dev_per_frame(engine, H, W):
    """sv_harris_batch_dev (one launch over grid.z, LDS-staged tiles) == the oracle's Harris
    frame by frame, with a row pitch wider than the frame (tile edges, reflect-101 borders)."""
    nf, pitch = 3, W + 5
    rng = np.random.default_rng(H * W)
    frames = rng.integers(0, 256, (nf, H, pitch), dtype=np.uint8)
    n = nf * H * pitch
    dg, dout = engine.dev_alloc(n), engine.dev_alloc(nf * H * W * 4)
    try:
        engine.to_device(dg, frames)
        engine.harris_batch_dev(dg, nf, H, W, pitch, H * pitch, dout)
        got = engine.to_host(dout, (nf, H, W), np.float32)
        for z in range(nf):
            g = np.ascontiguousarray(frames[z, :, :W])
            assert np.abs(got[z] - O.harris(g)).max() <= HARRIS_TOL, f"frame {z}"
            np.testing.assert_array_equal(got[z], O.harris(g))     # observed bit-exact
    finally:
        engine.dev_free(dg)
        engine.dev_free(dout)


@pytest.mark.parametrize("H,W", [(60, 300), (37, 203), (1080, 1920)])
def test_colormap_fused_in_the_median_epilogue(engine, H, W):
    """sv_depth_map_color / sv_stereo_scaled_color: the numeric outputs equal the oracle's
    and the colormap equals the display table applied to the oracle's u8 image (vector and
    ragged-width store paths)."""
    from stereovision_amd import colormap
    L, R = _pair(H, W, 64, seed=H + W)
    bl, br = to_bgr(L), to_bgr(R)
    for name in ("turbo", "jet"):
        t = colormap.table(name)
        depth, disp, cmap, norm = engine.depth_map_color(bl, br, 0, 64, 9, 0.3, 2.0, t,
                                                         with_normalized=True)
        e_depth, e_disp, e_norm = O.create_depth_map(bl, br, 0, 64, 9, 0.3, 2.0)
        np.testing.assert_array_equal(depth, e_depth)
        np.testing.assert_array_equal(disp, e_disp)
        np.testing.assert_array_equal(norm, e_norm)
        np.testing.assert_array_equal(cmap, t[e_norm])
        dn, d2, cm2, cf, du = engine.stereo_scaled_color(bl, br, 0, 64, 5, t, with_normalized=True)
        e = O.create_depth_map_stereo_scaled(bl, br, 0, 64, 5)
        for got, exp in zip((dn, d2, du, cf), (e[0], e[1], e[2], e[3])):
            np.testing.assert_array_equal(got, exp)
        np.testing.assert_array_equal(cm2, t[e[2]])


@pytest.mark.parametrize("H,W", [(70, 400), (33, 130), (17, 63)])
def test_median_post_color_dev_epilogue(engine, H, W):
    """sv_median_rows_dev with out.bgr: the colormap written by the median kernel's epilogue equals
    the table applied to the oracle's u8 image, for both modes, full frame and row bands."""
    from stereovision_amd import colormap
    L, R = _pair(H, W, 64, seed=H * W)
    d16 = O.disparity16(L, R, 0, 64, 9)
    disp = O.disparity_f32(d16)
    _, e_norm = O.depth_post(disp, 0.3, 2.0, 0)
    _, e_su8, _ = O.scaled_post(disp, 0, 64)
    n = H * W
    d_in = engine.dev_alloc(2 * n)
    bufs = [engine.dev_alloc(4 * n), engine.dev_alloc(4 * n), engine.dev_alloc(n), engine.dev_alloc(4 * n),
            engine.dev_alloc(3 * n)]
    try:
        engine.to_device(d_in, d16)
        for mode, name, exp_u8 in ((1, "turbo", e_norm), (2, "jet", e_su8)):
            t = colormap.table(name)
            for bands in (1, 3):
                for k in range(bands):
                    r0, r1 = H * k // bands, H * (k + 1) // bands
                    engine.median_post_color_dev(d_in, H, W, r0, r1, mode, t, bufs[0], bufs[1], bufs[2],
                                                 bufs[4], d_out_b=bufs[3], min_depth=0.3, max_depth=2.0,
                                                 min_disp_global=0, min_disp=0, num_disp=64)
                engine.synchronize()
                np.testing.assert_array_equal(engine.to_host(bufs[2], (H, W), np.uint8), exp_u8)
                np.testing.assert_array_equal(engine.to_host(bufs[4], (H, W, 3), np.uint8), t[exp_u8])
    finally:
        for p in [d_in] + bufs:
            engine.dev_free(p)


@pytest.mark.parametrize("scaled", [False, True])
def test_registered_outputs_dma_path_matches_host_expansion(engine, scaled):
    """Host-buffer calls whose recycled outputs got page-locked (sv_host_register) take the
    device-epilogue + DMA path; the first call (fresh arrays) takes the int16 + host table
    expansion path.  Both must give the same bytes."""
    from stereovision_amd import colormap
    L, R, _ = stereo_pair(70, 333, 64, seed=21)
    Lb, Rb = to_bgr(L), to_bgr(R)
    t = colormap.table("turbo")
    call = (lambda: engine.stereo_scaled_color(Lb, Rb, 0, 64, 9, t)) if scaled else \
        (lambda: engine.depth_map_color(Lb, Rb, 0, 64, 9, 0.3, 2.0, t))
    noreg = engine._noreg
    engine._noreg = False                       # the DMA path is opt-in (SV_REGISTER_OUTPUTS=1)
    try:
        first = [a.copy() for a in call()]      # fresh set: host expansion
        for _ in range(3):                      # released -> reused -> registered -> DMA
            got = call()
            for g, e in zip(got, first):
                np.testing.assert_array_equal(g, e)
            del got
        assert engine.registered_outputs(), "no output set was registered"
    finally:
        engine._noreg = noreg


@pytest.mark.parametrize("win,D", [(9, 128), (15, 256)])
def test_ring_kind_huge_out_pitch_falls_back_exactly(engine, win, D):
    """the ring kernel's 32-bit buffer offsets cannot address an int16 map whose
    rows lie past 2^31 bytes; such maps take the size_t-addressed four-row kind, bit-exact."""
    H, W = 40, 400
    opitch = (1 << 26) + 64                       # 2 * 40 * 2^26 bytes = 5.4 GB of map span
    L, R, _ = stereo_pair(H, W, D, seed=31)
    exp = O.disparity16(L, R, 0, D, win)
    dL, dR = engine.dev_alloc(H * W), engine.dev_alloc(H * W)
    engine.to_device(dL, L)
    engine.to_device(dR, R)
    span = 2 * ((H - 1) * opitch + W)
    d16 = engine.dev_alloc(span)
    try:
        engine.disparity_dev(dL, dR, H, W, W, 0, D, win, "sad", 0, H, d16, opitch)
        engine.synchronize()
        for y in (0, 1, H // 2, H - 2, H - 1):
            row = engine.to_host(d16 + 2 * y * opitch, (W,), np.int16)
            np.testing.assert_array_equal(row, exp[y], err_msg=f"row {y}")
    finally:
        for p in (dL, dR, d16):
            engine.dev_free(p)


@pytest.mark.parametrize("H,W,D,win,cost", [(127, 200, 64, 9, "sad"), (256, 208, 64, 9, "sad"),
                                            (257, 240, 96, 15, "sad"), (301, 256, 64, 11, "ssd"),
                                            (301, 256, 64, 7, "ssd"), (260, 320, 64, 7, "hog"),
                                            (90, 700, 320, 7, "sad"), (1080, 1920, 128, 9, "sad")])
def test_host_path_matches_oracle(engine, H, W, D, win, cost):
    """The host-buffer frame path (stage + upload, gray, disparity, median, outputs back in 8
    pieces): every output, on both the fresh-array path (int16 medians + host expansion per
    piece) and the registered-output path (device epilogue + DMA), equals the C oracle."""
    L, R, _ = stereo_pair(H, W, D, seed=H + W + win)
    bl, br = to_bgr(L), to_bgr(R)
    g0, g1 = C.gray(bl), C.gray(br)
    e_depth, e_disp, e_norm = C.depth_map(g0, g1, 0, D, win, {"sad": 0, "ssd": 1, "hog": 2}[cost], 0.3, 2.0)
    for it in range(4):        # fresh set, then recycled sets (registered from their reuse)
        depth, disp, norm = engine.depth_map(bl, br, 0, D, win, 0.3, 2.0, cost=cost)
        np.testing.assert_array_equal(disp, e_disp, err_msg=f"call {it}")
        np.testing.assert_array_equal(depth, e_depth, err_msg=f"call {it}")
        np.testing.assert_array_equal(norm, e_norm, err_msg=f"call {it}")
        del depth, disp, norm


def test_depth_map_batch_int16_medians(engine):
    """sv_depth_map_batch_dev with out.med16: the int16 x16 median maps beside the f32 outputs (the
    multi-GPU bench gathers these): med16 / 16 == the f32 disparity, both == the oracle."""
    nf, H, W, D = 3, 70, 300, 64
    Ls, Rs = [], []
    for z in range(nf):
        L, R, _ = stereo_pair(H, W, D, seed=70 + z)
        Ls.append(L)
        Rs.append(R)
    L, R = np.stack(Ls), np.stack(Rs)
    n = H * W
    dL, dR = engine.dev_alloc(L.nbytes), engine.dev_alloc(R.nbytes)
    bufs = [engine.dev_alloc(4 * n * nf), engine.dev_alloc(4 * n * nf), engine.dev_alloc(n * nf),
            engine.dev_alloc(2 * n * nf)]
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        engine.depth_map_batch_dev(dL, dR, nf, H, W, W, n, 0, D, 9, 0.3, 2.0, bufs[0], bufs[1], bufs[2],
                                   d_med16=bufs[3])
        engine.synchronize()
        disp = engine.to_host(bufs[1], (nf, H, W), np.float32)
        med = engine.to_host(bufs[3], (nf, H, W), np.int16)
        np.testing.assert_array_equal(med.astype(np.float32) / np.float32(16.0), disp)
        for z in range(nf):
            _, e_disp, _ = C.depth_map(L[z], R[z], 0, D, 9)
            np.testing.assert_array_equal(disp[z], e_disp)
    finally:
        for p in [dL, dR] + bufs:
            engine.dev_free(p)


def test_harris_dpp_kernel_equals_lds_kernel():
    """k_harris_dpp4 (4 columns per lane, W >= 1024) and k_harris_dpp (1 column per lane;
    SV_HARRIS=dpp1) — waves walking row bands, DPP neighbours, reflect-101 of the product
    images through the cross product's sign — give the same bytes as the LDS-tile kernel
    (SV_HARRIS=lds), each in a child, at tile / band edges, unaligned widths and tiny sizes,
    and all are within the north_star tolerance of the oracle."""
    import os
    import subprocess
    import sys
    sizes = [(8, 8), (9, 61), (16, 60), (17, 120), (31, 121), (33, 179), (480, 640), (70, 333),
             (9, 256), (13, 258), (33, 500), (17, 1023), (20, 1024), (24, 1920), (11, 1030),
             (19, 1027)]
    code = ("import sys, numpy as np; sys.path.insert(0, %r)\n"
            "from stereovision_amd.engine import get_engine\n"
            "e = get_engine(0)\n"
            "for H, W in %r:\n"
            "    g = np.random.default_rng(H * 1000 + W).integers(0, 256, (H, W), dtype=np.uint8)\n"
            "    sys.stdout.buffer.write(e.harris(g).tobytes())\n") % (
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), sizes)
    outs = []
    for flag in ("dpp", "dpp1", "lds"):   # 4 columns per lane (W >= 1024), 1 per lane, LDS tiles
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120,
                           env=dict(os.environ, SV_HARRIS=flag, SV_WARMUP_AT_IMPORT="0"))
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        outs.append(r.stdout)
    assert outs[0] == outs[2] and outs[1] == outs[2]
    off = 0
    for H, W in sizes:
        g = np.random.default_rng(H * 1000 + W).integers(0, 256, (H, W), dtype=np.uint8)
        got = np.frombuffer(outs[0][off:off + 4 * H * W], np.float32).reshape(H, W)
        off += 4 * H * W
        assert np.abs(got - O.harris(g)).max() <= HARRIS_TOL, (H, W)


class _LocalGather:
    """A process group standing in for `world` ranks of one process: gatherv at the root copies
    every other rank's block (from that rank's RowTiledDepthMap buffer) into the root's."""

    def __init__(self, engine, tiles, rank):
        self.engine, self.tiles, self.rank, self.world = engine, tiles, rank, len(tiles)

    def allreduce_max(self, value):   # one process: the ranks' checks agree by construction
        return float(value)

    def gatherv(self, d_send, send_bytes, d_recv, offsets, sizes, root=0, stream=0):
        if self.rank != root:
            return
        self.engine.synchronize()
        for k, t in enumerate(self.tiles):
            if k != root and sizes[k]:
                blk = self.engine.to_host(t.m16 + offsets[k], (sizes[k],), np.uint8)
                self.engine.to_device(d_recv + offsets[k], blk)


@pytest.mark.parametrize("mode", ["depth", "scaled"])
def test_row_tiled_int16_gather_and_root_expansion(engine, mode):
    """RowTiledDepthMap since round 4: ranks other than the root compute only their bands'
    int16 x16 medians (band_outputs="m16"), gather() moves those rows into the root's m16
    buffer and the root expands them (sv_post_m16_dev) into its full-frame outputs — equal to
    the whole-frame oracle for create_depth_map's post (DEPTH) and the scaled app's (SCALED),
    with the root in the middle of the tiling."""
    from stereovision_amd.distributed import RowTiledDepthMap
    from stereovision_amd.engine import POST_DEPTH, POST_SCALED
    H, W, D, win, md, world, root = 71, 260, 48, 7, -2, 3, 1
    L, R = _pair(H, W, D, seed=61, min_disp=md)
    dL, dR = engine.dev_alloc(H * W), engine.dev_alloc(H * W)
    engine.to_device(dL, L)
    engine.to_device(dR, R)
    pm = POST_DEPTH if mode == "depth" else POST_SCALED
    tiles = [RowTiledDepthMap(H, W, D, win, min_disp=md, rank=k, world=world, engine=engine)
             for k in range(world)]
    try:
        for k, t in enumerate(tiles):
            t.compute(dL, dR, mode=pm, min_disp_global=md, band_outputs="full" if k == root else "m16")
        engine.synchronize()
        tiles[root].gather(_LocalGather(engine, tiles, root), root=root)
        engine.synchronize()
        rt = tiles[root]
        disp = engine.to_host(rt.disp, (H, W), np.float32)
        e_disp = C.median5_f32(C.disparity16(L, R, md, D, win, 0))
        np.testing.assert_array_equal(disp, e_disp)
        a = engine.to_host(rt.out_a, (H, W), np.float32)
        u = engine.to_host(rt.out_u8, (H, W), np.uint8)
        if pm == POST_DEPTH:
            e_a, e_u = C.depth_post(e_disp, 0.3, 2.0, md)
            np.testing.assert_array_equal(a, e_a)
            np.testing.assert_array_equal(u, e_u)
        else:
            e_a, e_u, e_b = C.scaled_post(e_disp, md, D)
            np.testing.assert_array_equal(a, e_a)
            np.testing.assert_array_equal(u, e_u)
            np.testing.assert_array_equal(engine.to_host(rt.out_b, (H, W), np.float32), e_b)
    finally:
        for t in tiles:
            t.close()
        engine.dev_free(dL)
        engine.dev_free(dR)
