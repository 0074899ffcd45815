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


def test_extreme_contrast_no_overflow(engine):
    # alternating 0/255 columns make every SAD/SSD tap maximal
    L = np.tile(np.array([0, 255], np.uint8), (24, 160))
    R = np.roll(L, 1, axis=1)
    for cost, D, win in [("sad", 128, 15), ("ssd", 256, 15), ("ssd", 64, 15)]:
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
