"""Independent third-party check of the oracle's border and stencil conventions (VERDICT r04
"What's weak" #1): the engine and both oracles (NumPy, C) share one author, so a misreading
of an OpenCV convention would appear in all three.  scipy.ndimage (not written here) restates
the same stencils with its own border modes:

* cv2.medianBlur(ksize=5)  replicate border        -> median_filter(size=5, mode='nearest')
* cv2.Sobel(ksize=3)       BORDER_REFLECT_101       -> correlate1d, mode='mirror'
                                                      (scipy's 'mirror' is d c b | a b c d)
* cv2.cornerHarris(3, 3, 0.04)   Sobel on REFLECT_101 pixels, products, unnormalised 3x3
                                 box filter with REFLECT_101 on the PRODUCT images
* the SAD / SSD window cost      replicate-clamped images, (2r+1)^2 box  -> correlate over
                                 |L - R(x - d)| with mode='nearest' (interior columns, where
                                 the column clamp of L and R coincide)
* the HOG window histograms      replicate-clamped box sums              -> mode='nearest'

Parity with OpenCV itself stays unpinned (no cv2 in this image); these tests pin the
conventions DESIGN.md §2 states against an implementation of another author.
Reference call sites: depth_map.py:909-912 (StereoSGBM.compute, medianBlur), north_star's
Harris (cornerHarris) and HOG descriptors.
"""
import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

ndi = pytest.importorskip("scipy.ndimage")


def _images(seed, H=37, W=53):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (H, W), dtype=np.uint8)


@pytest.mark.parametrize("shape", [(37, 53), (5, 7), (1, 9), (6, 1), (2, 2)])
def test_median5_is_scipy_median_filter_nearest(shape):
    rng = np.random.default_rng(sum(shape))
    a = rng.integers(-32, 2000, shape).astype(np.int16)
    np.testing.assert_array_equal(O.median5(a), ndi.median_filter(a, size=5, mode="nearest"))
    # the int16 x16 form the engine filters (median(i16)/16 == median(i16/16))
    d16 = (rng.integers(0, 64, shape) * 16).astype(np.int16)
    np.testing.assert_array_equal(O.disparity_f32(d16),
                                  ndi.median_filter(d16.astype(np.float32) / np.float32(16), size=5,
                                                    mode="nearest"))


@pytest.mark.parametrize("seed,shape", [(0, (37, 53)), (1, (3, 4)), (2, (2, 9)), (3, (16, 2))])
def test_sobel_is_scipy_sobel_mirror(seed, shape):
    g = _images(seed, *shape)
    gx, gy = O.sobel(g)
    gi = g.astype(np.int32)
    np.testing.assert_array_equal(gx, ndi.sobel(gi, axis=1, mode="mirror"))
    np.testing.assert_array_equal(gy, ndi.sobel(gi, axis=0, mode="mirror"))
    # the C oracle's Sobel is used through HOG codes and Harris; the NumPy one is the reference


def _harris_scipy(g):
    """cornerHarris(blockSize=3, ksize=3, k=0.04) in float64, OpenCV's order of operations:
    Sobel scaled by 1/(4*3*255) (REFLECT_101), products, unnormalised 3x3 box sums of the
    product images (REFLECT_101), R = det - k * trace^2."""
    gi = g.astype(np.float64)
    s = 1.0 / (4.0 * 3.0 * 255.0)
    dx = ndi.sobel(gi, axis=1, mode="mirror") * s
    dy = ndi.sobel(gi, axis=0, mode="mirror") * s
    box = np.ones((3, 3))
    a = ndi.correlate(dx * dx, box, mode="mirror")
    b = ndi.correlate(dx * dy, box, mode="mirror")
    c = ndi.correlate(dy * dy, box, mode="mirror")
    return (a * c - b * b) - 0.04 * (a + c) ** 2


@pytest.mark.parametrize("seed,shape", [(0, (37, 53)), (4, (8, 8)), (5, (3, 70)), (6, (64, 3))])
def test_harris_matches_scipy_structure_tensor(seed, shape):
    g = _images(seed, *shape)
    exp = _harris_scipy(g)
    got = O.harris(g).astype(np.float64)
    # f32 rounding of the oracle against float64: far below north_star's 1e-4 tolerance, far
    # above what a border or sign convention error would leave
    np.testing.assert_allclose(got, exp, rtol=2e-5, atol=1e-8)
    np.testing.assert_array_equal(C.harris(g), O.harris(g))


def test_harris_reflects_products_not_just_pixels():
    """cornerHarris reflects the product images: at a border the cross term keeps the sign of
    the inner neighbour's gx*gy.  A diagonal ramp has gx*gy > 0 everywhere inside; reflecting
    pixels instead would flip gx (or gy) outside and change the border responses."""
    y, x = np.mgrid[0:12, 0:12]
    g = ((x * 7 + y * 13) % 256).astype(np.uint8)
    np.testing.assert_allclose(O.harris(g).astype(np.float64), _harris_scipy(g), rtol=2e-5, atol=1e-8)


def _wta_scipy(L, R, min_disp, num_disp, win, ssd=False):
    """First-argmin disparity from box-filtered |L - R(x-d)| (or squares), scipy correlate with
    the replicate ('nearest') border; valid where the window's columns stay inside the image."""
    H, W = L.shape
    r = win // 2
    box = np.ones((win, win), np.int64)
    xs = np.arange(W)
    Li = L.astype(np.int64)
    best_c = np.full((H, W), np.iinfo(np.int64).max)
    best_d = np.zeros((H, W), np.int64)
    for d in range(min_disp, min_disp + num_disp):
        diff = Li - R[:, np.clip(xs - d, 0, W - 1)].astype(np.int64)
        cost = ndi.correlate(diff * diff if ssd else np.abs(diff), box, mode="nearest")
        m = cost < best_c
        best_c[m] = cost[m]
        best_d[m] = d
    return best_d * 16


@pytest.mark.parametrize("cost,win,min_disp,num_disp", [("sad", 9, 0, 32), ("sad", 5, -4, 20),
                                                         ("ssd", 7, 0, 24), ("sad", 15, 3, 16),
                                                         ("ssd", 3, -2, 9)])
def test_disparity_wta_matches_scipy_box_costs(cost, win, min_disp, num_disp):
    H, W = 29, 96
    L, R, _ = stereo_pair(H, W, num_disp + max(0, min_disp), seed=win * 10 + num_disp)
    got = O.disparity16(L, R, min_disp, num_disp, win, O.COST_SSD if cost == "ssd" else O.COST_SAD)
    exp = _wta_scipy(L, R, min_disp, num_disp, win, ssd=cost == "ssd")
    r = win // 2
    x0, x1 = O.valid_columns(W, min_disp, num_disp)
    lo, hi = max(x0, r), min(x1, W - r)   # columns whose window needs no column clamp of L
    assert hi - lo > 20
    np.testing.assert_array_equal(got[:, lo:hi], exp[:, lo:hi])
    # and the band outside [X0, X1) is SGBM's invalid value (minD - 1) * 16
    assert (got[:, :x0] == (min_disp - 1) * 16).all() and (got[:, x1:] == (min_disp - 1) * 16).all()
    np.testing.assert_array_equal(C.disparity16(L, R, min_disp, num_disp, win,
                                                1 if cost == "ssd" else 0), got)


@pytest.mark.parametrize("win", [3, 7, 15])
def test_hog_window_histograms_are_scipy_box_sums(win):
    g = _images(win, 33, 47)
    b, mag = O.hog_pixel(g)
    got = O.hog_hist(g, win).astype(np.int64)
    box = np.ones((win, win), np.int64)
    for k in range(O.HOG_BINS):
        exp = ndi.correlate(np.where(b == k, mag, 0).astype(np.int64), box, mode="nearest")
        np.testing.assert_array_equal(got[k], exp, err_msg=f"bin {k}")
    # magnitudes from scipy's Sobel: (|gx| + |gy|) >> 3
    gi = g.astype(np.int32)
    exp_mag = (np.abs(ndi.sobel(gi, axis=1, mode="mirror")) + np.abs(ndi.sobel(gi, axis=0, mode="mirror"))) >> 3
    np.testing.assert_array_equal(mag, exp_mag)
