"""GPU parity at the BASELINE.json workloads themselves (configs C4 and C5), bit-exact against
the C oracle, plus worst-case-contrast checks of the argmin key of every SAD kernel kind.

* C5 — 3840x2160, D=256, 15x15 window (+ HOG descriptor match), row-tiled across 8 GPUs:
  the whole frame in one call, and the 8 row bands of the row-tiled mode computed through
  the device API (sv_disparity_dev over the band + median halo, sv_median_rows_dev over the
  band) and reassembled.  Reference arithmetic replaced: depth_map.py:894-912.
* C4 — 8 x 1920x1080, D=128, 11x11 window, one frame per GPU: one 8-frame batch
  (sv_depth_map_batch_dev) and sv_multi_gpu_batch over 8 contexts, checked frame by frame.
* hi-key SAD kind (4 output rows per wave, win <= 11: keys (cost << 16) | idx updated with
  v_sad_hi_u8) at maximal contrast: alternating 0/255 columns and checkerboards make every
  tap 255, i.e. the largest key the kind can form.
"""
import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd.distributed import band_rows, median_halo
from stereovision_amd.engine import POST_DEPTH, Engine, device_count, multi_gpu_batch
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu

COSTS = {"sad": 0, "ssd": 1, "hog": 2}


def _oracle_depth_map(L, R, D, win, cost, min_depth=0.3, max_depth=2.0):
    """create_depth_map's numeric body (depth_map.py:909-936) through the C oracle."""
    d16 = C.disparity16(L, R, 0, D, win, COSTS[cost])
    disp = C.median5_f32(d16)
    depth, norm = C.depth_post(disp, min_depth, max_depth)
    return d16, disp, depth, norm


def _bands_on_device(engine, L, R, D, win, cost, world):
    """The row-tiled mode of C5 on one device: band k = rows band_rows(H, k, world), its
    disparity computed over the band plus the 2-row median halo, then median + depth post of
    the band alone.  Returns the reassembled (d16 of the band rows, disparity, depth, norm)."""
    H, W = L.shape
    n = H * W
    dL, dR = engine.dev_alloc(n), engine.dev_alloc(n)
    d16 = engine.dev_alloc(2 * n)
    ddisp, ddepth, dnorm = engine.dev_alloc(4 * n), engine.dev_alloc(4 * n), engine.dev_alloc(n)
    out16 = np.zeros((H, W), np.int16)
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        for k in range(world):
            r0, r1 = band_rows(H, k, world)
            h0, h1 = median_halo(r0, r1, H)
            engine.disparity_dev(dL, dR, H, W, W, 0, D, win, cost, h0, h1, d16, W)
            band = engine.to_host(d16 + 2 * r0 * W, (r1 - r0, W), np.int16)
            out16[r0:r1] = band
            engine.median_post_dev(d16, H, W, r0, r1, POST_DEPTH, ddisp, ddepth, dnorm,
                                   min_depth=0.3, max_depth=2.0, min_disp_global=0,
                                   min_disp=0, num_disp=D)
        disp = engine.to_host(ddisp, (H, W), np.float32)
        depth = engine.to_host(ddepth, (H, W), np.float32)
        norm = engine.to_host(dnorm, (H, W), np.uint8)
    finally:
        for p in (dL, dR, d16, ddisp, ddepth, dnorm):
            engine.dev_free(p)
    return out16, disp, depth, norm


@pytest.fixture(scope="module")
def c5_pair():
    L, R, gt = stereo_pair(2160, 3840, 256, seed=55)
    return L, R, gt


@pytest.mark.parametrize("cost", ["sad", "hog"])
def test_c5_4k_d256_w15_full_frame_and_8_row_bands(engine, c5_pair, cost):
    L, R, gt = c5_pair
    D, win = 256, 15
    e16, e_disp, e_depth, e_norm = _oracle_depth_map(L, R, D, win, cost)
    got = engine.disparity(L, R, 0, D, win, cost)
    np.testing.assert_array_equal(got, e16)
    b16, disp, depth, norm = _bands_on_device(engine, L, R, D, win, cost, world=8)
    np.testing.assert_array_equal(b16, e16)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)
    if cost == "sad":   # property: the background plane (d = D/4) is recovered away from edges
        assert (got[40:500, 600:1200] == 64 * 16).mean() > 0.99


def test_c5_depth_map_entry_point(engine, c5_pair):
    """The full app-1 host entry point (sv_depth_map) at the C5 size."""
    L, R, _ = c5_pair
    _, e_disp, e_depth, e_norm = _oracle_depth_map(L, R, 256, 15, "sad")
    depth, disp, norm = engine.depth_map(L, R, 0, 256, 15, 0.3, 2.0)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


@pytest.fixture(scope="module")
def c4_frames():
    F, H, W, D = 8, 1080, 1920, 128
    pairs = [stereo_pair(H, W, D, seed=400 + f)[:2] for f in range(F)]
    L = np.stack([p[0] for p in pairs])
    R = np.stack([p[1] for p in pairs])
    ref = [_oracle_depth_map(L[f], R[f], D, 11, "sad") for f in range(F)]
    return L, R, ref


def test_c4_eight_frame_batch_1080p_d128_w11(engine, c4_frames):
    L, R, ref = c4_frames
    F, H, W = L.shape
    n = F * H * W
    dL, dR = engine.dev_alloc(n), engine.dev_alloc(n)
    ddepth, ddisp, dnorm = engine.dev_alloc(4 * n), engine.dev_alloc(4 * n), engine.dev_alloc(n)
    d16 = engine.dev_alloc(2 * n)
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        engine.disparity_batch_dev(dL, dR, F, H, W, W, H * W, 0, 128, 11, "sad", d16, W, H * W)
        got16 = engine.to_host(d16, (F, H, W), np.int16)
        engine.depth_map_batch_dev(dL, dR, F, H, W, W, H * W, 0, 128, 11, 0.3, 2.0, ddepth, ddisp,
                                   dnorm)
        depth = engine.to_host(ddepth, (F, H, W), np.float32)
        disp = engine.to_host(ddisp, (F, H, W), np.float32)
        norm = engine.to_host(dnorm, (F, H, W), np.uint8)
    finally:
        for p in (dL, dR, ddepth, ddisp, dnorm, d16):
            engine.dev_free(p)
    for f in range(F):
        e16, e_disp, e_depth, e_norm = ref[f]
        np.testing.assert_array_equal(got16[f], e16, err_msg=f"frame {f}")
        np.testing.assert_array_equal(disp[f], e_disp, err_msg=f"frame {f}")
        np.testing.assert_array_equal(depth[f], e_depth, err_msg=f"frame {f}")
        np.testing.assert_array_equal(norm[f], e_norm, err_msg=f"frame {f}")


def test_c4_multi_gpu_batch_eight_contexts(engine, c4_frames):
    """sv_multi_gpu_batch over 8 contexts: distinct devices where the box has them, extra
    contexts on device 0 otherwise (each context: own stream, buffers and host thread)."""
    L, R, ref = c4_frames
    nd = max(1, device_count())
    extra = [Engine(k % nd) for k in range(1, 8)]
    try:
        depth, disp, norm = multi_gpu_batch([engine] + extra, L, R, 0, 128, 11, 0.3, 2.0)
    finally:
        for e in extra:
            e.close()
    for f in range(L.shape[0]):
        _, e_disp, e_depth, e_norm = ref[f]
        np.testing.assert_array_equal(disp[f], e_disp, err_msg=f"frame {f}")
        np.testing.assert_array_equal(depth[f], e_depth, err_msg=f"frame {f}")
        np.testing.assert_array_equal(norm[f], e_norm, err_msg=f"frame {f}")


# ---- maximal-contrast inputs for the argmin keys -------------------------------------------
def _contrast_patterns(H, W):
    cols = np.tile(np.array([0, 255], np.uint8), (H, W // 2))
    yy, xx = np.mgrid[0:H, 0:W]
    checker = (((yy + xx) & 1) * 255).astype(np.uint8)
    return {"columns": (cols, np.roll(cols, 1, axis=1)),
            "checker": (checker, 255 - checker),
            "columns_vs_flat": (cols, np.full((H, W), 255 - cols[0, 0], np.uint8)),
            "black_white": (np.zeros((H, W), np.uint8), np.full((H, W), 255, np.uint8))}


@pytest.mark.parametrize("win", [5, 7, 9, 11])
@pytest.mark.parametrize("D,min_disp", [(64, 0), (128, 0), (64, -5), (128, -5)])
def test_hi_key_sad_kind_at_maximal_contrast(engine, win, D, min_disp):
    """Every tap |0 - 255|: window costs reach 255 * win^2 (30,855 at win 11), the largest
    `cost << 16` key of the v_sad_hi_u8 kind; ties resolve to the smallest disparity."""
    H, W = 29, 448
    for name, (L, R) in _contrast_patterns(H, W).items():
        got = engine.disparity(L, R, min_disp, D, win, "sad")
        exp = C.disparity16(L, R, min_disp, D, win, 0)
        np.testing.assert_array_equal(got, exp, err_msg=name)


@pytest.mark.parametrize("win", [5, 9, 11])
def test_hi_key_sad_kind_max_contrast_batch_and_full_hd(engine, win):
    """The same worst case at the metric geometry, through the batched launch (grid.z)."""
    H, W, D = 1080, 1920, 128
    pats = _contrast_patterns(H, W)
    L = np.stack([pats["columns"][0], pats["checker"][0]])
    R = np.stack([pats["columns"][1], pats["checker"][1]])
    n = L.size
    dL, dR, d16 = engine.dev_alloc(n), engine.dev_alloc(n), engine.dev_alloc(2 * n)
    try:
        engine.to_device(dL, L)
        engine.to_device(dR, R)
        engine.disparity_batch_dev(dL, dR, 2, H, W, W, H * W, 0, D, win, "sad", d16, W, H * W)
        got = engine.to_host(d16, (2, H, W), np.int16)
    finally:
        for p in (dL, dR, d16):
            engine.dev_free(p)
    for f in range(2):
        np.testing.assert_array_equal(got[f], C.disparity16(L[f], R[f], 0, D, win, 0))


def test_one_row_and_two_row_sad_kinds_at_maximal_contrast(engine):
    """win <= 3 runs the one-row kind; win 13/15 the 4-row kind with 32-bit keys."""
    H, W = 21, 400
    for win in (1, 3, 13, 15):
        for name, (L, R) in _contrast_patterns(H, W).items():
            for D in (64, 256):
                np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win),
                                              C.disparity16(L, R, 0, D, win, 0),
                                              err_msg=f"{name} win={win} D={D}")
    # the oracle itself: a flat black/white pair ties every disparity -> min_disp
    L, R = _contrast_patterns(H, W)["black_white"]
    assert (O.disparity16(L, R, 0, 64, 9)[:, 64:] == 0).all()
