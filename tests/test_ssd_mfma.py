"""GPU parity of the SSD matrix-core kind (sv_ssd_mfma.hip: v_mfma_i32_32x32x32_i8 on offset
images, the window's vertical sum carried in persistent accumulators) against the C oracle's
SSD winner-take-all (first minimum): every odd window 1..15 and D = 32..256 in steps of 32
(VERDICT r05 #2), row bands, frame batches, several row bands per block column, negative and
positive min_disp, saturated contrast and all-tie frames.  Bit-exact.  An image whose base is
not 4-byte aligned takes the ring / one-row kinds (the LDS-DMA staging loads aligned dwords);
where only this kind's centred keys fit 32 bits (D = 160 w13, say) such a call fails loudly
instead.  (D > 128 with win 15 fits no kind's keys: the planner refuses it.)"""
import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu


def _ref(L, R, md, D, win, rows=None):
    return C.disparity16(L, R, md, D, win, 1, rows=rows) if rows else C.disparity16(L, R, md, D, win, 1)


@pytest.mark.parametrize("win", [1, 3, 5, 7, 9, 11, 13, 15])
@pytest.mark.parametrize("D", [32, 64, 128])
def test_ssd_mfma_windows(engine, D, win):
    H, W = 37, D + 300
    L, R, _ = stereo_pair(H, W, D, seed=D * 3 + win)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win, "ssd"), _ref(L, R, 0, D, win))


@pytest.mark.parametrize("D,win", [(96, 9), (160, 7), (160, 13), (192, 11), (224, 5), (256, 9), (256, 13)])
def test_ssd_mfma_wide_disparity_ranges(engine, D, win):
    H, W = 29, D + 420
    L, R, _ = stereo_pair(H, W, D, seed=D + win)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win, "ssd"), _ref(L, R, 0, D, win))


@pytest.mark.parametrize("D,win,md", [(128, 9, -7), (64, 15, 5), (128, 11, -130), (32, 3, 40)])
def test_ssd_mfma_min_disparity(engine, D, win, md):
    H, W = 33, 700
    L, R, _ = stereo_pair(H, W, D, seed=abs(md) + win)
    np.testing.assert_array_equal(engine.disparity(L, R, md, D, win, "ssd"), _ref(L, R, md, D, win))


def test_ssd_mfma_tall_frames_band_seams(engine):
    """Frames taller than one block band (64 / 96 rows): the accumulators restart at every band
    start with a warm-up over the window rows — seams must not show."""
    for H, win in ((301, 9), (200, 15), (130, 1)):
        L, R, _ = stereo_pair(H, 520, 128, seed=H)
        np.testing.assert_array_equal(engine.disparity(L, R, 0, 128, win, "ssd"), _ref(L, R, 0, 128, win))


def test_ssd_mfma_row_bands_and_batches(engine):
    """sv_disparity_dev over row bands (the row tiling's unit) and sv_disparity_batch_dev over a
    batch of frames (grid.z), both against the oracle."""
    H, W, D, win = 90, 610, 128, 11
    frames = [stereo_pair(H, W, D, seed=70 + s)[:2] for s in range(3)]
    n = H * W
    e = engine
    dL, dR, d16 = e.dev_alloc(3 * n), e.dev_alloc(3 * n), e.dev_alloc(2 * 3 * n)
    try:
        e.to_device(dL, np.stack([f[0] for f in frames]))
        e.to_device(dR, np.stack([f[1] for f in frames]))
        e.to_device(d16, np.full(3 * n, 0x5555, np.int16))
        e.disparity_batch_dev(dL, dR, 3, H, W, W, n, 0, D, win, "ssd", d16, W, n)
        e.synchronize()
        got = e.to_host(d16, (3, H, W), np.int16)
        for z, (L, R) in enumerate(frames):
            np.testing.assert_array_equal(got[z], _ref(L, R, 0, D, win))
        e.to_device(d16, np.full(3 * n, 0x5555, np.int16))
        L, R = frames[1]
        for r0, r1 in ((0, 17), (17, 60), (60, 90)):
            e.disparity_dev(dL + n, dR + n, H, W, W, 0, D, win, "ssd", r0, r1, d16, W)
        e.synchronize()
        np.testing.assert_array_equal(e.to_host(d16, (H, W), np.int16), _ref(L, R, 0, D, win))
    finally:
        for p in (dL, dR, d16):
            e.dev_free(p)


def test_ssd_mfma_extremes_and_ties(engine):
    """Saturated contrast (255 / 0 stripes: the largest squared differences, the key range's
    edge at win 15), flat frames (every disparity ties: the smallest wins) and a ramp."""
    H, W, D = 23, 460, 128
    x = np.arange(W)
    stripes = np.tile(np.where((x // 3) % 2 == 0, 255, 0).astype(np.uint8), (H, 1))
    flipped = stripes[:, ::-1].copy()
    for win in (9, 15):
        np.testing.assert_array_equal(engine.disparity(stripes, flipped, 0, D, win, "ssd"),
                                      _ref(stripes, flipped, 0, D, win))
    flat = np.full((H, W), 200, np.uint8)
    np.testing.assert_array_equal(engine.disparity(flat, flat, 0, D, 13, "ssd"), _ref(flat, flat, 0, D, 13))
    zero, full = np.zeros((H, W), np.uint8), np.full((H, W), 255, np.uint8)
    np.testing.assert_array_equal(engine.disparity(zero, full, 0, D, 15, "ssd"), _ref(zero, full, 0, D, 15))
    ramp = np.tile((x % 256).astype(np.uint8), (H, 1))
    np.testing.assert_array_equal(engine.disparity(ramp, ramp, 0, 64, 7, "ssd"), _ref(ramp, ramp, 0, 64, 7))


def test_ssd_mfma_unaligned_images_fall_back(engine):
    """Images at an odd device address (sv_disparity_dev on a view one byte in) take another
    kind; the result is the same."""
    H, W, D, win = 41, 520, 128, 9
    L, R, _ = stereo_pair(H, W, D, seed=9)
    n = H * W
    e = engine
    dL, dR, d16 = e.dev_alloc(n + 4), e.dev_alloc(n + 4), e.dev_alloc(2 * n)
    try:
        e.to_device(dL + 1, L)
        e.to_device(dR + 1, R)
        e.disparity_dev(dL + 1, dR + 1, H, W, W, 0, D, win, "ssd", 0, H, d16, W)
        e.synchronize()
        np.testing.assert_array_equal(e.to_host(d16, (H, W), np.int16), _ref(L, R, 0, D, win))
    finally:
        for p in (dL, dR, d16):
            e.dev_free(p)


def test_ssd_mfma_only_keys_refuse_unaligned_images(engine):
    """D=160 w13: the other kinds' (cost << dbits | idx) keys overflow, so the planner admits the
    call for the matrix-core kind only; an unaligned view cannot take it and must error."""
    from stereovision_amd.engine import SVError
    H, W, D, win = 21, 500, 160, 13
    L, R, _ = stereo_pair(H, W, D, seed=13)
    n = H * W
    e = engine
    dL, dR, d16 = e.dev_alloc(n + 4), e.dev_alloc(n + 4), e.dev_alloc(2 * n)
    try:
        e.to_device(dL + 1, L)
        e.to_device(dR + 1, R)
        with pytest.raises(SVError):
            e.disparity_dev(dL + 1, dR + 1, H, W, W, 0, D, win, "ssd", 0, H, d16, W)
            e.synchronize()
    finally:
        for p in (dL, dR, d16):
            e.dev_free(p)


def test_ssd_mfma_narrow_frames(engine):
    """Frames narrower than one block's 256 output columns, and a frame whose matched band
    [X0, X1) is a few columns wide."""
    for W in (200, 140, 133):
        L, R, _ = stereo_pair(19, W, 128, seed=W)
        np.testing.assert_array_equal(engine.disparity(L, R, 0, 128, 9, "ssd"), _ref(L, R, 0, 128, 9))
