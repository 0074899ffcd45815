"""Seeded random sweep of the HIP path against the C / NumPy oracles (GPU).

Every kernel kind the planner can pick is reached by drawing the configuration at random:
cost (SAD / SSD / HOG), window 1..15, num_disp 1..256, min_disp -24..24, image sizes from a
single pixel to a few hundred columns, textures from flat to maximal contrast.  Each case is
bit-exact against the C oracle (disparity) and, for a third of the cases, the whole app-1 /
app-2 numeric path (median + post) against the NumPy oracle.  The seeds are fixed, so a
failure names a reproducible case.
"""
import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C

pytestmark = pytest.mark.gpu

COSTS = {"sad": 0, "ssd": 1, "hog": 2}


def _texture(rng, H, W, kind):
    if kind == 0:                                   # random bytes
        return rng.integers(0, 256, (H, W), dtype=np.uint8)
    if kind == 1:                                   # flat with a few steps
        img = np.full((H, W), rng.integers(0, 256), np.uint8)
        for _ in range(3):
            x = rng.integers(0, W)
            img[:, x:] = rng.integers(0, 256)
        return img
    if kind == 2:                                   # maximal contrast columns / checkerboard
        yy, xx = np.mgrid[0:H, 0:W]
        return np.where(((xx + (yy if rng.integers(0, 2) else 0)) & 1) == 0, 0, 255).astype(np.uint8)
    base = rng.integers(0, 256, (H, W + 64), dtype=np.uint8)   # smooth-ish shifted scene
    k = np.ones(5) / 5
    base = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, base.astype(np.float64))
    return np.clip(base[:, :W], 0, 255).astype(np.uint8)


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    cost = ["sad", "sad", "sad", "ssd", "hog"][rng.integers(0, 5)]
    win = int(rng.choice([1, 3, 5, 7, 9, 11, 13, 15]))
    D = int(rng.choice([1, 3, 4, 8, 16, 31, 48, 64, 96, 100, 128, 160, 200, 256]))
    if cost == "ssd" and D > 128 and win >= 13:
        D = 128
    min_disp = int(rng.integers(-24, 25))
    H = int(rng.choice([1, 2, 5, 17, 40, 63]))
    W = int(rng.choice([1, 7, 64, 129, 300, 411]))
    kind = int(rng.integers(0, 4))
    L = _texture(rng, H, W, kind)
    shift = int(rng.integers(0, max(1, min(D, W))))
    R = np.roll(L, -shift, axis=1) ^ rng.integers(0, 4, (H, W), dtype=np.uint8)
    return cost, win, D, min_disp, L, R


@pytest.mark.parametrize("seed", range(160))
def test_random_disparity_matches_c_oracle(engine, seed):
    cost, win, D, min_disp, L, R = _case(seed)
    got = engine.disparity(L, R, min_disp, D, win, cost)
    exp = C.disparity16(L, R, min_disp, D, win, COSTS[cost])
    np.testing.assert_array_equal(got, exp, err_msg=f"seed {seed}: {cost} win {win} D {D} minD {min_disp} {L.shape}")


@pytest.mark.parametrize("seed", range(0, 160, 3))
def test_random_depth_paths_match_numpy_oracle(engine, seed):
    cost, win, D, min_disp, L, R = _case(seed)
    if cost == "ssd":
        cost = "sad"
    d16 = C.disparity16(L, R, min_disp, D, win, COSTS[cost])
    disparity = O.disparity_f32(d16)
    depth, disp, norm = engine.depth_map(L, R, min_disp, D, win, 0.3, 2.0, cost=cost)
    e_depth, e_norm = O.depth_post(disparity, 0.3, 2.0, min_disp)
    np.testing.assert_array_equal(disp, disparity, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(depth, e_depth, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(norm, e_norm, err_msg=f"seed {seed}")


@pytest.mark.parametrize("seed", range(1, 160, 4))
def test_random_row_bands_reassemble(engine, seed):
    """Random row bands (the row-tiled multi-GPU shards) reassemble the full map bit-exactly."""
    cost, win, D, min_disp, L, R = _case(seed)
    H = L.shape[0]
    rng = np.random.default_rng(seed)
    cuts = sorted({0, H, *[int(c) for c in rng.integers(0, H + 1, 3)]})
    out = np.full(L.shape, 12345, np.int16)
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        engine.disparity_rows(L, R, min_disp, D, win, r0, r1, cost=cost, out=out)
    np.testing.assert_array_equal(out, C.disparity16(L, R, min_disp, D, win, COSTS[cost]),
                                  err_msg=f"seed {seed} cuts {cuts}")


@pytest.mark.parametrize("seed", range(2, 160, 4))
def test_random_scaled_path_matches_numpy_oracle(engine, seed):
    cost, win, D, min_disp, L, R = _case(seed)
    if cost == "ssd":
        cost = "sad"
    disparity = O.disparity_f32(C.disparity16(L, R, min_disp, D, win, COSTS[cost]))
    dn, disp, du, cf = engine.stereo_scaled(L, R, min_disp, D, win, cost=cost)
    e_dn, e_du, e_cf = O.scaled_post(disparity, min_disp, D)
    np.testing.assert_array_equal(disp, disparity, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(dn, e_dn, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(du, e_du, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(cf, e_cf, err_msg=f"seed {seed}")


@pytest.mark.parametrize("seed", range(40))
def test_random_hog_hist_bands_match_oracle(engine, seed):
    """The HOG window histograms alone over random sizes (one pixel to ~3 column-run waves),
    windows, pitches, textures and row bands [row0, row1), against the NumPy oracle."""
    rng = np.random.default_rng(5000 + seed)
    win = int(rng.choice([1, 3, 5, 7, 9, 11, 13, 15]))
    H = int(rng.choice([1, 2, 3, 9, 24, 25, 49, 70]))
    W = int(rng.choice([1, 5, 63, 239, 240, 241, 248, 256, 481, 700]))
    pitch = W + int(rng.integers(0, 9))
    g = _texture(rng, H, W, int(rng.integers(0, 4)))
    row0 = int(rng.integers(0, H))
    row1 = int(rng.integers(row0 + 1, H + 1))
    img = np.zeros((H, pitch), np.uint8)
    img[:, :W] = g
    dimg, dout = engine.dev_alloc(img.nbytes), engine.dev_alloc(H * W * 20)
    try:
        engine.to_device(dimg, img)
        engine.hog_hist_dev(dimg, H, W, pitch, win, row0, row1, dout)
        engine.synchronize()
        got = engine.to_host(dout, (H, W, 10), np.uint16)[row0:row1]
    finally:
        engine.dev_free(dimg)
        engine.dev_free(dout)
    exp = O.hog_hist(g, win)[:, row0:row1]
    np.testing.assert_array_equal(got[:, :, :9].transpose(2, 0, 1), exp, err_msg=f"{H}x{W} p{pitch} win {win} rows {row0}:{row1}")
    assert (got[:, :, 9] == 0).all()
