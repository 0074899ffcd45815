"""GPU parity of the split ring kind: SAD windows with 256 < D <= 512 (the reference's own
default NUM_DISP = 16*20 = 320 with WINDOW_SIZE = 7, depth_map.py:31-33) run the ring kind
twice (d < 256 and d >= 256) into argmin-key planes and merge them (sv_match.hip
ring_split / k_merge_ring_keys), against the C oracle's winner-take-all (first minimum)."""
import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,win", [(260, 5), (272, 7), (320, 7), (320, 9), (336, 11), (384, 13),
                                   (448, 15), (512, 7), (257, 9)])
def test_split_ring_matches_oracle(engine, D, win):
    H, W = 23, D + 150
    L, R, _ = stereo_pair(H, W, D, seed=D + win)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win), C.disparity16(L, R, 0, D, win, 0))


@pytest.mark.parametrize("min_disp", [-16, 5])
def test_split_ring_min_disp(engine, min_disp):
    H, W, D, win = 17, 520, 320, 7
    L, R, _ = stereo_pair(H, W, D, seed=3, min_disp=max(0, min_disp))
    np.testing.assert_array_equal(engine.disparity(L, R, min_disp, D, win),
                                  C.disparity16(L, R, min_disp, D, win, 0))


def test_split_ring_ties_go_to_the_smaller_disparity(engine):
    """Flat and periodic images: every disparity costs the same (or the pattern repeats
    across the two passes' ranges), so the first minimum must come from pass A."""
    H, W, D, win = 13, 700, 320, 7
    flat = np.full((H, W), 77, np.uint8)
    np.testing.assert_array_equal(engine.disparity(flat, flat, 0, D, win), C.disparity16(flat, flat, 0, D, win, 0))
    x = np.arange(W)
    per = np.tile(((x % 8) * 30).astype(np.uint8), (H, 1))   # period 8: costs repeat every 8 d
    np.testing.assert_array_equal(engine.disparity(per, per, 0, D, win), C.disparity16(per, per, 0, D, win, 0))


def test_split_ring_row_band_and_frame_batch(engine):
    """A row band (rows [7, 30)) and a pitched 3-frame batch through the device entry point:
    the key planes follow the output's pitch and frame stride."""
    H, W, D, win = 37, 480, 320, 7
    L, R, _ = stereo_pair(H, W, D, seed=21)
    got = engine.disparity_rows(L, R, 0, D, win, 7, 30)
    exp = C.disparity16(L, R, 0, D, win, 0)
    np.testing.assert_array_equal(got[7:30], exp[7:30])
    nf, pitch = 3, W + 16
    fs = (H + 2) * pitch
    Ls = np.zeros((nf, H + 2, pitch), np.uint8)
    Rs = np.zeros_like(Ls)
    for z in range(nf):
        l, r, _ = stereo_pair(H, W, D, seed=40 + z)
        Ls[z, :H, :W], Rs[z, :H, :W] = l, r
    opitch, ofs = W + 8, H * (W + 8) + 24
    dL, dR, dO = engine.dev_alloc(Ls.nbytes), engine.dev_alloc(Rs.nbytes), engine.dev_alloc(nf * ofs * 2)
    try:
        engine.to_device(dL, Ls)
        engine.to_device(dR, Rs)
        engine.disparity_batch_dev(dL, dR, nf, H, W, pitch, fs, 0, D, win, "sad", dO, opitch, ofs)
        engine.synchronize()
        flat = engine.to_host(dO, (nf * ofs,), np.int16)
        for z in range(nf):
            got = flat[z * ofs:z * ofs + H * opitch].reshape(H, opitch)[:, :W]
            np.testing.assert_array_equal(got, C.disparity16(Ls[z, :H, :W], Rs[z, :H, :W], 0, D, win, 0))
    finally:
        for p in (dL, dR, dO):
            engine.dev_free(p)
