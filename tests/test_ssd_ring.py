"""GPU parity of the ring kind's SSD form (win 5..9, D <= 256: sv_match.hip ring_ssd): the SAD
ring's packs and cost ring with Σ(L-R)² = ΣL² + ΣR² - 2ΣLR per window column, against the C
oracle's SSD winner-take-all (first minimum); north_star's "SAD/SSD over a disparity sweep"."""
import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,win", [(16, 5), (48, 7), (64, 9), (100, 5), (128, 7), (128, 9), (192, 9),
                                   (256, 5), (256, 9), (250, 9)])
def test_ssd_ring_matches_oracle(engine, D, win):
    H, W = 21, D + 140
    L, R, _ = stereo_pair(H, W, D, seed=D * 7 + win)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, D, win, "ssd"), C.disparity16(L, R, 0, D, win, 1))


def test_ssd_ring_extremes_and_ties(engine):
    """Saturated contrast (255 vs 0 columns: the largest squared differences a window holds),
    flat frames (every disparity ties: the smallest wins) and a negative min_disp."""
    H, W, D, win = 13, 400, 128, 9
    x = np.arange(W)
    stripes = np.tile(np.where((x // 3) % 2 == 0, 255, 0).astype(np.uint8), (H, 1))
    np.testing.assert_array_equal(engine.disparity(stripes, stripes[:, ::-1].copy(), 0, D, win, "ssd"),
                                  C.disparity16(stripes, stripes[:, ::-1].copy(), 0, D, win, 1))
    flat = np.full((H, W), 200, np.uint8)
    np.testing.assert_array_equal(engine.disparity(flat, flat, 0, D, win, "ssd"),
                                  C.disparity16(flat, flat, 0, D, win, 1))
    L, R, _ = stereo_pair(H, W, D, seed=5)
    np.testing.assert_array_equal(engine.disparity(L, R, -7, D, win, "ssd"), C.disparity16(L, R, -7, D, win, 1))
