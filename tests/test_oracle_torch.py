"""A second independent check of the oracle's conventions, with PyTorch's CPU operators (test
infrastructure only — the product never imports torch): full frames, borders included, where
tests/test_oracle_scipy.py compares interior columns.

* the SAD / SSD winner-take-all: replicate-clamped L and R (F.pad 'replicate' + a clamped
  column gather), the (2r+1)² box as a float64 conv2d of ones (exact for these integer sums),
  the first minimum over d by torch.argmin (documented: the first minimal index), the invalid
  band outside [X0, X1) — against oracle/sv_oracle.py and oracle/sv_oracle.c;
* medianBlur(5): F.pad 'replicate' + unfold + torch.median (25 values: the 13th);
* the Harris response: Sobel as conv2d on 'reflect' padding (torch's reflect = OpenCV's
  REFLECT_101), products, 3×3 box on reflect-padded products, float64.

Reference call sites: depth_map.py:909-912 (StereoSGBM.compute, medianBlur); north_star's
Harris (cornerHarris(3, 3, 0.04))."""
import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

torch = F = None


@pytest.fixture(autouse=True)
def _torch():
    """torch is imported by the tests themselves, never at collection: the GPU test process
    collects this module too (deselected), and must map exactly one HIP runtime — ROCm's, not
    torch's bundled copy (test_gpu_parity.py::test_row_tiled_module_and_single_hip_runtime)."""
    global torch, F
    torch = pytest.importorskip("torch")
    F = torch.nn.functional


def _wta_torch(L, R, min_disp, num_disp, win, ssd=False):
    H, W = L.shape
    r = win // 2
    Lt = torch.from_numpy(L.astype(np.float64))[None, None]
    Lp = F.pad(Lt, (r, r, r, r), mode="replicate")[0, 0]              # Lp(x+i, y+j)
    Rrows = F.pad(torch.from_numpy(R.astype(np.float64))[None, None], (0, 0, r, r), mode="replicate")[0, 0]
    cols = torch.arange(-r, W + r)
    box = torch.ones((1, 1, win, win), dtype=torch.float64)
    costs = []
    for d in range(min_disp, min_disp + num_disp):
        Rp = Rrows[:, torch.clamp(cols - d, 0, W - 1)]                  # Rp(x+i-d, y+j)
        diff = Lp - Rp
        a = diff * diff if ssd else diff.abs()
        costs.append(F.conv2d(a[None, None], box)[0, 0])
    vol = torch.stack(costs)                                            # [D, H, W]
    best = torch.argmin(vol, dim=0).numpy().astype(np.int64) + min_disp
    out = np.full((H, W), (min_disp - 1) * 16, np.int16)
    x0, x1 = O.valid_columns(W, min_disp, num_disp)
    out[:, x0:x1] = (best[:, x0:x1] * 16).astype(np.int16)
    return out


@pytest.mark.parametrize("cost,win,min_disp,num_disp,H,W", [
    ("sad", 9, 0, 32, 23, 80), ("sad", 5, -6, 24, 17, 61), ("ssd", 7, 0, 16, 19, 50),
    ("sad", 15, 4, 16, 31, 70), ("ssd", 3, -3, 12, 9, 33), ("sad", 1, 0, 8, 6, 20),
    ("sad", 11, 0, 64, 12, 96)])
def test_disparity_matches_torch_full_frame(cost, win, min_disp, num_disp, H, W):
    L, R, _ = stereo_pair(H, W, max(1, num_disp + max(0, min_disp)), seed=H * 7 + W)
    c = O.COST_SSD if cost == "ssd" else O.COST_SAD
    exp = _wta_torch(L, R, min_disp, num_disp, win, ssd=cost == "ssd")
    np.testing.assert_array_equal(O.disparity16(L, R, min_disp, num_disp, win, c), exp)
    np.testing.assert_array_equal(C.disparity16(L, R, min_disp, num_disp, win, c), exp)


def test_disparity_ties_take_the_first_minimum_torch():
    """Flat and periodic images: every d ties somewhere; the first minimum wins everywhere."""
    H, W = 12, 48
    flat = np.full((H, W), 77, np.uint8)
    per = np.tile((np.arange(W) % 4 * 60).astype(np.uint8), (H, 1))
    for L, R in ((flat, flat), (per, per)):
        exp = _wta_torch(L, R, 0, 16, 5)
        np.testing.assert_array_equal(O.disparity16(L, R, 0, 16, 5), exp)


@pytest.mark.parametrize("shape", [(21, 34), (4, 4), (1, 7), (9, 1)])
def test_median5_matches_torch(shape):
    rng = np.random.default_rng(shape[0] * 100 + shape[1])
    a = rng.integers(-300, 3000, shape).astype(np.int16)
    t = F.pad(torch.from_numpy(a.astype(np.float64))[None, None], (2, 2, 2, 2), mode="replicate")
    win = F.unfold(t, 5)[0]                      # [25, H*W]
    exp = torch.median(win, dim=0).values.numpy().reshape(shape)
    np.testing.assert_array_equal(O.median5(a).astype(np.float64), exp)


def test_harris_matches_torch_reflect101():
    rng = np.random.default_rng(3)
    g = rng.integers(0, 256, (29, 41), dtype=np.uint8)
    t = torch.from_numpy(g.astype(np.float64))[None, None]
    s = 1.0 / (4.0 * 3.0 * 255.0)
    kx = torch.tensor([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], dtype=torch.float64)[None, None]
    p = F.pad(t, (1, 1, 1, 1), mode="reflect")   # reflect = d c b | a b c d (REFLECT_101)
    dx = F.conv2d(p, kx) * s
    dy = F.conv2d(p, kx.transpose(2, 3)) * s
    box = torch.ones((1, 1, 3, 3), dtype=torch.float64)
    sm = [F.conv2d(F.pad(v, (1, 1, 1, 1), mode="reflect"), box) for v in (dx * dx, dx * dy, dy * dy)]
    a, b, c = (v[0, 0] for v in sm)
    exp = ((a * c - b * b) - 0.04 * (a + c) ** 2).numpy()
    np.testing.assert_allclose(O.harris(g).astype(np.float64), exp, rtol=2e-5, atol=1e-8)
