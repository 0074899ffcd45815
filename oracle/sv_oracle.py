"""CPU oracle for the stereo-disparity hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path
(``stereovision_amd``) never imports it and fails loudly when its HIP library is missing.

What it restates
----------------
* The reference's Python around the disparity call, line by line:
  - gray conversion + uint8 clip          ``depth_map.py:868-885``, ``fused_depth_map.py:976-984``
  - ``/16.0`` scaling + ``medianBlur(.,5)``  ``depth_map.py:909-912``, ``fused_depth_map.py:1004-1007``
  - depth post (fx=700, B=0.08, clip, mask, u8 normalise)   ``depth_map.py:915-937``
  - scaled-app post (clip, u8 normalise, confidence mask)   ``fused_depth_map.py:1010-1029``
  - scaled D / window rules                 ``fused_depth_map.py:2258-2266``
* The disparity arithmetic itself.  The reference calls OpenCV
  ``cv2.StereoSGBM_create(...).compute`` (``depth_map.py:894-909``,
  ``fused_depth_map.py:988-1004``), a third-party C++ library that is NOT vendored, whose
  version is NOT pinned (no requirements file) and which is NOT importable in this image.
  BASELINE.json's north_star replaces that call with a block-matching engine (SAD / SSD
  winner-take-all over a disparity sweep, HOG-descriptor matching, Harris response).  The
  semantics of that engine are DEFINED HERE (see DESIGN.md "Semantics"), following the
  OpenCV conventions the reference depends on:
  - output int16 = d * 16, invalid = (minDisparity - 1) * 16, columns outside
    [max(minD+numD, 0), W + min(minD, 0)) invalid (SGBM's ``minX1``/``maxX1`` band);
  - cvtColor BGR2GRAY 14-bit fixed point (B*1868 + G*9617 + R*4899 + 2^13) >> 14;
  - medianBlur ksize 5 with replicate border;
  - cornerHarris(blockSize=3, ksize=3, k=0.04) with BORDER_REFLECT_101.

PARITY STATUS: **parity unpinned** against the reference's own outputs.  The reference
has no tests, no fixtures and no golden vectors, and its arithmetic
lives in OpenCV, which cannot be imported here.  This oracle is pinned instead by
(a) analytic known-answer tests (integer-shift pairs recover the shift exactly, flat
images give cost ties resolved to minD and Harris R == 0), and (b) agreement with the
independent C restatement in ``oracle/sv_oracle.c``.  Golden fixtures under
``tests/golden/`` are generated from this module by ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import numpy as np

COST_SAD = 0
COST_SSD = 1
COST_HOG = 2

# Harris constants (cv2.cornerHarris convention, blockSize=3, ksize=3, CV_8U source):
# scale = 1 / ((1 << (ksize-1)) * blockSize * 255)
HARRIS_K = np.float32(0.04)
HARRIS_SCALE2 = np.float32((1.0 / (4.0 * 3.0 * 255.0)) ** 2)

# HOG orientation boundaries: 9 unsigned bins of 20 degrees, integer tangent tests.
HOG_BINS = 9
HOG_COS = np.array([int(round(16384 * np.cos(np.deg2rad(20 * k)))) for k in range(1, 9)], np.int64)
HOG_SIN = np.array([int(round(16384 * np.sin(np.deg2rad(20 * k)))) for k in range(1, 9)], np.int64)


# ----------------------------------------------------------------------------------------
# Preamble: gray conversion  (depth_map.py:871-885, fused_depth_map.py:979-984)
# ----------------------------------------------------------------------------------------
def bgr_to_gray(img: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for uint8 (OpenCV 14-bit fixed point)."""
    if img.ndim == 2:
        return img
    b = img[..., 0].astype(np.int32)
    g = img[..., 1].astype(np.int32)
    r = img[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def valid_columns(W: int, min_disp: int, num_disp: int) -> tuple[int, int]:
    """SGBM's matched-column band [minX1, maxX1): outside it the output is invalid."""
    max_d = min_disp + num_disp
    x0 = max(max_d, 0)
    x1 = min(W + min(min_disp, 0), W)
    return x0, max(x0, x1)


def key_bits(num_disp: int) -> int:
    """Bits used by the (cost << bits | d) argmin key (first-min tie-break)."""
    return max(1, int(num_disp - 1).bit_length())


def max_cost(win: int, cost: int) -> int:
    if cost == COST_SAD:
        return win * win * 255
    if cost == COST_SSD:
        return win * win * 255 * 255
    return HOG_BINS * win * win * 255


def _box_sum(a: np.ndarray, r: int) -> np.ndarray:
    """Sum over (2r+1)x(2r+1) windows of an array padded by r on every side."""
    a = a.astype(np.int64)
    c = np.zeros((a.shape[0] + 1, a.shape[1] + 1), np.int64)
    c[1:, 1:] = a.cumsum(0).cumsum(1)
    k = 2 * r + 1
    return c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]


# ----------------------------------------------------------------------------------------
# Gradients: Sobel 3x3, BORDER_REFLECT_101 (shared by Harris and HOG)
# ----------------------------------------------------------------------------------------
def _reflect101(idx: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(idx)
    idx = np.where(idx < 0, -idx, idx)
    idx = np.where(idx >= n, 2 * (n - 1) - idx, idx)
    return idx


def sobel(gray: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    H, W = gray.shape
    ry = _reflect101(np.arange(-1, H + 1), H)
    rx = _reflect101(np.arange(-1, W + 1), W)
    p = gray.astype(np.int32)[ry][:, rx]
    gx = (p[:-2, 2:] + 2 * p[1:-1, 2:] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[1:-1, :-2] + p[2:, :-2])
    gy = (p[2:, :-2] + 2 * p[2:, 1:-1] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[:-2, 1:-1] + p[:-2, 2:])
    return gx.astype(np.int32), gy.astype(np.int32)


def harris(gray: np.ndarray) -> np.ndarray:
    """Harris response (cornerHarris blockSize=3, ksize=3, k=0.04, REFLECT_101), float32.

    The structure tensor is summed exactly in integers, then scaled once:
    a = f32(Sxx) * s^2 etc.; R = (a*c - b*b) - k*((a+c)*(a+c)), each op rounded to f32.
    """
    H, W = gray.shape
    gx, gy = sobel(gray)
    ry = _reflect101(np.arange(-1, H + 1), H)
    rx = _reflect101(np.arange(-1, W + 1), W)
    out = []
    for prod in (gx * gx, gx * gy, gy * gy):
        p = prod.astype(np.int64)[ry][:, rx]
        s = np.zeros((H, W), np.int64)
        for j in range(3):
            for i in range(3):
                s += p[j:j + H, i:i + W]
        out.append(s.astype(np.float32) * HARRIS_SCALE2)
    a, b, c = out
    t1 = a * c
    t2 = b * b
    t3 = a + c
    t4 = t3 * t3
    return ((t1 - t2) - HARRIS_K * t4).astype(np.float32)


def hog_pixel(gray: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Per-pixel (bin, magnitude): unsigned 9-bin orientation by integer tangent tests,
    magnitude (|gx| + |gy|) >> 3 in [0, 255]."""
    gx, gy = sobel(gray)
    mag = ((np.abs(gx) + np.abs(gy)) >> 3).astype(np.int32)
    flip = (gy < 0) | ((gy == 0) & (gx < 0))
    fx = np.where(flip, -gx, gx).astype(np.int64)
    fy = np.where(flip, -gy, gy).astype(np.int64)
    b = np.zeros(gray.shape, np.int32)
    for k in range(8):
        b += (HOG_COS[k] * fy - HOG_SIN[k] * fx >= 0).astype(np.int32)
    return b, mag


def hog_hist(gray: np.ndarray, win: int) -> np.ndarray:
    """Window histograms H[b, y, x] = sum over the win x win window (replicate clamp)."""
    H, W = gray.shape
    r = win // 2
    b, mag = hog_pixel(gray)
    cy = np.clip(np.arange(-r, H + r), 0, H - 1)
    cx = np.clip(np.arange(-r, W + r), 0, W - 1)
    out = np.zeros((HOG_BINS, H, W), np.int64)
    for k in range(HOG_BINS):
        m = np.where(b == k, mag, 0)
        out[k] = _box_sum(m[cy][:, cx], r)
    return out.astype(np.uint16)


# ----------------------------------------------------------------------------------------
# The replaced call: stereo.compute(gray_left, gray_right) -> int16 (x16)
# ----------------------------------------------------------------------------------------
def disparity16(L: np.ndarray, R: np.ndarray, min_disp: int, num_disp: int, win: int,
                cost: int = COST_SAD, rows: tuple[int, int] | None = None) -> np.ndarray:
    """Winner-take-all disparity, int16 scaled by 16 (SGBM output convention).

    cost(x,y,d) = sum_{|i|,|j|<=r} f(Lp(x+i, y+j) - Rp(x+i-d, y+j)), f = |.| (SAD) or (.)^2
    (SSD), Lp/Rp = replicate-clamped images; HOG: sum_b |HL_b(x,y) - HR_b(x-d,y)|.
    d* = first argmin over d in [minD, minD+numD).  ``rows`` restricts the output rows
    (used to check row-band sharding); rows outside are left invalid.
    """
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    H, W = L.shape
    r = win // 2
    y0, y1 = (0, H) if rows is None else rows
    invalid = (min_disp - 1) * 16
    out = np.full((H, W), invalid, np.int16)
    x0, x1 = valid_columns(W, min_disp, num_disp)
    if x1 <= x0 or y1 <= y0:
        return out
    nx = x1 - x0
    best_c = np.full((y1 - y0, nx), np.iinfo(np.int64).max, np.int64)
    best_d = np.zeros((y1 - y0, nx), np.int64)
    if cost == COST_HOG:
        hl = hog_hist(L, win).astype(np.int64)[:, y0:y1, x0:x1]
        hr = hog_hist(R, win).astype(np.int64)[:, y0:y1, :]
        xs = np.arange(x0, x1)
        for d in range(min_disp, min_disp + num_disp):
            cx = np.clip(xs - d, 0, W - 1)
            c = np.abs(hl - hr[:, :, cx]).sum(0)
            m = c < best_c
            best_c[m] = c[m]
            best_d[m] = d
    else:
        cy = np.clip(np.arange(y0 - r, y1 + r), 0, H - 1)
        xs = np.arange(x0 - r, x1 + r)
        lp = L[cy][:, np.clip(xs, 0, W - 1)].astype(np.int64)
        rows_r = R[cy]
        for d in range(min_disp, min_disp + num_disp):
            rp = rows_r[:, np.clip(xs - d, 0, W - 1)].astype(np.int64)
            diff = lp - rp
            ad = np.abs(diff) if cost == COST_SAD else diff * diff
            c = _box_sum(ad, r)
            m = c < best_c
            best_c[m] = c[m]
            best_d[m] = d
    out[y0:y1, x0:x1] = (best_d * 16).astype(np.int16)
    return out


def median5(a: np.ndarray) -> np.ndarray:
    """cv2.medianBlur(a, 5): 5x5 median, replicate border (exact element selection)."""
    H, W = a.shape
    cy = np.clip(np.arange(-2, H + 2), 0, H - 1)
    cx = np.clip(np.arange(-2, W + 2), 0, W - 1)
    p = a[cy][:, cx]
    stack = np.stack([p[j:j + H, i:i + W] for j in range(5) for i in range(5)])
    return np.partition(stack, 12, axis=0)[12]


# ----------------------------------------------------------------------------------------
# Post-processing, restated from the reference
# ----------------------------------------------------------------------------------------
def disparity_f32(d16: np.ndarray) -> np.ndarray:
    """``stereo.compute(...).astype(np.float32) / 16.0`` then ``cv2.medianBlur(.,5)``
    (depth_map.py:909-912).  The median of i16/16 values equals median(i16)/16."""
    return median5(d16).astype(np.float32) / np.float32(16.0)


def depth_post(disparity: np.ndarray, min_depth: float, max_depth: float,
               min_disp_global: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """depth_map.py:915-937 (fx = 700 because 'calibration_data' is never a key of the
    calibration dict, :915-920; BASELINE = 0.08, :923).  Returns (depth_final f32,
    depth_normalized u8).  NumPy-2 (NEP 50) keeps every step in float32."""
    fx = 700
    baseline = 0.08
    depth = (fx * baseline) / (disparity + 1e-6)
    depth_clipped = np.clip(depth, min_depth, max_depth)
    valid_mask = (disparity > min_disp_global) & (depth_clipped >= min_depth) & \
        (depth_clipped <= max_depth)
    depth_final = np.where(valid_mask, depth_clipped, 0)
    depth_normalized = ((depth_clipped - min_depth) / (max_depth - min_depth) * 255).astype(np.uint8)
    return depth_final, depth_normalized


def scaled_post(disparity: np.ndarray, min_disp: int, num_disp: int
                ) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """fused_depth_map.py:1010-1029.  Returns (disparity_normalized f32, u8 image fed to
    the colormap, confidence f32)."""
    disparity_clipped = np.clip(disparity, min_disp, min_disp + num_disp - 1)
    disparity_normalized = ((disparity_clipped - min_disp) / num_disp * 255.0).astype(np.uint8)
    valid_mask = (disparity > min_disp + 1) & (disparity < min_disp + num_disp - 1)
    confidence = np.zeros_like(disparity, dtype=np.float32)
    confidence[valid_mask] = 1.0
    return disparity_normalized.astype(np.float32), disparity_normalized, confidence


def scaled_params(processing_scale: float, num_disp_base: int = 320,
                  window_size_base: int = 7) -> tuple[int, int]:
    """fused_depth_map.py:2258-2266."""
    num_disp_scaled = max(16, int(num_disp_base * processing_scale) // 16 * 16)
    window_size_scaled = max(5, int(window_size_base * processing_scale))
    if window_size_scaled % 2 == 0:
        window_size_scaled += 1
    return num_disp_scaled, window_size_scaled


def create_depth_map(left, right, min_disp=0, num_disp=320, win=7, min_depth=0.3,
                     max_depth=2.0, cost=COST_SAD):
    """Whole app-1 path (depth_map.py:837-939) minus the colormap."""
    gl, gr = bgr_to_gray(left), bgr_to_gray(right)
    d16 = disparity16(gl, gr, min_disp, num_disp, win, cost)
    disparity = disparity_f32(d16)
    depth_final, depth_norm = depth_post(disparity, min_depth, max_depth, min_disp)
    return depth_final, disparity, depth_norm


def create_depth_map_stereo_scaled(left, right, min_disp, num_disp, win, cost=COST_SAD):
    """Whole app-2 path (fused_depth_map.py:934-1029) minus the colormap."""
    gl, gr = bgr_to_gray(left), bgr_to_gray(right)
    d16 = disparity16(gl, gr, min_disp, num_disp, win, cost)
    disparity = disparity_f32(d16)
    dn, dn_u8, conf = scaled_post(disparity, min_disp, num_disp)
    return dn, disparity, dn_u8, conf
