"""CPU oracle for the reductions around the disparity path —
TEST INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg; never the product).

The reference's own NumPy code, restated line for line, with its OpenCV calls replaced by
the oracle's restatements:
  detect_camera_occlusion      fused_depth_map.py:131-301  (cv2.cvtColor -> bgr_to_gray,
                               cv2.calcHist -> float32 bincount)
  calibrate_midas_to_stereo    fused_depth_map.py:1169-1257 (cv2.resize -> resize_linear_f32)
  normalize_to_stereo_range    fused_depth_map.py:1503-1554
np.std / np.mean / np.percentile are the reference's NumPy calls themselves, so for these
functions parity is pinned to the reference's code (only the cv2 substitutions above are
restatements: BGR2GRAY is OpenCV's documented 14-bit fixed point, calcHist of u8 is an
exact count, and the float resize follows OpenCV's scalar float path — unpinned).
"""
from __future__ import annotations

import numpy as np

import sv_oracle as O


def calc_hist(gray: np.ndarray) -> np.ndarray:
    """cv2.calcHist([gray], [0], None, [256], [0, 256]) -> float32 (256, 1)."""
    return np.bincount(gray.ravel(), minlength=256).astype(np.float32).reshape(256, 1)


def _gray(img):
    return O.bgr_to_gray(img) if len(img.shape) == 3 else img


def occlusion_metrics(gray):
    """The per-camera metrics of fused_depth_map.py:184-248."""
    def compute_block_homogeneity(gray, block_size=48):
        h, w = gray.shape
        blocks_h = max(1, h // block_size)
        blocks_w = max(1, w // block_size)
        std_values = []
        for i in range(blocks_h):
            for j in range(blocks_w):
                y1 = i * block_size
                y2 = min((i + 1) * block_size, h)
                x1 = j * block_size
                x2 = min((j + 1) * block_size, w)
                block = gray[y1:y2, x1:x2]
                if block.size > 0:
                    std_values.append(np.std(block))
        avg_std = np.mean(std_values) if std_values else 0
        low_var_ratio = np.sum(np.array(std_values) < 12) / max(len(std_values), 1)
        return avg_std, low_var_ratio

    def compute_entropy(gray):
        hist = calc_hist(gray)
        hist = hist.flatten() + 1e-10
        hist = hist / hist.sum()
        entropy = -np.sum(hist * np.log2(hist + 1e-10))
        return entropy

    std, low = compute_block_homogeneity(gray)
    return {"std": std, "low_var": low, "contrast": np.std(gray),
            "entropy": compute_entropy(gray), "brightness": np.mean(gray)}


def detect_camera_occlusion(left_img, right_img, occlusion_threshold=0.45):
    L = occlusion_metrics(_gray(left_img))
    R = occlusion_metrics(_gray(right_img))
    STD_THRESHOLD = 28.0
    LOW_VAR_THRESHOLD = 0.55
    CONTRAST_RATIO = 2.2
    ENTROPY_RATIO = 1.6
    BRIGHTNESS_DIFF = 45.0
    left_occlusion_score = 0.0
    right_occlusion_score = 0.0
    if L["std"] < STD_THRESHOLD * 0.8:
        left_occlusion_score += 0.35
    if L["low_var"] > LOW_VAR_THRESHOLD:
        left_occlusion_score += 0.35
    if L["contrast"] < R["contrast"] / CONTRAST_RATIO and R["contrast"] > 15:
        left_occlusion_score += 0.25
    if L["entropy"] < R["entropy"] / ENTROPY_RATIO and R["entropy"] > 5.0:
        left_occlusion_score += 0.25
    if abs(L["brightness"] - R["brightness"]) > BRIGHTNESS_DIFF and L["brightness"] < 80:
        left_occlusion_score += 0.2
    if R["std"] < STD_THRESHOLD * 0.8:
        right_occlusion_score += 0.35
    if R["low_var"] > LOW_VAR_THRESHOLD:
        right_occlusion_score += 0.35
    if R["contrast"] < L["contrast"] / CONTRAST_RATIO and L["contrast"] > 15:
        right_occlusion_score += 0.25
    if R["entropy"] < L["entropy"] / ENTROPY_RATIO and L["entropy"] > 5.0:
        right_occlusion_score += 0.25
    if abs(R["brightness"] - L["brightness"]) > BRIGHTNESS_DIFF and R["brightness"] < 80:
        right_occlusion_score += 0.2
    if left_occlusion_score > occlusion_threshold and right_occlusion_score < occlusion_threshold * 0.6:
        result = 'left'
    elif right_occlusion_score > occlusion_threshold and left_occlusion_score < occlusion_threshold * 0.6:
        result = 'right'
    elif left_occlusion_score > occlusion_threshold and right_occlusion_score > occlusion_threshold:
        result = 'both'
    else:
        result = 'none'
    return result, left_occlusion_score, right_occlusion_score


def resize_linear_f32(src: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(float32 HxW, (width, height), INTER_LINEAR): OpenCV's scalar float path
    (f32 coordinates as for u8, columns clamped with zero fraction, rows clamped;
    S0*b0 + S1*b1 without contraction); exact 2x downscale = INTER_AREA fast path."""
    sH, sW = src.shape
    if (sH, sW) == (height, width):
        return src.copy()
    scale_x = 1.0 / (width / sW)
    scale_y = 1.0 / (height / sH)
    s = src.astype(np.float32)
    if scale_x == 2.0 and scale_y == 2.0:
        out = (((s[0::2, 0::2] + s[0::2, 1::2]) + s[1::2, 0::2]) + s[1::2, 1::2]) * np.float32(0.25)
        return out[:height, :width].astype(np.float32)

    def coords(dn, sn, scale, clamp):
        d = np.arange(dn, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        i = np.floor(f).astype(np.int64)
        f = (f - i.astype(np.float32)).astype(np.float32)
        if clamp:
            lo = i < 0
            f[lo] = 0
            i[lo] = 0
            hi = i >= sn - 1
            f[hi] = 0
            i[hi] = sn - 1
        return np.clip(i, 0, sn - 1), np.clip(i + 1, 0, sn - 1), f

    x0, x1, fx = coords(width, sW, scale_x, True)
    y0, y1, fy = coords(height, sH, scale_y, False)
    ax0, ax1 = (np.float32(1) - fx).astype(np.float32), fx
    by0, by1 = (np.float32(1) - fy).astype(np.float32), fy
    h0 = s[y0][:, x0] * ax0 + s[y0][:, x1] * ax1
    h1 = s[y1][:, x0] * ax0 + s[y1][:, x1] * ax1
    return (h0 * by0[:, None] + h1 * by1[:, None]).astype(np.float32)


def calibrate_midas_to_stereo(midas_depth, stereo_disparity, stereo_confidence):
    if midas_depth is None or stereo_disparity is None:
        return None
    if midas_depth.shape != stereo_disparity.shape:
        midas_depth = resize_linear_f32(midas_depth, stereo_disparity.shape[1], stereo_disparity.shape[0])
    reliable_mask = stereo_confidence > 0.7
    if np.sum(reliable_mask) < 100:
        midas_min = np.percentile(midas_depth, 5)
        midas_max = np.percentile(midas_depth, 95)
        stereo_min = np.percentile(stereo_disparity, 5)
        stereo_max = np.percentile(stereo_disparity, 95)
        if (midas_max - midas_min) < 1e-6:
            return np.full_like(midas_depth, (stereo_min + stereo_max) / 2.0)
        normalized = (midas_depth - midas_min) / (midas_max - midas_min + 1e-8)
        calibrated = stereo_min + normalized * (stereo_max - stereo_min)
        return calibrated.astype(np.float32)
    stereo_vals = stereo_disparity[reliable_mask]
    midas_vals = midas_depth[reliable_mask]
    stereo_min, stereo_max = np.percentile(stereo_vals, [10, 90])
    midas_min, midas_max = np.percentile(midas_vals, [10, 90])
    if (midas_max - midas_min) < 1e-6:
        scale = 1.0
    else:
        scale = (stereo_max - stereo_min) / (midas_max - midas_min + 1e-8)
    offset = stereo_min - midas_min * scale
    calibrated = midas_depth * scale + offset
    return calibrated.astype(np.float32)


def normalize_to_stereo_range(depth_map, stereo_disparity):
    if depth_map is None or stereo_disparity is None:
        return None
    stereo_valid = stereo_disparity > 0
    if np.any(stereo_valid):
        stereo_min = np.percentile(stereo_disparity[stereo_valid], 5)
        stereo_max = np.percentile(stereo_disparity[stereo_valid], 95)
    else:
        stereo_min, stereo_max = 0, 255
    d_min = np.percentile(depth_map, 5)
    d_max = np.percentile(depth_map, 95)
    if (d_max - d_min) < 1e-6:
        normalized = np.full_like(depth_map, (stereo_min + stereo_max) / 2.0)
    else:
        normalized = (depth_map - d_min) / (d_max - d_min + 1e-8)
        normalized = stereo_min + normalized * (stereo_max - stereo_min)
    return normalized.astype(np.float32)
