"""Host-side input normalisation shared by the drop-in entry points.

Mirrors the reference's preamble before the disparity call:
  ensure_same_size        depth_map.py:39-71, fused_depth_map.py:506-537
  BGR->gray + u8 clip     depth_map.py:871-885, fused_depth_map.py:979-984
uint8 inputs (the reference's camera frames) go to the GPU untouched — BGR->gray runs in
the HIP k_gray kernel.  Only non-uint8 inputs are normalised here, following OpenCV's
float cvtColor and the reference's ``np.uint8(np.clip(x, 0, 255))``.
"""
from __future__ import annotations

import numpy as np


def resize_linear(img: np.ndarray, w: int, h: int) -> np.ndarray:
    """cv2.resize(img, (w, h)) INTER_LINEAR on the GPU (k_resize_linear, OpenCV's fixed-point
    bilinear).  uint8 gray/BGR frames only — the reference's camera frames; there is no
    host fallback."""
    img = np.asarray(img)
    if img.dtype != np.uint8:
        raise TypeError(f"resize: uint8 frames only, got {img.dtype}")
    from .engine import get_engine
    return get_engine().resize(img, int(w), int(h))


def ensure_same_size(left_img, right_img, verbose: bool = False):
    """depth_map.py:39-71 / fused_depth_map.py:506-537: both images resized (INTER_LINEAR)
    to the smaller common size when their sizes differ."""
    h1, w1 = left_img.shape[:2]
    h2, w2 = right_img.shape[:2]
    if (h1, w1) == (h2, w2):
        return left_img, right_img
    h_min, w_min = min(h1, h2), min(w1, w2)
    left_r = resize_linear(left_img, w_min, h_min)
    right_r = resize_linear(right_img, w_min, h_min)
    if verbose:
        print(f"Resized: {w1}x{h1} and {w2}x{h2} -> {w_min}x{h_min}")
    return left_r, right_r


def to_engine_image(img: np.ndarray) -> np.ndarray:
    """uint8 HxW / HxWx3 pass through (gray conversion happens on the GPU); anything else
    is converted the way the reference does it: float cvtColor, then
    np.uint8(np.clip(gray, 0, 255))."""
    img = np.asarray(img)
    if img.dtype == np.uint8 and (img.ndim == 2 or (img.ndim == 3 and img.shape[2] == 3)):
        return img
    if img.ndim == 3:
        if img.shape[2] != 3:
            raise ValueError(f"BGR2GRAY needs 3 channels, got {img.shape[2]}")
        f = img.astype(np.float32)
        gray = f[..., 0] * np.float32(0.114) + f[..., 1] * np.float32(0.587) + \
            f[..., 2] * np.float32(0.299)
    else:
        gray = img
    return np.uint8(np.clip(gray, 0, 255))


def gray_shape(img: np.ndarray) -> tuple[int, int]:
    return tuple(np.asarray(img).shape[:2])
