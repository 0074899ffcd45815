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

try:  # optional: exact cv2.resize when available
    import cv2  # type: ignore
except Exception:  # pragma: no cover
    cv2 = None


def _resize_linear(img: np.ndarray, w: int, h: int) -> np.ndarray:
    """Bilinear resize with half-pixel centres (cv2.INTER_LINEAR geometry; not its
    fixed-point rounding — only used when cv2 is absent and sizes differ)."""
    H, W = img.shape[:2]
    ys = np.clip((np.arange(h) + 0.5) * (H / h) - 0.5, 0, H - 1)
    xs = np.clip((np.arange(w) + 0.5) * (W / w) - 0.5, 0, W - 1)
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    y1 = np.minimum(y0 + 1, H - 1)
    x1 = np.minimum(x0 + 1, W - 1)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    a = img.astype(np.float32)
    if a.ndim == 3:
        fy = fy[..., None]
        fx = fx[..., None]
    top = a[y0][:, x0] * (1 - fx) + a[y0][:, x1] * fx
    bot = a[y1][:, x0] * (1 - fx) + a[y1][:, x1] * fx
    out = top * (1 - fy) + bot * fy
    if np.issubdtype(img.dtype, np.integer):
        out = np.clip(np.rint(out), np.iinfo(img.dtype).min, np.iinfo(img.dtype).max)
    return out.astype(img.dtype)


def ensure_same_size(left_img, right_img, verbose: bool = False):
    h1, w1 = left_img.shape[:2]
    h2, w2 = right_img.shape[:2]
    if (h1, w1) == (h2, w2):
        return left_img, right_img
    h_min, w_min = min(h1, h2), min(w1, w2)
    if cv2 is not None:
        left_r = cv2.resize(left_img, (w_min, h_min))
        right_r = cv2.resize(right_img, (w_min, h_min))
    else:
        left_r = _resize_linear(left_img, w_min, h_min)
        right_r = _resize_linear(right_img, w_min, h_min)
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
