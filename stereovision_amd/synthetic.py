"""Synthetic rectified stereo pairs (SURVEY.md §8(d) "Synthetic inputs").

* left  = uniform u8 noise, box-blurred 3x3 and re-quantised to u8 (matchable texture);
* right(x, y) = left(x + d_gt(x, y), y) with a piecewise-planar integer ground truth:
  background plane d = D/4, a fronto-parallel rectangle at d = D/2 and a slanted strip
  from D/8 to 3D/8; samples that fall outside the left image get fresh noise;
* +-2 LSB uniform noise is added to the right image (``noise=2``).

Deterministic for a given seed (numpy ``default_rng``).  BGR variants replicate the gray
plane three times (B = G = R), so BGR->gray is identity-exact.
"""
from __future__ import annotations

import numpy as np


def _texture(rng: np.random.Generator, H: int, W: int) -> np.ndarray:
    n = rng.integers(0, 256, size=(H + 2, W + 2), dtype=np.int32)
    s = np.zeros((H, W), np.int32)
    for j in range(3):
        for i in range(3):
            s += n[j:j + H, i:i + W]
    return ((s + 4) // 9).astype(np.uint8)


def ground_truth(H: int, W: int, num_disp: int, min_disp: int = 0) -> np.ndarray:
    """Integer disparity map (in right-image coordinates) with values in [minD, minD+D)."""
    D = num_disp
    d = np.full((H, W), D // 4, np.int32)
    y0, y1 = int(0.30 * H), int(0.70 * H)
    x0, x1 = int(0.35 * W), int(0.60 * W)
    d[y0:y1, x0:x1] = D // 2
    sx0, sx1 = int(0.68 * W), int(0.92 * W)
    if sx1 > sx0:
        ramp = D // 8 + (np.arange(sx1 - sx0) * (3 * D // 8 - D // 8)) // max(1, sx1 - sx0)
        d[int(0.15 * H):int(0.85 * H), sx0:sx1] = ramp[None, :]
    return np.clip(d + min_disp, min_disp, min_disp + D - 1)


def stereo_pair(H: int, W: int, num_disp: int, seed: int = 0, min_disp: int = 0,
                noise: int = 2) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Returns (left u8 HxW, right u8 HxW, d_gt int32 HxW)."""
    rng = np.random.default_rng(seed)
    left = _texture(rng, H, W)
    fresh = _texture(rng, H, W)
    dgt = ground_truth(H, W, num_disp, min_disp)
    xs = np.arange(W)[None, :] + dgt
    inside = (xs >= 0) & (xs < W)
    rows = np.arange(H)[:, None]
    right = np.where(inside, left[rows, np.clip(xs, 0, W - 1)], fresh).astype(np.int32)
    if noise:
        right = right + rng.integers(-noise, noise + 1, size=(H, W), dtype=np.int32)
    return left, np.clip(right, 0, 255).astype(np.uint8), dgt


def to_bgr(gray: np.ndarray) -> np.ndarray:
    return np.repeat(gray[:, :, None], 3, axis=2)


def stereo_batch(n: int, H: int, W: int, num_disp: int, seed: int = 0, min_disp: int = 0):
    """n independent pairs stacked as (n, H, W) u8 arrays (seeds seed .. seed+n-1)."""
    L = np.empty((n, H, W), np.uint8)
    R = np.empty((n, H, W), np.uint8)
    for i in range(n):
        L[i], R[i], _ = stereo_pair(H, W, num_disp, seed + i, min_disp)
    return L, R


def synthetic_calibration(width: int, height: int, seed: int = 0) -> dict:
    """A plausible stereo calibration in the reference's file schema
    (stereo_calibration.py:276-297): two ~70-degree-FOV cameras with radial/tangential
    distortion, a 8 cm baseline and a ~1 degree relative rotation."""
    rng = np.random.default_rng(seed)
    f = 0.7 * width

    def cam(df, dc):
        return np.array([[f + df[0], 0, width / 2 + dc[0]], [0, f + df[1], height / 2 + dc[1]],
                         [0, 0, 1.0]])

    r = rng.normal(size=3)
    r *= np.deg2rad(1.0) / np.linalg.norm(r)
    theta = np.linalg.norm(r)
    k = r / theta
    kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.cos(theta) * np.eye(3) + (1 - np.cos(theta)) * np.outer(k, k) + np.sin(theta) * kx
    return {
        "mtx_left": cam(rng.normal(size=2) * 0.005 * f, rng.normal(size=2) * 0.01 * width),
        "dist_left": np.array([[-0.12, 0.05, 0.001, -0.0008, -0.01]]),
        "mtx_right": cam(rng.normal(size=2) * 0.005 * f, rng.normal(size=2) * 0.01 * width),
        "dist_right": np.array([[-0.10, 0.04, -0.0005, 0.0009, -0.008]]),
        "R": R, "T": np.array([[-0.08], [0.001], [0.0005]]),
        "img_size": (int(width), int(height)),
    }
