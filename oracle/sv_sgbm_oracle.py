"""CPU oracle of the SGBM-3WAY disparity mode — TEST INFRASTRUCTURE ONLY (tests/ and
bench.py's cpu_baseline leg; never the product).

The reference's disparity call is ``cv2.StereoSGBM_create(minDisparity, numDisparities,
blockSize, P1=8*3*w^2, P2=32*3*w^2, disp12MaxDiff=1, uniquenessRatio=10,
speckleWindowSize=100, speckleRange=32, preFilterCap=63, mode=MODE_SGBM_3WAY).compute``
(depth_map.py:894-909, fused_depth_map.py:988-1004).  OpenCV is third-party, not vendored,
version-unpinned and not importable here, so this module restates its published algorithm
(calib3d/src/stereosgbm.cpp: calcPixelCostBT, the block-sum loop, the 3-way dynamic
programming, uniqueness, sub-pixel, left-right check, filterSpeckles) and DEFINES the
engine's SGBM mode.  Deviations fixed here (documented in DESIGN.md):
  * one stripe: OpenCV splits the rows into getNumThreads() stripes whose top-down paths
    restart at each stripe (so its output depends on the thread count); here the vertical
    path runs over the whole image (OpenCV with one thread);
  * path and aggregated costs in int32 (OpenCV stores them in int16 with saturate_cast;
    identical while they stay within int16).
PARITY STATUS: **parity unpinned** against OpenCV (absent; no golden vectors).  Pinned by
known answers in tests/test_sgbm.py (integer-shift pairs, invalid-band conventions,
speckle removal of small islands) and by agreement with the GPU kernels.

Layout conventions: band columns [X0, X1) with X0 = max(minD + D, 0), X1 = W + min(minD, 0)
(SGBM's minX1/maxX1); disparity index k in [0, D) means d = minD + k; output int16 x16
with invalid = (minD - 1) * 16.
"""
from __future__ import annotations

from collections import deque

import numpy as np


def params_for(win: int) -> dict:
    """The reference's SGBM parameters for a block size (depth_map.py:894-906)."""
    return {"P1": 8 * 3 * win * win, "P2": 32 * 3 * win * win, "disp12MaxDiff": 1,
            "uniquenessRatio": 10, "speckleWindowSize": 100, "speckleRange": 32,
            "preFilterCap": 63}


# ----------------------------------------------------------------------------------------
# pixel cost: Birchfield-Tomasi on the clipped x-Sobel image + BT on the raw image >> 2
# ----------------------------------------------------------------------------------------
def _prefilter(img: np.ndarray, cap: int):
    """Per row: the two channels calcPixelCostBT matches.  Channel 0: clip(x-Sobel, -cap,
    cap) + cap with rows replicated at the top/bottom; channel 1: the raw pixel.  Columns 0
    and W-1 of BOTH channels hold tab[0] = cap (OpenCV's border fill)."""
    a = img.astype(np.int32)
    H, W = a.shape
    up = np.vstack([a[:1], a[:-1]])
    dn = np.vstack([a[1:], a[-1:]])
    pf = np.full((H, W), cap, np.int32)
    raw = np.full((H, W), cap, np.int32)
    if W > 2:
        s = (a[:, 2:] - a[:, :-2]) * 2 + up[:, 2:] - up[:, :-2] + dn[:, 2:] - dn[:, :-2]
        pf[:, 1:-1] = np.clip(s, -cap, cap) + cap
        raw[:, 1:-1] = a[:, 1:-1]
    return pf, raw


def _half_range(c: np.ndarray):
    """(min, max) of {c, (c + c_left)/2, (c + c_right)/2} per pixel (BT's interval)."""
    W = c.shape[1]
    cl = np.concatenate([c[:, :1], c[:, :-1]], 1)
    cr = np.concatenate([c[:, 1:], c[:, -1:]], 1)
    vl = (c + cl) // 2
    vr = (c + cr) // 2
    vl[:, 0] = c[:, 0]
    vr[:, W - 1] = c[:, W - 1]
    return np.minimum(np.minimum(vl, vr), c), np.maximum(np.maximum(vl, vr), c)


def pixel_cost(L, R, min_disp: int, num_disp: int, cap: int = 63) -> np.ndarray:
    """[H, X1-X0, D] int32 pixel costs of the band (calcPixelCostBT)."""
    H, W = L.shape
    D = num_disp
    X0 = max(min_disp + D, 0)
    X1 = W + min(min_disp, 0)
    X1 = max(X1, X0)
    out = np.zeros((H, X1 - X0, D), np.int32)
    if X1 == X0:
        return out
    for ch, shift in ((0, 0), (1, 2)):
        p1 = _prefilter(L, cap)[ch]
        p2 = _prefilter(R, cap)[ch]
        u0, u1 = _half_range(p1)
        v0, v1 = _half_range(p2)
        xs = np.arange(X0, X1)
        for k in range(D):
            xr = xs - (min_disp + k)
            u, ul, uh = p1[:, xs], u0[:, xs], u1[:, xs]
            v, vl, vh = p2[:, xr], v0[:, xr], v1[:, xr]
            c0 = np.maximum(np.maximum(0, u - vh), vl - u)
            c1 = np.maximum(np.maximum(0, v - uh), ul - v)
            out[:, :, k] += np.minimum(c0, c1) >> shift
    return out


def block_cost(pc: np.ndarray, win: int) -> np.ndarray:
    """Window sums of the pixel cost with replicated band columns and image rows."""
    H, Wb, D = pc.shape
    r = win // 2
    if Wb == 0:
        return pc.copy()
    xi = np.clip(np.arange(-r, Wb + r), 0, Wb - 1)
    yi = np.clip(np.arange(-r, H + r), 0, H - 1)
    p = pc[yi][:, xi]
    cs = np.cumsum(np.cumsum(p, 0, dtype=np.int64), 1, dtype=np.int64)
    cs = np.pad(cs, ((1, 0), (1, 0), (0, 0)))
    w = win
    out = cs[w:, w:] - cs[:-w, w:] - cs[w:, :-w] + cs[:-w, :-w]
    return out.astype(np.int32)


# ----------------------------------------------------------------------------------------
# 3-way dynamic programming (left->right, right->left, top->bottom)
# ----------------------------------------------------------------------------------------
def _step(prev: np.ndarray, C: np.ndarray, P1: int, P2: int) -> np.ndarray:
    """One SGBM path step over the last axis (disparity): OpenCV's form
    L = C + min(prev[d], prev[d-1] + P1, prev[d+1] + P1, minprev + P2) - (minprev + P2)."""
    mn = prev.min(-1, keepdims=True)
    big = np.iinfo(np.int32).max // 4
    lo = np.concatenate([np.full(prev.shape[:-1] + (1,), big, np.int64), prev[..., :-1]], -1)
    hi = np.concatenate([prev[..., 1:], np.full(prev.shape[:-1] + (1,), big, np.int64)], -1)
    m = np.minimum(np.minimum(prev, np.minimum(lo, hi) + P1), mn + P2)
    return C + m - (mn + P2)


def aggregate(C: np.ndarray, P1: int, P2: int) -> np.ndarray:
    """S = L_left + L_right + L_top, int64 [H, Wb, D]."""
    H, Wb, D = C.shape
    C = C.astype(np.int64)
    S = np.zeros_like(C)
    prev = np.zeros((H, D), np.int64)
    for x in range(Wb):
        prev = _step(prev, C[:, x], P1, P2)
        S[:, x] += prev
    prev = np.zeros((H, D), np.int64)
    for x in range(Wb - 1, -1, -1):
        prev = _step(prev, C[:, x], P1, P2)
        S[:, x] += prev
    prev = np.zeros((Wb, D), np.int64)
    for y in range(H):
        prev = _step(prev, C[y], P1, P2)
        S[y] += prev
    return S


# ----------------------------------------------------------------------------------------
# winner-take-all, uniqueness, sub-pixel, left-right check
# ----------------------------------------------------------------------------------------
SHRT_MAX = 32767


def select(S: np.ndarray, W: int, min_disp: int, num_disp: int, uniqueness: int,
           disp12: int) -> np.ndarray:
    """int16 x16 disparity of the whole image from the aggregated costs of the band."""
    H, Wb, D = S.shape
    X0 = max(min_disp + D, 0)
    inv = (min_disp - 1) * 16
    out = np.full((H, W), inv, np.int32)
    if Wb == 0:
        return out.astype(np.int16)
    best = S.argmin(-1)                                   # first minimum
    minS = np.take_along_axis(S, best[..., None], -1)[..., 0]
    kk = np.arange(D)
    viol = (S * (100 - uniqueness) < minS[..., None] * 100) & (np.abs(kk - best[..., None]) > 1)
    unique = ~viol.any(-1)
    # sub-pixel (parabola through best-1, best, best+1)
    b = best
    inner = (b > 0) & (b < D - 1)
    sm = np.take_along_axis(S, np.clip(b - 1, 0, D - 1)[..., None], -1)[..., 0]
    sp = np.take_along_axis(S, np.clip(b + 1, 0, D - 1)[..., None], -1)[..., 0]
    denom2 = np.maximum(sm + sp - 2 * minS, 1)
    num = (sm - sp) * 16 + denom2
    q = np.trunc(num / (denom2 * 2)).astype(np.int64)    # C integer division
    d16 = np.where(inner, b * 16 + q, b * 16) + min_disp * 16
    for y in range(H):
        row = np.full(W, inv, np.int64)
        disp2 = np.full(W, min_disp - 1, np.int64)
        cost2 = np.full(W, SHRT_MAX, np.int64)
        for xb in range(Wb - 1, -1, -1):                  # OpenCV's backward pass order
            if not unique[y, xb]:
                continue
            x = xb + X0
            x2 = x - (int(best[y, xb]) + min_disp)
            if cost2[x2] > minS[y, xb]:
                cost2[x2] = minS[y, xb]
                disp2[x2] = int(best[y, xb]) + min_disp
            row[x] = d16[y, xb]
        if disp12 >= 0:
            for x in range(X0, X0 + Wb):
                d1 = int(row[x])
                if d1 == inv:
                    continue
                _d = d1 >> 4
                d_ = (d1 + 15) >> 4
                _x, x_ = x - _d, x - d_
                if (0 <= _x < W and disp2[_x] >= min_disp and abs(disp2[_x] - _d) > disp12 and
                        0 <= x_ < W and disp2[x_] >= min_disp and abs(disp2[x_] - d_) > disp12):
                    row[x] = inv
        out[y] = row
    return out.astype(np.int16)


def filter_speckles(img: np.ndarray, new_val: int, max_size: int, max_diff: int) -> np.ndarray:
    """cv::filterSpeckles: 4-connected regions of pixels != new_val whose neighbours differ
    by <= max_diff; regions of <= max_size pixels are set to new_val."""
    a = img.astype(np.int32)
    H, W = a.shape
    lab = np.zeros((H, W), np.int32)
    out = img.copy()
    cur = 0
    for y0 in range(H):
        for x0 in range(W):
            if lab[y0, x0] or a[y0, x0] == new_val:
                continue
            cur += 1
            lab[y0, x0] = cur
            comp = [(y0, x0)]
            dq = deque(comp)
            while dq:
                y, x = dq.popleft()
                v = a[y, x]
                for yy, xx in ((y - 1, x), (y + 1, x), (y, x - 1), (y, x + 1)):
                    if 0 <= yy < H and 0 <= xx < W and not lab[yy, xx] and a[yy, xx] != new_val \
                            and abs(int(a[yy, xx]) - int(v)) <= max_diff:
                        lab[yy, xx] = cur
                        comp.append((yy, xx))
                        dq.append((yy, xx))
            if len(comp) <= max_size:
                for y, x in comp:
                    out[y, x] = new_val
    return out


def sgbm(L, R, min_disp: int, num_disp: int, win: int, P1=None, P2=None, disp12MaxDiff=1,
         uniquenessRatio=10, speckleWindowSize=100, speckleRange=32, preFilterCap=63):
    """StereoSGBM(MODE_SGBM_3WAY).compute(L, R) -> int16 x16 disparity (engine semantics)."""
    p = params_for(win)
    P1 = p["P1"] if P1 is None else P1
    P2 = p["P2"] if P2 is None else P2
    cap = max(preFilterCap, 15) | 1                      # OpenCV's ftzero
    H, W = L.shape
    pc = pixel_cost(L, R, min_disp, num_disp, cap)
    C = block_cost(pc, win)
    S = aggregate(C, P1, max(P2, P1 + 1))
    d = select(S, W, min_disp, num_disp, uniquenessRatio, disp12MaxDiff)
    if speckleWindowSize > 0:
        d = filter_speckles(d, (min_disp - 1) * 16, speckleWindowSize, 16 * speckleRange)
    return d
