"""CPU oracle for the rectification stage in front of the disparity path — TEST
INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path (``stereovision_amd``)
never imports it.

What it restates
-------------------------------------------
The reference rectifies every captured pair before the disparity call:

* ``cv2.initUndistortRectifyMap(K, dist, R, P, size, cv2.CV_16SC2)``
  (depth_map.py:636-641, fused_depth_map.py:402-407) — per output pixel, the inverse of
  (P[:, :3] @ R) maps the pixel to a normalised ray, the Brown-Conrady distortion model
  (k1..k6 rational radial, p1 p2 tangential, s1..s4 thin prism) maps it to the raw image,
  and the raw position is stored as 1/32-pixel fixed point: map1 = (x >> 5, y >> 5) int16
  pairs, map2 = (y & 31) * 32 + (x & 31) uint16.  Rounding: cvRound (half to even).
* ``cv2.remap(img, map1, map2, cv2.INTER_LINEAR)`` (depth_map.py:815-826,
  fused_depth_map.py:480-491) — bilinear interpolation with OpenCV's fixed-point weight
  table (INTER_BITS = 5, INTER_REMAP_COEF_BITS = 15), default border BORDER_CONSTANT with
  value 0 applied per tap.

OpenCV (third-party, version unpinned, not importable in this image) is the reference's
implementation; this module follows its published algorithm (imgproc/undistort,
imgproc/imgwarp: initInterTab2D, remapBilinear).  Two build-dependent details are fixed
here and documented in DESIGN.md:
  - OpenCV accumulates the per-row ray incrementally (``_x += ir[0]``; its SIMD lanes use
    vector offsets), so its maps depend on the SIMD width it was built for.  This oracle
    (and the GPU kernel) evaluates ``(i*ir[1] + ir[2]) + j*ir[0]`` per pixel: a map entry
    can differ from a given OpenCV build only where u*32 lies within ~1e-9 of a rounding
    boundary.
  - The u8 bilinear weights: OpenCV's table holds 32*w' with w' = (32-fy)(32-fx),
    (32-fy)fx, fy(32-fx), fy*fx, except that the (0, 0) entry saturates 32768 to 32767;
    for u8 data every variant of that entry yields the same byte, so the result is
    ``(sum(w' * v) + 512) >> 10`` exactly (checked exhaustively by tests/test_rectify.py).

PARITY STATUS: **parity unpinned** against OpenCV itself (absent here, no golden vectors
in the reference).  Pinned by analytic known-answer tests: identity calibrations give
identity maps, integer maps make remap a gather, the fixed-point bilinear equals the
exact rational bilinear rounded half-up, and maps agree with an independent forward
projection of the distortion model.
"""
from __future__ import annotations

import numpy as np

INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS
INTER_REMAP_COEF_BITS = 15
INTER_REMAP_COEF_SCALE = 1 << INTER_REMAP_COEF_BITS


# ----------------------------------------------------------------------------------------
# 3x3 helpers with OpenCV's operation order (Matx33d product and cofactor inverse)
# ----------------------------------------------------------------------------------------
def matmul33(a, b):
    """Matx33d * Matx33d: c(i,j) = a(i,0)b(0,j) + a(i,1)b(1,j) + a(i,2)b(2,j), left to
    right in double."""
    a = [[float(v) for v in r] for r in np.asarray(a, np.float64).reshape(3, 3)]
    b = [[float(v) for v in r] for r in np.asarray(b, np.float64).reshape(3, 3)]
    return [[(a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j] for j in range(3)]
            for i in range(3)]


def inv33(a):
    """Matx_FastInvOp<double, 3> (cofactors times 1/det, det by the first-row expansion)."""
    a = [[float(v) for v in r] for r in np.asarray(a, np.float64).reshape(3, 3)]
    det = (a[0][0] * (a[1][1] * a[2][2] - a[2][1] * a[1][2])
           - a[0][1] * (a[1][0] * a[2][2] - a[2][0] * a[1][2])
           + a[0][2] * (a[1][0] * a[2][1] - a[2][0] * a[1][1]))
    if det == 0.0:
        raise ZeroDivisionError("singular newCameraMatrix * R")
    d = 1.0 / det
    return [
        [(a[1][1] * a[2][2] - a[1][2] * a[2][1]) * d, (a[0][2] * a[2][1] - a[0][1] * a[2][2]) * d,
         (a[0][1] * a[1][2] - a[0][2] * a[1][1]) * d],
        [(a[1][2] * a[2][0] - a[1][0] * a[2][2]) * d, (a[0][0] * a[2][2] - a[0][2] * a[2][0]) * d,
         (a[0][2] * a[1][0] - a[0][0] * a[1][2]) * d],
        [(a[1][0] * a[2][1] - a[1][1] * a[2][0]) * d, (a[0][1] * a[2][0] - a[0][0] * a[2][1]) * d,
         (a[0][0] * a[1][1] - a[0][1] * a[1][0]) * d],
    ]


def dist12(dist) -> np.ndarray:
    """distCoeffs (4, 5, 8 or 12 values) -> k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4."""
    d = np.zeros(12, np.float64)
    if dist is not None:
        v = np.asarray(dist, np.float64).ravel()
        if v.size not in (0, 4, 5, 8, 12, 14):
            raise ValueError(f"distCoeffs must have 4, 5, 8, 12 or 14 elements, got {v.size}")
        if v.size == 14 and (v[12] != 0 or v[13] != 0):
            raise ValueError("tilted sensor model (tauX, tauY != 0) is not supported")
        d[:min(v.size, 12)] = v[:12]
    return d


def _cv_round_i32(v: np.ndarray) -> np.ndarray:
    """saturate_cast<int>(double) on x86 (cvRound): round half to even; NaN and values
    outside int32 give INT_MIN (the cvtsd2si 'integer indefinite' value)."""
    out = np.full(v.shape, np.iinfo(np.int32).min, np.int64)
    ok = np.isfinite(v) & (v > -2147483648.5) & (v < 2147483647.5)
    out[ok] = np.rint(v[ok]).astype(np.int64)
    return out


# ----------------------------------------------------------------------------------------
# initUndistortRectifyMap(..., CV_16SC2)   depth_map.py:636-641, fused_depth_map.py:402-407
# ----------------------------------------------------------------------------------------
def undistort_rectify_map(K, dist, R, P, width: int, height: int):
    """-> (map1 int16 [H, W, 2], map2 uint16 [H, W]); also returns the f64 (u, v)."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    Rm = np.eye(3) if R is None else np.asarray(R, np.float64).reshape(3, 3)
    Pm = K if P is None else np.asarray(P, np.float64)
    Ar = Pm.reshape(3, -1)[:, :3]
    ir = np.array(inv33(matmul33(Ar, Rm)), np.float64).ravel()
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = dist12(dist)
    fx, fy, u0, v0 = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    i = np.arange(height, dtype=np.float64)[:, None]
    j = np.arange(width, dtype=np.float64)[None, :]
    _x = (i * ir[1] + ir[2]) + j * ir[0]
    _y = (i * ir[4] + ir[5]) + j * ir[3]
    _w = (i * ir[7] + ir[8]) + j * ir[6]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        w = 1.0 / _w
        x = _x * w
        y = _y * w
        x2 = x * x
        y2 = y * y
        r2 = x2 + y2
        _2xy = 2 * x * y
        kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
        xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2
        yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2
        u = fx * xd + u0
        v = fy * yd + v0
        iu = _cv_round_i32(u * INTER_TAB_SIZE)
        iv = _cv_round_i32(v * INTER_TAB_SIZE)
    map1 = np.empty((height, width, 2), np.int16)
    map1[..., 0] = (iu >> INTER_BITS).astype(np.int16)   # (short) truncation
    map1[..., 1] = (iv >> INTER_BITS).astype(np.int16)
    map2 = ((iv & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE + (iu & (INTER_TAB_SIZE - 1))).astype(np.uint16)
    return map1, map2, u, v


# ----------------------------------------------------------------------------------------
# remap(INTER_LINEAR, BORDER_CONSTANT 0)   depth_map.py:815-826, fused_depth_map.py:480-491
# ----------------------------------------------------------------------------------------
def bilinear_tab_i() -> np.ndarray:
    """OpenCV's BilinearTab_i: [1024, 4] int16-range weights scaled by 2^15 (initInterTab2D
    with fixpt; the (0, 0) entry saturates 32768 -> 32767)."""
    t = np.zeros((INTER_TAB_SIZE * INTER_TAB_SIZE, 4), np.int64)
    for fy in range(INTER_TAB_SIZE):
        for fx in range(INTER_TAB_SIZE):
            ay = (1.0 - fy / 32.0, fy / 32.0)
            ax = (1.0 - fx / 32.0, fx / 32.0)
            vals = [ay[k1] * ax[k2] * INTER_REMAP_COEF_SCALE for k1 in range(2) for k2 in range(2)]
            t[fy * 32 + fx] = [min(32767, int(np.rint(v))) for v in vals]
    return t


def remap_linear(src: np.ndarray, map1: np.ndarray, map2: np.ndarray,
                 table: str = "opencv") -> np.ndarray:
    """cv2.remap(src, map1, map2, INTER_LINEAR) for uint8 HxW or HxWxC source; output
    has the maps' shape.  Out-of-image taps read 0 (BORDER_CONSTANT, value 0).

    table="opencv": OpenCV's 2^15 weight table and (sum + 2^14) >> 15;
    table="exact":  the 10-bit form (sum(w' v) + 512) >> 10 the GPU kernel uses."""
    src = np.asarray(src)
    if src.dtype != np.uint8:
        raise TypeError("remap oracle: uint8 source only")
    s = src if src.ndim == 3 else src[..., None]
    Hs, Ws, C = s.shape
    sx = map1[..., 0].astype(np.int64)
    sy = map1[..., 1].astype(np.int64)
    f = map2.astype(np.int64) & (INTER_TAB_SIZE * INTER_TAB_SIZE - 1)
    fx = f & 31
    fy = f >> 5
    if table == "opencv":
        w = bilinear_tab_i()[f]          # [H, W, 4]
        shift, delta = 15, 1 << 14
    else:
        w = np.stack([(32 - fy) * (32 - fx), (32 - fy) * fx, fy * (32 - fx), fy * fx], -1)
        shift, delta = 10, 1 << 9
    acc = np.zeros(sx.shape + (C,), np.int64)
    for k, (dy, dx) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        yy = sy + dy
        xx = sx + dx
        inside = (yy >= 0) & (yy < Hs) & (xx >= 0) & (xx < Ws)
        v = np.zeros(sx.shape + (C,), np.int64)
        v[inside] = s[yy[inside], xx[inside]]
        acc += v * w[..., k:k + 1]
    out = np.clip((acc + delta) >> shift, 0, 255).astype(np.uint8)
    return out if src.ndim == 3 else out[..., 0]


def remap_gray(src_bgr: np.ndarray, map1, map2) -> np.ndarray:
    """cvtColor(remap(BGR), BGR2GRAY): the fused rectify+gray stage."""
    r = remap_linear(src_bgr, map1, map2).astype(np.int64)
    return ((r[..., 0] * 1868 + r[..., 1] * 9617 + r[..., 2] * 4899 + (1 << 13)) >> 14).astype(np.uint8)


# ----------------------------------------------------------------------------------------
# resize(INTER_LINEAR)   fused_depth_map.py:474-476, :2498-2507; depth_map.py:757-776
# ----------------------------------------------------------------------------------------
def _resize_coords(dn: int, sn: int, scale: float, clamp_frac: bool):
    d = np.arange(dn, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp_frac:
        lo = s < 0
        f[lo] = 0
        s[lo] = 0
        hi = s >= sn - 1
        f[hi] = 0
        s[hi] = sn - 1
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return np.clip(s, 0, sn - 1), np.clip(s + 1, 0, sn - 1), a0, a1


def resize_linear(src: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(src, (width, height), interpolation=INTER_LINEAR) for uint8: OpenCV's
    resizeGeneric_ with HResizeLinear (2^11 coefficients from the f32 source coordinate,
    columns clamped with a zero fraction) and VResizeLinear's scalar FixedPtCast<int, uchar,
    22> rounding; rows clamped.  An exact 2x downscale is OpenCV's INTER_AREA fast path.
    OpenCV's SSE/AVX vertical pass (mulhi of values >> 4) can differ by 1 on some pixels:
    parity unpinned."""
    src = np.asarray(src)
    s = src if src.ndim == 3 else src[..., None]
    sH, sW, C = s.shape
    if (sH, sW) == (height, width):
        return src.copy()
    scale_x = 1.0 / (width / sW)
    scale_y = 1.0 / (height / sH)
    if scale_x == 2.0 and scale_y == 2.0:
        a = s.astype(np.int64)
        out = (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
        out = out[:height, :width].astype(np.uint8)
        return out if src.ndim == 3 else out[..., 0]
    x0, x1, ax0, ax1 = _resize_coords(width, sW, scale_x, True)
    y0, y1, by0, by1 = _resize_coords(height, sH, scale_y, False)
    a = s.astype(np.int64)
    h0 = a[y0][:, x0] * ax0[None, :, None] + a[y0][:, x1] * ax1[None, :, None]
    h1 = a[y1][:, x0] * ax0[None, :, None] + a[y1][:, x1] * ax1[None, :, None]
    v = (h0 * by0[:, None, None] + h1 * by1[:, None, None] + (1 << 21)) >> 22
    out = np.clip(v, 0, 255).astype(np.uint8)
    return out if src.ndim == 3 else out[..., 0]


# ----------------------------------------------------------------------------------------
# Independent forward model (for known-answer tests of the maps)
# ----------------------------------------------------------------------------------------
def distort_normalised(x, y, dist):
    """Brown-Conrady forward distortion of normalised coordinates (projectPoints)."""
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = dist12(dist)
    r2 = x * x + y * y
    kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x) + s1 * r2 + s2 * r2 * r2
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y + s3 * r2 + s4 * r2 * r2
    return xd, yd
