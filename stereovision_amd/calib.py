"""Calibration ingestion and stereo rectification geometry (host side, one-time setup).

The reference loads the stereo-calibration pickle and builds rectification maps once per
session (depth_map.py:591-668 ``load_stereo_calibration``, fused_depth_map.py:307-441
``load_stereo_calibration_with_scaling``) through three OpenCV calls:

* ``cv2.stereoRectify(K1, D1, K2, D2, size, R, T, alpha=0, flags=CALIB_ZERO_DISPARITY)``
  — restated here in NumPy (:func:`stereo_rectify`, Bouguet's algorithm as OpenCV 3.x/4.x
  implements it in calib3d ``cvStereoRectify``: half rotations, global Z rotation, common
  focal length = mean of the two fy, principal points from the undistorted corner
  centroid, alpha scaling from the inner/outer rectangles of a 9x9 undistorted grid);
* ``cv2.initUndistortRectifyMap(..., CV_16SC2)`` — runs on the GPU (``k_undistort_map``,
  ``sv_init_undistort_rectify_map``);
* ``cv2.remap(..., INTER_LINEAR)`` per frame — runs on the GPU (``k_remap``).

This is 3x3 geometry executed once per calibration, so it stays host NumPy like the
reference's own setup code; the per-pixel work is all HIP.  Parity with OpenCV is
unpinned (OpenCV is not importable here); tests/test_rectify.py checks the geometric
invariants instead (orthonormal rotations, row-aligned epipolar geometry, baseline along
x, Q reprojection, identity calibrations).

The calibration file is the reference's pickle (schema stereo_calibration.py:276-297).
It is read with a restricted unpickler that only reconstructs NumPy arrays and plain
Python containers — no other global can be instantiated from the file.  ``.npz`` and
``.json`` files with the same keys are accepted too.
"""
from __future__ import annotations

import io
import json
import math
import os
import pickle

import numpy as np

CALIB_ZERO_DISPARITY = 0x400          # cv2.CALIB_ZERO_DISPARITY
FLT_MAX = float(np.finfo(np.float32).max)


# ----------------------------------------------------------------------------------------
# Calibration file
# ----------------------------------------------------------------------------------------
class _NumpyOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
        ("builtins", "tuple"), ("builtins", "list"), ("builtins", "dict"),
        ("builtins", "float"), ("builtins", "int"), ("builtins", "complex"),
        ("_codecs", "encode"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"calibration file references {module}.{name}: only "
                                     "NumPy arrays and plain containers are accepted")


REQUIRED_KEYS = ("mtx_left", "dist_left", "mtx_right", "dist_right", "R", "T", "img_size")


def read_calibration(path: str) -> dict:
    """Read the stereo-calibration file (pickle / .npz / .json with the keys of
    stereo_calibration.py:276-297)."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npz":
        with np.load(path, allow_pickle=False) as z:
            data = {k: z[k] for k in z.files}
    elif ext == ".json":
        with open(path) as f:
            data = {k: np.asarray(v) if isinstance(v, list) else v for k, v in json.load(f).items()}
    else:
        with open(path, "rb") as f:
            data = _NumpyOnlyUnpickler(io.BytesIO(f.read())).load()
    missing = [k for k in REQUIRED_KEYS if k not in data]
    if missing:
        raise KeyError(f"calibration file {path} lacks {missing}")
    return data


# ----------------------------------------------------------------------------------------
# Rodrigues (calib3d cvRodrigues2)
# ----------------------------------------------------------------------------------------
def rodrigues_to_matrix(r) -> np.ndarray:
    r = np.asarray(r, np.float64).ravel()
    theta = math.sqrt(float(r @ r))
    if theta < np.finfo(np.float64).eps:
        return np.eye(3)
    c, s = math.cos(theta), math.sin(theta)
    c1 = 1.0 - c
    k = r / theta
    rrt = np.outer(k, k)
    rx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return c * np.eye(3) + c1 * rrt + s * rx


def rodrigues_to_vector(R) -> np.ndarray:
    R = np.asarray(R, np.float64).reshape(3, 3)
    u, _, vt = np.linalg.svd(R)
    R = u @ vt                                        # nearest rotation (as OpenCV does)
    rx = R[2, 1] - R[1, 2]
    ry = R[0, 2] - R[2, 0]
    rz = R[1, 0] - R[0, 1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5
    c = min(max(c, -1.0), 1.0)
    theta = math.acos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros(3)
        t = (R[0, 0] + 1) * 0.5
        rx = math.sqrt(max(t, 0.0))
        t = (R[1, 1] + 1) * 0.5
        ry = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 1] < 0 else 1.0)
        t = (R[2, 2] + 1) * 0.5
        rz = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 2] < 0 else 1.0)
        if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1, 2] > 0) != (ry * rz > 0):
            rz = -rz
        v = np.array([rx, ry, rz])
        return v * (theta / math.sqrt(float(v @ v)))
    vth = 1.0 / (2 * s) * theta
    return np.array([rx, ry, rz]) * vth


# ----------------------------------------------------------------------------------------
# undistortPoints / projectPoints (the pieces stereoRectify uses)
# ----------------------------------------------------------------------------------------
def _dist12(dist) -> np.ndarray:
    d = np.zeros(12, np.float64)
    if dist is not None:
        v = np.asarray(dist, np.float64).ravel()
        if v.size not in (0, 4, 5, 8, 12, 14):
            raise ValueError(f"distCoeffs must have 4, 5, 8, 12 or 14 elements, got {v.size}")
        if v.size == 14 and (v[12] != 0 or v[13] != 0):
            raise ValueError("tilted sensor model (tauX, tauY != 0) is not supported")
        d[:min(v.size, 12)] = v[:12]
    return d


def undistort_points(pts, K, dist, R=None, P=None, iters: int = 5) -> np.ndarray:
    """cv::undistortPoints with the default 5-iteration criterion; points as float32 in
    and out (the CV_32FC2 buffers stereoRectify uses)."""
    pts = np.asarray(pts, np.float32).reshape(-1, 2).astype(np.float64)
    K = np.asarray(K, np.float64).reshape(3, 3)
    k = _dist12(dist)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    ifx, ify = 1.0 / fx, 1.0 / fy
    u, v = pts[:, 0], pts[:, 1]
    x0 = (u - cx) * ifx
    y0 = (v - cy) * ify
    x, y = x0.copy(), y0.copy()
    if np.any(k != 0):
        live = np.ones(x.shape, bool)
        for _ in range(iters):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            neg = live & (icdist < 0)
            x = np.where(neg, x0, x)
            y = np.where(neg, y0, y)
            live &= ~neg
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
            x = np.where(live, (x0 - dx) * icdist, x)
            y = np.where(live, (y0 - dy) * icdist, y)
    RR = np.eye(3)
    if P is not None:
        RR = np.asarray(P, np.float64).reshape(3, -1)[:, :3].copy()
    if R is not None:
        RR = RR @ np.asarray(R, np.float64).reshape(3, 3)
    xx = RR[0, 0] * x + RR[0, 1] * y + RR[0, 2]
    yy = RR[1, 0] * x + RR[1, 1] * y + RR[1, 2]
    ww = 1.0 / (RR[2, 0] * x + RR[2, 1] * y + RR[2, 2])
    return np.stack([xx * ww, yy * ww], -1).astype(np.float32)


def _project_no_dist(pts3, R, f) -> np.ndarray:
    """cvProjectPoints2 with zero translation and distortion, K = diag(f, f, 1), c = 0."""
    X = np.asarray(pts3, np.float64) @ np.asarray(R, np.float64).T
    z = 1.0 / X[:, 2]
    return np.stack([f * X[:, 0] * z, f * X[:, 1] * z], -1).astype(np.float32)


def _get_rectangles(K, dist, R, P, size):
    """icvGetRectangles: inner/outer rectangles (float) of the undistorted 9x9 grid."""
    N = 9
    w, h = size
    gx, gy = np.meshgrid(np.arange(N, dtype=np.float32), np.arange(N, dtype=np.float32))
    pts = np.stack([gx.ravel() * np.float32(w) / np.float32(N - 1),
                    gy.ravel() * np.float32(h) / np.float32(N - 1)], -1).astype(np.float32)
    p = undistort_points(pts, K, dist, R, P).reshape(N, N, 2)
    ix0 = float(np.max(p[:, 0, 0]))
    ix1 = float(np.min(p[:, N - 1, 0]))
    iy0 = float(np.max(p[0, :, 1]))
    iy1 = float(np.min(p[N - 1, :, 1]))
    ox0, ox1 = float(p[..., 0].min()), float(p[..., 0].max())
    oy0, oy1 = float(p[..., 1].min()), float(p[..., 1].max())
    f32 = np.float32
    inner = tuple(float(f32(v)) for v in (ix0, iy0, f32(ix1) - f32(ix0), f32(iy1) - f32(iy0)))
    outer = tuple(float(f32(v)) for v in (ox0, oy0, f32(ox1) - f32(ox0), f32(oy1) - f32(oy0)))
    return inner, outer


def _rect_and(a, b):
    x0, y0 = max(a[0], b[0]), max(a[1], b[1])
    x1, y1 = min(a[0] + a[2], b[0] + b[2]), min(a[1] + a[3], b[1] + b[3])
    if x1 <= x0 or y1 <= y0:
        return (0, 0, 0, 0)
    return (x0, y0, x1 - x0, y1 - y0)


# ----------------------------------------------------------------------------------------
# stereoRectify (calib3d cvStereoRectify)
# ----------------------------------------------------------------------------------------
def stereo_rectify(K1, D1, K2, D2, image_size, R, T, flags: int = CALIB_ZERO_DISPARITY,
                   alpha: float = -1, new_image_size=(0, 0)):
    """-> (R1, R2, P1, P2, Q, roi1, roi2) as cv2.stereoRectify returns them.

    image_size / new_image_size are (width, height) as in OpenCV."""
    K1 = np.asarray(K1, np.float64).reshape(3, 3)
    K2 = np.asarray(K2, np.float64).reshape(3, 3)
    nx, ny = int(image_size[0]), int(image_size[1])
    Rm = np.asarray(R, np.float64)
    om = rodrigues_to_vector(Rm) if Rm.size == 9 else Rm.ravel().copy()
    om = om * -0.5                                    # average rotation
    r_r = rodrigues_to_matrix(om)
    t = r_r @ np.asarray(T, np.float64).ravel()
    idx = 0 if abs(t[0]) > abs(t[1]) else 1
    c = t[idx]
    nt = math.sqrt(float(t @ t))
    if not nt > 0.0:
        raise ValueError("stereoRectify: zero translation")
    uu = np.zeros(3)
    uu[idx] = 1.0 if c > 0 else -1.0
    ww = np.cross(t, uu)
    nw = math.sqrt(float(ww @ ww))
    if nw > 0.0:
        ww = ww * (math.acos(abs(c) / nt) / nw)
    wR = rodrigues_to_matrix(ww)
    R1 = wR @ r_r.T
    R2 = wR @ r_r
    t = R2 @ np.asarray(T, np.float64).ravel()

    nsz = (int(new_image_size[0]), int(new_image_size[1]))
    if nsz[0] * nsz[1] == 0:
        nsz = (nx, ny)
    ratio_x = nsz[0] / nx / 2
    ratio_y = nsz[1] / ny / 2
    ratio = ratio_x if idx == 1 else ratio_y
    fc_new = (K1[idx ^ 1, idx ^ 1] + K2[idx ^ 1, idx ^ 1]) * ratio

    cc_new = []
    for k in range(2):
        A, Dk, Rk = (K1, D1, R1) if k == 0 else (K2, D2, R2)
        pts = np.array([[0, 0], [nx - 1, 0], [0, ny - 1], [nx - 1, ny - 1]], np.float32)
        und = undistort_points(pts, A, Dk)
        p3 = np.concatenate([und.astype(np.float64), np.ones((4, 1))], 1).astype(np.float32)
        proj = _project_no_dist(p3, Rk, fc_new)
        avg = proj.astype(np.float64).mean(0)
        # (nx-1)/2 is an integer division in OpenCV
        cc_new.append([(nx - 1) // 2 - avg[0], (ny - 1) // 2 - avg[1]])
    cc_new = np.array(cc_new)
    if flags & CALIB_ZERO_DISPARITY:
        cc_new[:, 0] = (cc_new[0, 0] + cc_new[1, 0]) * 0.5
        cc_new[:, 1] = (cc_new[0, 1] + cc_new[1, 1]) * 0.5
    elif idx == 0:
        cc_new[:, 1] = (cc_new[0, 1] + cc_new[1, 1]) * 0.5
    else:
        cc_new[:, 0] = (cc_new[0, 0] + cc_new[1, 0]) * 0.5

    P1 = np.zeros((3, 4))
    P1[0, 0] = P1[1, 1] = fc_new
    P1[0, 2], P1[1, 2], P1[2, 2] = cc_new[0, 0], cc_new[0, 1], 1.0
    P2 = P1.copy()
    P2[0, 2], P2[1, 2] = cc_new[1, 0], cc_new[1, 1]
    P2[idx, 3] = t[idx] * fc_new

    alpha = min(alpha, 1.0)
    inner1, outer1 = _get_rectangles(K1, D1, R1, P1, (nx, ny))
    inner2, outer2 = _get_rectangles(K2, D2, R2, P2, (nx, ny))

    cx1_0, cy1_0 = cc_new[0]
    cx2_0, cy2_0 = cc_new[1]
    cx1 = nsz[0] * cx1_0 / nx
    cy1 = nsz[1] * cy1_0 / ny
    cx2 = nsz[0] * cx2_0 / nx
    cy2 = nsz[1] * cy2_0 / ny
    s = 1.0
    if alpha >= 0:
        def f32sum(a, b):      # Rect_<float> x + width is a float addition
            return float(np.float32(a) + np.float32(b))

        def s_in(cx, cy, cx0, cy0, r):
            return max(max(max(cx / (cx0 - r[0]), cy / (cy0 - r[1])),
                           (nsz[0] - 1 - cx) / (f32sum(r[0], r[2]) - cx0 - 1)),
                       (nsz[1] - 1 - cy) / (f32sum(r[1], r[3]) - cy0 - 1))

        def s_out(cx, cy, cx0, cy0, r):
            return min(min(min(cx / (cx0 - r[0]), cy / (cy0 - r[1])),
                           (nsz[0] - 1 - cx) / (f32sum(r[0], r[2]) - cx0 - 1)),
                       (nsz[1] - 1 - cy) / (f32sum(r[1], r[3]) - cy0 - 1))

        s0 = max(s_in(cx2, cy2, cx2_0, cy2_0, inner2), s_in(cx1, cy1, cx1_0, cy1_0, inner1))
        s1 = min(s_out(cx2, cy2, cx2_0, cy2_0, outer2), s_out(cx1, cy1, cx1_0, cy1_0, outer1))
        s = s0 * (1 - alpha) + s1 * alpha
    fc_new *= s
    P1[0, 0] = P1[1, 1] = fc_new
    P1[0, 2], P1[1, 2] = cx1, cy1
    P2[0, 0] = P2[1, 1] = fc_new
    P2[0, 2], P2[1, 2] = cx2, cy2
    P2[idx, 3] = s * P2[idx, 3]

    def roi(inner, cx0, cy0, cx, cy):
        r = (math.ceil((inner[0] - cx0) * s + cx), math.ceil((inner[1] - cy0) * s + cy),
             math.floor(inner[2] * s), math.floor(inner[3] * s))
        return _rect_and(r, (0, 0, nsz[0], nsz[1]))

    roi1 = roi(inner1, cx1_0, cy1_0, cx1, cy1)
    roi2 = roi(inner2, cx2_0, cy2_0, cx2, cy2)
    Q = np.array([[1, 0, 0, -cx1], [0, 1, 0, -cy1], [0, 0, 0, fc_new],
                  [0, 0, -1.0 / t[idx], ((cx1 - cx2) if idx == 0 else (cy1 - cy2)) / t[idx]]])
    return R1, R2, P1, P2, Q, roi1, roi2


def scale_camera_matrix(K, scale: float) -> np.ndarray:
    """fused_depth_map.py:366-377: fx, fy, cx, cy multiplied by the processing scale."""
    K = np.array(K, np.float64, copy=True)
    K[0, 0] *= scale
    K[1, 1] *= scale
    K[0, 2] *= scale
    K[1, 2] *= scale
    return K
