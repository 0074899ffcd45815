"""Stereo rectification on the MI355X: the step in front of the disparity path.

Drop-ins for the reference's rectification helpers:

  load_stereo_calibration()                    depth_map.py:591-668
  load_stereo_calibration_with_scaling(scale)  fused_depth_map.py:307-441
  apply_stereo_rectification(l, r, calib)      depth_map.py:779-834, fused_depth_map.py:444-500
  init_undistort_rectify_map(K, D, R, P, size, m1type)   cv2.initUndistortRectifyMap
  remap(src, map1, map2, interpolation)                  cv2.remap (INTER_LINEAR)

Geometry (stereoRectify) is host NumPy (:mod:`stereovision_amd.calib`); the per-pixel maps
and every remap run in the gfx950 kernels of ``sv_rectify.hip``.  The calibration dict
keeps the reference's keys (host NumPy maps included) and additionally carries a
:class:`StereoRectifier` holding the four maps in HBM under ``"sv_rectifier"``, so
rectifying a frame pair uploads only the frames.  Errors follow the reference: the
loaders print and return None, apply_stereo_rectification prints and returns its inputs.
"""
from __future__ import annotations

import os
import traceback

import numpy as np

from . import calib as _calib
from .engine import Engine, get_engine
from .preamble import resize_linear

STEREO_CALIBRATION_FILE = "output/stereo_calibration_data.pkl"   # depth_map.py:22
CV_16SC2 = 11                                                    # cv2.CV_16SC2
INTER_LINEAR = 1                                                 # cv2.INTER_LINEAR


class StereoRectifier:
    """The left/right CV_16SC2 maps of one calibration, resident in device memory."""

    def __init__(self, engine: Engine, height: int, width: int):
        self.engine = engine
        self.H, self.W = int(height), int(width)
        n = self.H * self.W
        self._bufs = [engine.dev_alloc(4 * n), engine.dev_alloc(2 * n),
                      engine.dev_alloc(4 * n), engine.dev_alloc(2 * n)]
        self.host_ids = None      # ids of the host maps these were uploaded from

    @classmethod
    def from_maps(cls, left_map1, left_map2, right_map1, right_map2, engine: Engine = None):
        eng = engine or get_engine()
        H, W = np.asarray(left_map1).shape[:2]
        r = cls(eng, H, W)
        for buf, m, dt in zip(r._bufs, (left_map1, left_map2, right_map1, right_map2),
                              (np.int16, np.uint16, np.int16, np.uint16)):
            a = np.ascontiguousarray(m, dt)
            if a.shape[:2] != (H, W):
                raise ValueError(f"map shape {a.shape} does not match {(H, W)}")
            eng.to_device(buf, a)
        r.host_ids = tuple(id(m) for m in (left_map1, left_map2, right_map1, right_map2))
        return r

    @classmethod
    def from_calibration(cls, K1, D1, R1, P1, K2, D2, R2, P2, size, engine: Engine = None):
        """Both initUndistortRectifyMap calls, computed on the GPU into device memory."""
        eng = engine or get_engine()
        W, H = int(size[0]), int(size[1])
        r = cls(eng, H, W)
        eng.init_undistort_rectify_map_dev(K1, D1, R1, P1, W, H, r._bufs[0], r._bufs[1])
        eng.init_undistort_rectify_map_dev(K2, D2, R2, P2, W, H, r._bufs[2], r._bufs[3])
        eng.synchronize()
        return r

    @property
    def device_maps(self):
        return (*self._bufs, self.H, self.W)

    def host_maps(self):
        """-> (left_map1, left_map2, right_map1, right_map2) as NumPy arrays."""
        e = self.engine
        return (e.to_host(self._bufs[0], (self.H, self.W, 2), np.int16),
                e.to_host(self._bufs[1], (self.H, self.W), np.uint16),
                e.to_host(self._bufs[2], (self.H, self.W, 2), np.int16),
                e.to_host(self._bufs[3], (self.H, self.W), np.uint16))

    def rectify(self, left, right):
        """Both cv2.remap(..., INTER_LINEAR) calls of apply_stereo_rectification."""
        return self.engine.rectify_pair(self.device_maps, left, right)

    def close(self):
        for b in self._bufs or []:
            try:
                self.engine.dev_free(b)
            except Exception:
                pass
        self._bufs = []

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


# ----------------------------------------------------------------------------------------
# cv2-shaped helpers
# ----------------------------------------------------------------------------------------
def init_undistort_rectify_map(K, dist, R, P, size, m1type=CV_16SC2):
    """cv2.initUndistortRectifyMap(K, dist, R, P, (w, h), cv2.CV_16SC2) on the GPU."""
    if m1type != CV_16SC2:
        raise ValueError("only m1type=CV_16SC2 (the reference's map format) is supported")
    return get_engine().init_undistort_rectify_map(K, dist, R, P, int(size[0]), int(size[1]))


def remap(src, map1, map2, interpolation=INTER_LINEAR):
    """cv2.remap(src, map1, map2, cv2.INTER_LINEAR) (BORDER_CONSTANT 0) on the GPU."""
    if interpolation != INTER_LINEAR:
        raise ValueError("only INTER_LINEAR (the reference's interpolation) is supported")
    return get_engine().remap(src, map1, map2)


def _build(mtx_l, dist_l, mtx_r, dist_r, R, T, img_size, flags=_calib.CALIB_ZERO_DISPARITY):
    R1, R2, P1, P2, Q, roi1, roi2 = _calib.stereo_rectify(mtx_l, dist_l, mtx_r, dist_r, img_size, R,
                                                          T, flags=flags, alpha=0)
    rect = StereoRectifier.from_calibration(mtx_l, dist_l, R1, P1, mtx_r, dist_r, R2, P2, img_size)
    lm1, lm2, rm1, rm2 = rect.host_maps()
    rect.host_ids = (id(lm1), id(lm2), id(rm1), id(rm2))
    return {"left_map1": lm1, "left_map2": lm2, "right_map1": rm1, "right_map2": rm2,
            "roi1": roi1, "roi2": roi2, "Q": Q, "R1": R1, "R2": R2, "P1": P1, "P2": P2,
            "sv_rectifier": rect}


def load_stereo_calibration(path: str = None):
    """depth_map.py:591-668: read the calibration, stereoRectify(alpha=0), both maps."""
    path = path or STEREO_CALIBRATION_FILE
    if not os.path.exists(path):
        print(f"Error: stereo calibration file not found: {path}")
        return None
    try:
        d = _calib.read_calibration(path)
        T = np.asarray(d["T"], np.float64).reshape(3, 1)
        img_size = tuple(int(v) for v in np.asarray(d["img_size"]).ravel()[:2])
        out = _build(d["mtx_left"], d["dist_left"], d["mtx_right"], d["dist_right"], d["R"], T,
                     img_size)
        out.update({"R": d["R"], "T": T, "mtx_left": d["mtx_left"], "dist_left": d["dist_left"],
                    "mtx_right": d["mtx_right"], "dist_right": d["dist_right"],
                    "baseline": abs(T[0, 0]), "img_size": img_size})
        print(f"Stereo rectification ready. Baseline: {abs(T[0, 0]):.4f} m")
        return out
    except Exception as e:
        print(f"Error loading stereo calibration: {e}")
        traceback.print_exc()
        return None


def load_stereo_calibration_with_scaling(scale_factor: float = 1.0, path: str = None):
    """fused_depth_map.py:307-441: camera matrices scaled by the processing scale, maps at
    int(w * scale) x int(h * scale)."""
    path = path or STEREO_CALIBRATION_FILE
    if not os.path.exists(path):
        print(f"Error: stereo calibration file not found: {path}")
        return None
    try:
        d = _calib.read_calibration(path)
        T = np.asarray(d["T"], np.float64).reshape(3, 1)
        size0 = tuple(int(v) for v in np.asarray(d["img_size"]).ravel()[:2])
        Kl = _calib.scale_camera_matrix(d["mtx_left"], scale_factor)
        Kr = _calib.scale_camera_matrix(d["mtx_right"], scale_factor)
        size = (int(size0[0] * scale_factor), int(size0[1] * scale_factor))
        out = _build(Kl, d["dist_left"], Kr, d["dist_right"], d["R"], T, size)
        out.update({"R": d["R"], "T": T, "mtx_left": Kl, "dist_left": d["dist_left"],
                    "mtx_right": Kr, "dist_right": d["dist_right"], "baseline": abs(T[0, 0]),
                    "img_size_orig": size0, "img_size_proc": size, "focal_length": Kl[0, 0],
                    "scale_factor": scale_factor})
        print(f"Stereo rectification ready. Baseline: {abs(T[0, 0]):.4f} m, maps {size}")
        return out
    except Exception as e:
        print(f"Error loading stereo calibration: {e}")
        traceback.print_exc()
        return None


def _rectifier_for(calib: dict) -> StereoRectifier:
    keys = ("left_map1", "left_map2", "right_map1", "right_map2")
    ids = tuple(id(calib[k]) for k in keys)
    rect = calib.get("sv_rectifier")
    if rect is None or rect.host_ids != ids:
        rect = StereoRectifier.from_maps(*(calib[k] for k in keys))
        calib["sv_rectifier"] = rect      # cached with the calibration (maps live in HBM)
    return rect


def apply_stereo_rectification(left_img, right_img, stereo_calib):
    """depth_map.py:779-834 / fused_depth_map.py:444-500: resize to the calibration size
    if needed, then both INTER_LINEAR remaps (on the GPU, maps resident in HBM)."""
    if stereo_calib is None:
        return left_img, right_img
    try:
        if "img_size_proc" in stereo_calib:
            tw, th = stereo_calib["img_size_proc"]
        else:
            tw, th = stereo_calib["img_size"]
        if (left_img.shape[1], left_img.shape[0]) != (tw, th):
            left_img = resize_linear(left_img, tw, th)
        if (right_img.shape[1], right_img.shape[0]) != (tw, th):
            right_img = resize_linear(right_img, tw, th)
        return _rectifier_for(stereo_calib).rectify(left_img, right_img)
    except Exception as e:
        print(f"Stereo rectification error: {e}")
        traceback.print_exc()
        return left_img, right_img
