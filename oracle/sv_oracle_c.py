"""ctypes loader for oracle/build/libsv_oracle.so (the C restatement) — TEST INFRASTRUCTURE.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libsv_oracle.so")
_lib = None

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i = ctypes.c_int
_f = ctypes.c_float


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.svo_disparity16.argtypes = [_u8p, _u8p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i16p, _i, _i]
        L.svo_disparity16.restype = _i
        L.svo_median5_f32.argtypes = [_i16p, _i, _i, _f32p]
        L.svo_median5_f32.restype = None
        L.svo_depth_post.argtypes = [_f32p, _i, _f, _f, _f, _f, _f32p, _u8p]
        L.svo_depth_post.restype = None
        L.svo_scaled_post.argtypes = [_f32p, _i, _i, _i, _f32p, _u8p, _f32p]
        L.svo_scaled_post.restype = None
        L.svo_harris.argtypes = [_u8p, _i, _i, _i, _f32p]
        L.svo_harris.restype = None
        L.svo_hog_hist.argtypes = [_u8p, _i, _i, _i, _i, _u16p]
        L.svo_hog_hist.restype = None
        L.svo_gray.argtypes = [_u8p, _i, _i, _i, _u8p]
        L.svo_gray.restype = None
        L.svo_depth_map.argtypes = [_u8p, _u8p, _i, _i, _i, _i, _i, _i, _f, _f, _f, _f32p, _f32p,
                                    _u8p, _i]
        L.svo_depth_map.restype = _i
        L.svo_max_threads.argtypes = []
        L.svo_max_threads.restype = _i
        _lib = L
    return _lib


def disparity16(L, R, min_disp, num_disp, win, cost=0, rows=None, nthreads=0):
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    H, W = L.shape
    r0, r1 = (0, H) if rows is None else rows
    out = np.empty((H, W), np.int16)
    rc = lib().svo_disparity16(L, R, H, W, W, min_disp, num_disp, win, cost, r0, r1, out, W,
                               nthreads)
    if rc != 0:
        raise ValueError(f"svo_disparity16 failed: {rc}")
    return out


def median5_f32(d16):
    d16 = np.ascontiguousarray(d16, np.int16)
    out = np.empty(d16.shape, np.float32)
    lib().svo_median5_f32(d16, d16.shape[0], d16.shape[1], out)
    return out


def depth_post(disp, min_depth, max_depth, min_disp_global=0):
    disp = np.ascontiguousarray(disp, np.float32)
    df = np.empty_like(disp)
    nm = np.empty(disp.shape, np.uint8)
    lib().svo_depth_post(disp, disp.size, np.float32(min_depth), np.float32(max_depth),
                         np.float32(max_depth - min_depth), np.float32(min_disp_global), df, nm)
    return df, nm


def scaled_post(disp, min_disp, num_disp):
    disp = np.ascontiguousarray(disp, np.float32)
    dn = np.empty_like(disp)
    du = np.empty(disp.shape, np.uint8)
    cf = np.empty_like(disp)
    lib().svo_scaled_post(disp, disp.size, min_disp, num_disp, dn, du, cf)
    return dn, du, cf


def harris(gray):
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty(gray.shape, np.float32)
    lib().svo_harris(gray, gray.shape[0], gray.shape[1], gray.shape[1], out)
    return out


def hog_hist(gray, win):
    gray = np.ascontiguousarray(gray, np.uint8)
    H, W = gray.shape
    out = np.empty((9, H, W), np.uint16)
    lib().svo_hog_hist(gray, H, W, W, win, out)
    return out


def gray(bgr):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    H, W = bgr.shape[:2]
    out = np.empty((H, W), np.uint8)
    lib().svo_gray(bgr, H, W, W * 3, out)
    return out


def depth_map(L, R, min_disp, num_disp, win, cost=0, min_depth=0.3, max_depth=2.0, nthreads=0):
    """The whole app-1 path of one gray pair (svo_depth_map): (depth_final, disparity,
    depth_normalized) with create_depth_map's float32 casts (depth_map.py:909-936)."""
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    H, W = L.shape
    depth = np.empty((H, W), np.float32)
    disp = np.empty((H, W), np.float32)
    norm = np.empty((H, W), np.uint8)
    rc = lib().svo_depth_map(L, R, H, W, min_disp, num_disp, win, cost, np.float32(min_depth),
                             np.float32(max_depth), np.float32(float(max_depth) - float(min_depth)),
                             depth, disp, norm, nthreads)
    if rc != 0:
        raise ValueError(f"svo_depth_map failed: {rc}")
    return depth, disp, norm


def max_threads() -> int:
    return lib().svo_max_threads()
