"""Drop-in for the reference's ``depth_map.py`` disparity path.

``create_depth_map(left_img, right_img, stereo_calib=None, min_depth=0.3, max_depth=2.0)``
keeps the reference's name, arguments, module globals and return tuple
(depth_map.py:837-946):

    returns (depth_final float32 HxW, disparity float32 HxW, depth_colormap uint8 HxWx3)

and its never-raise convention for per-frame failures (print, then zero arrays,
depth_map.py:941-946).  Importing the module warms the engine up on a background thread
(:func:`warmup`; ``SV_WARMUP_AT_IMPORT=0`` disables it).  The numeric body — BGR->gray, the disparity engine (which
replaces cv2.StereoSGBM), medianBlur(5), depth = 56/(d+1e-6), clip, mask and
u8 normalisation — runs in one pass of the gfx950 kernels (include/stereovision_amd.h,
``sv_depth_map``).  A missing HIP library or GPU is NOT a per-frame failure: it raises
:class:`stereovision_amd.engine.EngineUnavailable` before any compute (no CPU fallback).
"""
from __future__ import annotations

import os

import numpy as np

from . import colormap
from . import rectify as _rectify
from .engine import get_engine, start_warmup
from .preamble import ensure_same_size as _ensure_same_size
from .preamble import resize_linear as _resize_linear
from .preamble import to_engine_image

STEREO_CALIBRATION_FILE = "output/stereo_calibration_data.pkl"   # depth_map.py:22

# Matching parameters — module globals read at call time, as in depth_map.py:31-33.
MIN_DISP = 16 * 0
NUM_DISP = 16 * 20
WINDOW_SIZE = 7
# Cost function of the north_star engine that replaces StereoSGBM: "sad" | "ssd" | "hog".
COST = "sad"


def ensure_same_size(left_img, right_img):
    """depth_map.py:39-71."""
    return _ensure_same_size(left_img, right_img, verbose=True)


def load_stereo_calibration(path=None):
    """depth_map.py:591-668: calibration file -> stereoRectify(alpha=0) -> CV_16SC2 maps
    (computed on the GPU; the dict also carries the maps resident in HBM)."""
    return _rectify.load_stereo_calibration(path or STEREO_CALIBRATION_FILE)


def resize_to_target(frame, target_size):
    """depth_map.py:757-776 (cv2.resize INTER_LINEAR on the GPU)."""
    if frame.shape[1] == target_size[0] and frame.shape[0] == target_size[1]:
        return frame
    return _resize_linear(frame, target_size[0], target_size[1])


def apply_stereo_rectification(left_img, right_img, stereo_calib):
    """depth_map.py:779-834: resize to the calibration size, both INTER_LINEAR remaps."""
    return _rectify.apply_stereo_rectification(left_img, right_img, stereo_calib)


def _gray_pair(engine, left_img, right_img):
    gl = to_engine_image(left_img)
    gr = to_engine_image(right_img)
    if gl.ndim != gr.ndim:   # one BGR, one gray: convert the BGR one on the GPU
        gl = engine.gray(gl) if gl.ndim == 3 else gl
        gr = engine.gray(gr) if gr.ndim == 3 else gr
    return gl, gr


def create_depth_map(left_img, right_img, stereo_calib=None, min_depth=0.3, max_depth=2.0):
    """depth_map.py:837-946 on the MI355X engine.

    ``stereo_calib`` is accepted for signature compatibility; as in the reference it does
    not change the result (its 'calibration_data' key is never produced, so fx = 700,
    depth_map.py:915-920).
    """
    left_img, right_img = ensure_same_size(left_img, right_img)
    engine = get_engine()          # raises loudly when the HIP path is unavailable
    h, w = np.asarray(left_img).shape[:2]
    try:
        gl, gr = _gray_pair(engine, left_img, right_img)
        if gl.shape[:2] != gr.shape[:2]:
            print(f"ERROR: shapes differ after conversion: {gl.shape} vs {gr.shape}")
            gl, gr = _ensure_same_size(gl, gr)
            h, w = gl.shape[:2]
        # applyColorMap(depth_normalized, TURBO) (:937) runs in the same GPU epilogue
        depth_final, disparity, depth_colormap = engine.depth_map_color(
            gl, gr, MIN_DISP, NUM_DISP, WINDOW_SIZE, float(min_depth), float(max_depth),
            colormap.table("turbo"), min_disp_global=MIN_DISP, cost=COST)
        return depth_final, disparity, depth_colormap
    except Exception as e:  # the reference's per-frame error convention (:941-946)
        print(f"Error creating depth map: {e}")
        empty_uint8 = np.zeros((h, w), dtype=np.uint8)
        empty_colormap = colormap.apply(empty_uint8, "turbo")
        return np.zeros((h, w), dtype=np.float32), np.zeros((h, w), dtype=np.float32), empty_colormap


def warmup(height: int = 480, width: int = 640) -> None:
    """Create the engine and run create_depth_map's device path once with the module
    globals (BGR frames of the given size), so the first captured frame does not pay HIP
    initialisation, code-object loading and staging allocation."""
    z = np.zeros((height, width, 3), np.uint8)
    get_engine().depth_map_color(z, z, MIN_DISP, NUM_DISP, WINDOW_SIZE, 0.3, 2.0,
                                 colormap.table("turbo"), min_disp_global=MIN_DISP, cost=COST)


warmup_done = None
if os.environ.get("SV_WARMUP_AT_IMPORT", "1") != "0":
    warmup_done = start_warmup(warmup, "sv-warmup-depth-map")
