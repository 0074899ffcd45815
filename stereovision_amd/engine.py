"""ctypes binding of libsvhip.so (include/stereovision_amd.h).

The product path: NumPy arrays in, NumPy arrays out, all arithmetic in the gfx950 HIP
kernels.  There is no CPU fallback — if the library or a GPU is missing,
:func:`get_engine` raises :class:`EngineUnavailable` loudly.

ctypes releases the GIL for the duration of every foreign call, so an Engine can be
driven from the reference's ThreadPoolExecutor workers (fused_depth_map.py:2591-2598)
while the main thread keeps working.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SV_LIB_PATH", os.path.join(_HERE, "lib", "libsvhip.so"))

COSTS = {"sad": 0, "ssd": 1, "hog": 2, "sgbm": 3}
POST_NONE, POST_DEPTH, POST_SCALED = 0, 1, 2
KERNELS = {"gray": 0, "harris": 1, "hog": 2, "match": 3, "median": 4, "post": 5, "remap": 6,
           "undistort": 7, "resize": 8, "stats": 9, "select": 10, "affine": 11, "sgbm": 12,
           "speckle": 13, "gather": 14, "scatter": 15, "h2d": 16, "d2h": 17}

# Every symbol include/stereovision_amd.h declares (checked by tests/test_capi.py).
EXPORTED = [
    "sv_version", "sv_last_error", "sv_device_count", "sv_create", "sv_destroy",
    "sv_synchronize", "sv_stream", "sv_plan", "sv_gray", "sv_disparity", "sv_median5_f32",
    "sv_depth_post", "sv_scaled_post", "sv_depth_map", "sv_stereo_scaled", "sv_harris",
    "sv_hog_hist", "sv_gray_dev", "sv_disparity_dev", "sv_median_rows_dev", "sv_harris_dev",
    "sv_hog_hist_dev", "sv_profile_enable", "sv_profile_read", "sv_profile_reset",
    "sv_disparity_rows", "sv_dev_alloc", "sv_dev_free", "sv_copy_to_device", "sv_copy_to_host",
    "sv_host_register", "sv_host_unregister", "sv_host_profile_enable", "sv_host_profile_read",
    "sv_timer_begin", "sv_timer_end", "sv_disparity_batch_dev", "sv_depth_map_batch_dev",
    "sv_init_undistort_rectify_map", "sv_init_undistort_rectify_map_dev", "sv_remap", "sv_remap_dev",
    "sv_rectify_pair", "sv_resize_linear", "sv_resize_linear_dev", "sv_resize_linear_f32_dev",
    "sv_frame_stats", "sv_affine_f32_dev", "sv_sgbm", "sv_sgbm_dev", "sv_filter_speckles",
    "sv_filter_speckles_dev", "sv_multi_gpu_batch", "sv_harris_batch_dev", "sv_comm_available",
    "sv_comm_unique_id", "sv_comm_init_rank", "sv_comm_init_all", "sv_comm_destroy", "sv_comm_rank",
    "sv_comm_barrier", "sv_comm_allreduce_max_f64", "sv_comm_gatherv", "sv_comm_synchronize",
    "sv_multi_gpu_dev", "sv_depth_map_color", "sv_stereo_scaled_color", "sv_profile_region_begin",
    "sv_profile_region_end", "sv_comm_scatterv", "sv_band_rows_in", "sv_release_scratch",
    "sv_frame_stats_batch_dev", "sv_select_count_batch", "sv_select_ranks_batch", "sv_event_record",
    "sv_stream_wait_event", "sv_post_m16_dev",
]
BAND_MARGIN = 8   # SV_BAND_MARGIN: spare rows around a band-only input buffer
COMM_ID_BYTES = 128


class SVError(RuntimeError):
    """A libsvhip call returned a nonzero status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


class EngineUnavailable(SVError):
    """libsvhip.so is missing or no HIP device is visible: the HIP path cannot run."""

    def __init__(self, msg: str):
        RuntimeError.__init__(self, msg)
        self.code = -19


_c_int = ctypes.c_int
_c_float = ctypes.c_float
_vp = ctypes.c_void_p
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")


class _NullableF64:
    """ndpointer that also accepts None (optional matrices)."""

    @classmethod
    def from_param(cls, obj):
        if obj is None:
            return None
        return _f64p.from_param(obj)


class _NullableU16:
    @classmethod
    def from_param(cls, obj):
        if obj is None:
            return None
        return _u16p.from_param(obj)


class _NullableU8:
    @classmethod
    def from_param(cls, obj):
        if obj is None:
            return None
        return _u8p.from_param(obj)


class _NullableF32:
    """ndpointer that also accepts None (for optional outputs)."""

    @classmethod
    def from_param(cls, obj):
        if obj is None:
            return None
        return _f32p.from_param(obj)


STAGE_MATCH, STAGE_MEDIAN, STAGE_ALL = 1, 2, 3          # SV_STAGE_*
SHARD_FRAMES, SHARD_ROWS = 0, 1                         # SV_SHARD_*
INPUTS_RESIDENT, INPUTS_SCATTER, INPUTS_HOST = 0, 1, 2  # SV_INPUTS_*


class MapOut(ctypes.Structure):
    """sv_map_out: the outputs of one median + post launch (every pointer optional)."""
    _fields_ = [("mode", _c_int), ("min_depth", _c_float), ("max_depth", _c_float),
                ("depth_range", _c_float), ("min_disp_global", _c_float), ("disparity", _vp),
                ("out_a", _vp), ("out_u8", _vp), ("out_b", _vp), ("med16", _vp), ("d8", _vp),
                ("cmap_bgr", _vp), ("bgr", _vp), ("harris", _vp)]


def map_out(mode: int = POST_NONE, disparity: int = 0, out_a: int = 0, out_u8: int = 0, out_b: int = 0,
            med16: int = 0, d8: int = 0, harris: int = 0, bgr: int = 0, cmap=None, min_depth=0.0,
            max_depth=0.0, min_disp_global=0.0) -> MapOut:
    """An sv_map_out (depth_range = float32 of max_depth - min_depth computed in double, the
    NumPy-2 semantics of depth_map.py:936).  ``cmap``: a 256 x 3 uint8 BGR table (kept alive on
    the returned structure)."""
    m = MapOut(int(mode), np.float32(min_depth), np.float32(max_depth),
               np.float32(float(max_depth) - float(min_depth)), np.float32(min_disp_global),
               disparity or None, out_a or None, out_u8 or None, out_b or None, med16 or None, d8 or None,
               None, bgr or None, harris or None)
    if cmap is not None:
        m._cmap = np.ascontiguousarray(cmap, np.uint8).reshape(256, 3)
        m.cmap_bgr = m._cmap.ctypes.data
    return m


_lib = None
_lib_lock = threading.Lock()


def _declare(lib):
    sig = {
        "sv_version": ([], _c_int),
        "sv_last_error": ([], ctypes.c_char_p),
        "sv_device_count": ([ctypes.POINTER(_c_int)], _c_int),
        "sv_create": ([_c_int, ctypes.POINTER(_vp)], _c_int),
        "sv_destroy": ([_vp], None),
        "sv_synchronize": ([_vp], _c_int),
        "sv_release_scratch": ([_vp], _c_int),
        "sv_event_record": ([_vp, _c_int, _vp], _c_int),
        "sv_stream_wait_event": ([_vp, _c_int, _vp], _c_int),
        "sv_stream": ([_vp], _vp),
        "sv_plan": ([_c_int, _c_int, _c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int),
                     ctypes.POINTER(_c_int)], _c_int),
        "sv_gray": ([_vp, _u8p, _c_int, _c_int, _c_int, _u8p], _c_int),
        "sv_disparity": ([_vp, _u8p, _u8p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                          _c_int, _c_int, _i16p, _NullableF32], _c_int),
        "sv_median5_f32": ([_vp, _f32p, _c_int, _c_int, _f32p], _c_int),
        "sv_depth_post": ([_vp, _f32p, _c_int, _c_float, _c_float, _c_float, _c_float, _f32p,
                           _u8p], _c_int),
        "sv_scaled_post": ([_vp, _f32p, _c_int, _c_int, _c_int, _f32p, _u8p, _f32p], _c_int),
        "sv_depth_map": ([_vp, _u8p, _u8p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                          _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _f32p, _f32p,
                          _u8p], _c_int),
        "sv_harris_batch_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.c_int64, _vp,
                                 _vp], _c_int),
        "sv_multi_gpu_batch": ([ctypes.POINTER(_vp), _c_int, _u8p, _u8p, _c_int, _c_int, _c_int,
                                _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float,
                                _c_float, _c_float, _f32p, _f32p, _u8p], _c_int),
        "sv_stereo_scaled": ([_vp, _u8p, _u8p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                              _c_int, _c_int, _f32p, _f32p, _u8p, _f32p], _c_int),
        "sv_harris": ([_vp, _u8p, _c_int, _c_int, _c_int, _f32p], _c_int),
        "sv_hog_hist": ([_vp, _u8p, _c_int, _c_int, _c_int, _c_int, _u16p], _c_int),
        "sv_gray_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp], _c_int),
        "sv_disparity_dev": ([_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                              _c_int, _c_int, _c_int, _vp, _c_int, _vp], _c_int),
        "sv_harris_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp], _c_int),
        "sv_hog_hist_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp],
                            _c_int),
        "sv_disparity_rows": ([_vp, _u8p, _u8p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                               _c_int, _c_int, _c_int, _c_int, _i16p], _c_int),
        "sv_dev_alloc": ([_vp, ctypes.c_uint64, ctypes.POINTER(_vp)], _c_int),
        "sv_dev_free": ([_vp, _vp], _c_int),
        "sv_host_register": ([_vp, ctypes.c_uint64], _c_int),
        "sv_host_profile_enable": ([_c_int], _c_int),
        "sv_host_profile_read": ([ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong), _c_int],
                                 _c_int),
        "sv_host_unregister": ([_vp], _c_int),
        "sv_timer_begin": ([_vp, _vp], _c_int),
        "sv_timer_end": ([_vp, _vp, ctypes.POINTER(ctypes.c_double)], _c_int),
        "sv_disparity_batch_dev": ([_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.c_int64,
                                    _c_int, _c_int, _c_int, _c_int, _vp, _c_int, ctypes.c_int64,
                                    _vp], _c_int),
        "sv_init_undistort_rectify_map": ([_vp, _f64p, _NullableF64, _c_int, _NullableF64,
                                           _NullableF64, _c_int, _c_int, _c_int, _i16p, _u16p],
                                          _c_int),
        "sv_init_undistort_rectify_map_dev": ([_vp, _f64p, _NullableF64, _c_int, _NullableF64,
                                               _NullableF64, _c_int, _c_int, _c_int, _vp, _vp, _vp],
                                              _c_int),
        "sv_remap": ([_vp, _u8p, _c_int, _c_int, _c_int, _c_int, _i16p, _NullableU16, _c_int,
                      _c_int, _u8p], _c_int),
        "sv_remap_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.c_int64, _vp, _vp,
                          _c_int, _c_int, _c_int, _vp, _c_int, ctypes.c_int64, _c_int, _vp], _c_int),
        "sv_rectify_pair": ([_vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _u8p, _u8p, _c_int, _c_int,
                             _c_int, _c_int, _u8p, _u8p], _c_int),
        "sv_resize_linear": ([_vp, _u8p, _c_int, _c_int, _c_int, _c_int, _u8p, _c_int, _c_int],
                             _c_int),
        "sv_resize_linear_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.c_int64, _vp,
                                  _c_int, _c_int, _c_int, ctypes.c_int64, _c_int, _vp], _c_int),
        "sv_resize_linear_f32_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int,
                                      _vp], _c_int),
        "sv_frame_stats": ([_vp, _u8p, _vp, _c_int, _c_int, _c_int, _c_int, _u32p, _u32p, _u32p],
                           _c_int),
        "sv_frame_stats_batch_dev": ([_vp, _vp, _vp, _c_int, ctypes.c_int64, _c_int, _c_int, _c_int,
                                      _c_int, _vp, _vp, _vp, _vp], _c_int),
        "sv_select_count_batch": ([_vp, _vp, ctypes.c_int64, ctypes.c_int64, _c_int, _c_int, _vp,
                                   ctypes.c_int64, _c_float, _i64p, _i64p], _c_int),
        "sv_select_ranks_batch": ([_vp, _vp, ctypes.c_int64, ctypes.c_int64, _c_int, _c_int, _vp,
                                   ctypes.c_int64, _c_float, _i64p, _c_int, _f32p], _c_int),
        "sv_affine_f32_dev": ([_vp, _vp, ctypes.c_int64, _c_int, _c_float, _c_float, _c_float, _c_float,
                               ctypes.c_double, ctypes.c_double, _vp, _vp], _c_int),
        "sv_sgbm": ([_vp, _u8p, _u8p] + [_c_int] * 14 + [_i16p], _c_int),
        "sv_sgbm_dev": ([_vp, _vp, _vp] + [_c_int] * 13 + [_vp, _c_int, _vp], _c_int),
        "sv_filter_speckles": ([_vp, _i16p] + [_c_int] * 5, _c_int),
        "sv_filter_speckles_dev": ([_vp, _vp] + [_c_int] * 6 + [_vp], _c_int),
        "sv_comm_available": ([], _c_int),
        "sv_comm_unique_id": ([ctypes.c_char_p], _c_int),
        "sv_comm_init_all": ([_c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_vp)], _c_int),
        "sv_comm_destroy": ([_vp], None),
        "sv_comm_rank": ([_vp, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)],
                         _c_int),
        "sv_comm_barrier": ([_vp], _c_int),
        "sv_comm_allreduce_max_f64": ([_vp, ctypes.POINTER(ctypes.c_double)], _c_int),
        "sv_comm_gatherv": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.POINTER(ctypes.c_uint64),
                             ctypes.POINTER(ctypes.c_uint64), _c_int, _vp], _c_int),
        "sv_comm_synchronize": ([_vp], _c_int),
        "sv_comm_scatterv": ([_vp, _vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                              _vp, ctypes.c_uint64, _c_int, _vp], _c_int),
        "sv_band_rows_in": ([_c_int, _c_int, _c_int, _c_int, _c_int, ctypes.POINTER(_c_int)], _c_int),
        "sv_post_m16_dev": ([_vp, _vp, ctypes.c_int64, _c_int, _c_float, _c_float, _c_float,
                             _c_float, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp], _c_int),
        "sv_depth_map_color": ([_vp, _u8p, _u8p] + [_c_int] * 8 + [_c_float] * 4 +
                               [_u8p, _f32p, _f32p, _NullableU8, _u8p], _c_int),
        "sv_stereo_scaled_color": ([_vp, _u8p, _u8p] + [_c_int] * 8 +
                                   [_u8p, _f32p, _f32p, _NullableU8, _f32p, _u8p], _c_int),
        "sv_median_rows_dev": ([_vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                ctypes.POINTER(MapOut), _vp], _c_int),
        "sv_depth_map_batch_dev": ([_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.c_int64,
                                    _c_int, _c_int, _c_int, _c_int, _c_int, _vp, ctypes.POINTER(MapOut),
                                    _vp], _c_int),
        "sv_multi_gpu_dev": ([ctypes.POINTER(_vp), ctypes.POINTER(_vp), _c_int, _c_int, _c_int,
                              ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_c_int), _c_int,
                              _c_int, _c_int, ctypes.c_int64, _c_int, _c_int, _c_int, _c_int,
                              ctypes.POINTER(MapOut)], _c_int),
        "sv_copy_to_device": ([_vp, _vp, _vp, ctypes.c_uint64, _vp], _c_int),
        "sv_copy_to_host": ([_vp, _vp, _vp, ctypes.c_uint64, _vp], _c_int),
        "sv_comm_init_rank": ([_c_int, _c_int, _c_int, ctypes.c_char_p, ctypes.c_double, ctypes.POINTER(_vp)],
                              _c_int),
        "sv_profile_enable": ([_vp, _c_int], _c_int),
        "sv_profile_read": ([_vp, _c_int, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_longlong)], _c_int),
        "sv_profile_reset": ([_vp], _c_int),
        "sv_profile_region_begin": ([_vp, _c_int, _vp], _c_int),
        "sv_profile_region_end": ([_vp, _vp], _c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libsvhip.so (raises EngineUnavailable when it is not built)."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise EngineUnavailable(
                f"libsvhip.so not found at {p}: build it with `python -c 'import "
                f"__graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(p)
        _declare(lib)
        if path is None:
            _lib = lib
        return lib


def last_error() -> str:
    return load_library().sv_last_error().decode(errors="replace")


def _check(fn: str, rc: int):
    if rc != 0:
        raise SVError(fn, rc, last_error())


def device_count() -> int:
    n = _c_int(0)
    rc = load_library().sv_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def plan(num_disp: int, win: int, cost: str | int = "sad") -> dict:
    dpl, lpg, lds = _c_int(), _c_int(), _c_int()
    _check("sv_plan", load_library().sv_plan(num_disp, win, _cost(cost), ctypes.byref(dpl),
                                              ctypes.byref(lpg), ctypes.byref(lds)))
    return {"dpl": dpl.value, "lpg": lpg.value, "lds_bytes": lds.value}


def _cost(cost) -> int:
    if isinstance(cost, str):
        try:
            return COSTS[cost.lower()]
        except KeyError:
            raise ValueError(f"unknown cost {cost!r}; expected one of {sorted(COSTS)}") from None
    return int(cost)


def _image(a: np.ndarray) -> tuple[np.ndarray, int, int, int]:
    a = np.ascontiguousarray(a)
    if a.dtype != np.uint8:
        raise TypeError(f"expected uint8 image, got {a.dtype}")
    if a.ndim == 2:
        return a, a.shape[0], a.shape[1], 1
    if a.ndim == 3 and a.shape[2] == 3:
        return a, a.shape[0], a.shape[1], 3
    raise ValueError(f"expected HxW or HxWx3 image, got shape {a.shape}")


def _refs_first(arrs) -> int:
    for a in arrs:
        return sys.getrefcount(a)
    return 0


def _set_unreferenced(arrs) -> bool:
    """True when no array of the recycling slot `arrs` is referenced outside it."""
    for a in arrs:
        if sys.getrefcount(a) > _BASE_REFS:
            return False
    return True


# references of an array held only by a recycling slot, seen from the same loop shape
# (slot, loop variable, getrefcount's argument): measured, not assumed
_BASE_REFS = _refs_first([np.empty(1)])


class Engine:
    """One libsvhip context (device + stream + cached buffers)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = device_count()
        if n <= 0:
            raise EngineUnavailable("no HIP device visible: the MI355X path cannot run")
        h = _vp()
        rc = self.lib.sv_create(device, ctypes.byref(h))
        if rc != 0:
            raise EngineUnavailable(f"sv_create({device}) failed ({rc}): {last_error()}")
        self._h = h
        self.device = device
        self._scratch: dict[str, tuple[int, int]] = {}
        self._recycle: dict[tuple, list] = {}
        # page-locking recycled outputs (the device epilogue then fills them by DMA, 11 B/px
        # over PCIe) measured slower than downloading the int16 medians (2 B/px) and expanding
        # them on the host (round 5, profiles/r05b/host_ab.txt: 1.26k vs 1.47k frames/s per
        # call, 2.0k vs 2.9k with 4 in flight): opt-in with SV_REGISTER_OUTPUTS=1
        self._noreg = os.environ.get("SV_REGISTER_OUTPUTS", "0") != "1"
        self._out_lock = threading.Lock()

    # -- lifetime -------------------------------------------------------------------
    def close(self):
        for sets in getattr(self, "_recycle", {}).values():
            for arrs in sets:
                self._unregister(arrs)
        self._recycle = {}
        if getattr(self, "_h", None):
            for p, _ in self._scratch.values():
                self.lib.sv_dev_free(self._h, p)
            self._scratch = {}
            self.lib.sv_destroy(self._h)
            self._h = None

    def scratch(self, name: str, nbytes: int) -> int:
        """A grow-only device buffer owned by this engine (for host-array entry points)."""
        p, cap = self._scratch.get(name, (0, 0))
        if cap < nbytes:
            if p:
                self.dev_free(p)
            p = self.dev_alloc(max(int(nbytes), 256))
            self._scratch[name] = (p, max(int(nbytes), 256))
        return p

    def outputs(self, specs) -> tuple:
        """Fresh-looking output arrays for a host-buffer call: ((shape, dtype), ...) ->
        arrays.  A set this engine returned before is handed out again once the caller holds
        no reference to any of its arrays (or to views of them), so a steady stream of
        frames writes into resident pages instead of page-faulting 20+ MB of new memory per
        1080p frame.  At most 3 sets per shape are kept."""
        key = tuple((tuple(sh), np.dtype(dt).str) for sh, dt in specs)
        # the reference calls the path from a 2-worker thread pool (fused_depth_map.py:2299,
        # :2591-2598): the check-and-take must be atomic, or two threads could both find a
        # released set and share it
        with self._out_lock:
            sets = self._recycle.setdefault(key, [])
            for arrs in sets:
                if _set_unreferenced(arrs):
                    self._register(arrs)
                    return tuple(arrs)
            arrs = [np.empty(sh, dt) for sh, dt in specs]
            if len(sets) < 3:
                sets.append(arrs)
            else:
                # a full slot evicts its oldest RELEASED set (never one a caller — or another
                # thread's call in flight — still holds: unregistering it could pull pinned
                # pages from under a DMA); when every kept set is in use the new one is handed
                # out untracked
                for i in range(len(sets)):
                    if _set_unreferenced(sets[i]):
                        self._unregister(sets.pop(i))
                        sets.append(arrs)
                        break
            return tuple(arrs)

    def _register(self, arrs):
        """Page-lock a recycled output set (on its first reuse, so callers that keep every
        result never pay for it): the C path then DMAs the outputs straight into it."""
        if getattr(self, "_noreg", False) or not hasattr(self, "lib"):
            return
        # keyed by id with the address only: a strong reference here would count against
        # _set_unreferenced, so a registered set would never be handed out again (every
        # other call then allocated, page-faulted and registered a fresh set)
        regs = self.__dict__.setdefault("_registered", {})
        for a in arrs:
            if a.nbytes and id(a) not in regs:
                if self.lib.sv_host_register(a.ctypes.data, a.nbytes) != 0:
                    self._noreg = True     # e.g. a page-lock limit: keep the host expansion
                    return
                regs[id(a)] = a.ctypes.data

    def _unregister(self, arrs):
        regs = self.__dict__.get("_registered", {})
        for a in arrs:
            if regs.pop(id(a), None) is not None:
                self.lib.sv_host_unregister(a.ctypes.data)

    def registered_outputs(self) -> int:
        """Output arrays currently page-locked for the DMA path (diagnostics)."""
        return len(self.__dict__.get("_registered", {}))

    def upload(self, name: str, a: np.ndarray) -> int:
        """Copy a host array into the named scratch buffer; returns its device pointer."""
        a = np.ascontiguousarray(a)
        p = self.scratch(name, a.nbytes)
        if a.nbytes:
            self.to_device(p, a)
        return p

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return self.lib.sv_stream(self._h) or 0

    def synchronize(self):
        _check("sv_synchronize", self.lib.sv_synchronize(self._h))

    def event_record(self, slot: int, stream: int = 0):
        """Mark the work enqueued on `stream` so far (event slot 0..15 of this context)."""
        _check("sv_event_record", self.lib.sv_event_record(self._h, int(slot), stream or None))

    def stream_wait_event(self, slot: int, stream: int = 0):
        """Work enqueued on `stream` from now on waits for the mark in `slot`."""
        _check("sv_stream_wait_event", self.lib.sv_stream_wait_event(self._h, int(slot), stream or None))

    def release_scratch(self):
        """Free the context's grow-only device scratch (e.g. after a large SGBM batch)."""
        _check("sv_release_scratch", self.lib.sv_release_scratch(self._h))

    # -- host-memory entry points -----------------------------------------------------
    def gray(self, bgr: np.ndarray) -> np.ndarray:
        bgr, H, W, C = _image(bgr)
        if C != 3:
            raise ValueError("gray() expects an HxWx3 BGR image")
        out = np.empty((H, W), np.uint8)
        _check("sv_gray", self.lib.sv_gray(self._h, bgr, H, W, W * 3, out))
        return out

    def disparity(self, left, right, min_disp: int, num_disp: int, win: int, cost="sad",
                  harris: bool = False):
        """int16 x16 disparity (StereoSGBM.compute convention) [+ Harris of the left]."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        d16 = np.empty((H, W), np.int16)
        hr = np.empty((H, W), np.float32) if harris else None
        _check("sv_disparity", self.lib.sv_disparity(self._h, left, right, H, W, C, W * C,
                                                     int(min_disp), int(num_disp), int(win),
                                                     _cost(cost), d16, hr))
        return (d16, hr) if harris else d16

    def sgbm(self, left, right, min_disp: int, num_disp: int, block_size: int, P1: int = None,
             P2: int = None, disp12_max_diff: int = 1, pre_filter_cap: int = 63,
             uniqueness_ratio: int = 10, speckle_window_size: int = 100,
             speckle_range: int = 32) -> np.ndarray:
        """cv2.StereoSGBM_create(..., mode=MODE_SGBM_3WAY).compute(left, right) -> int16 x16
        (defaults: the reference's parameters, depth_map.py:894-906)."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        P1 = 8 * 3 * block_size * block_size if P1 is None else P1
        P2 = 32 * 3 * block_size * block_size if P2 is None else P2
        d16 = np.empty((H, W), np.int16)
        _check("sv_sgbm", self.lib.sv_sgbm(self._h, left, right, H, W, C, W * C, int(min_disp),
                                           int(num_disp), int(block_size), int(P1), int(P2),
                                           int(disp12_max_diff), int(pre_filter_cap),
                                           int(uniqueness_ratio), int(speckle_window_size),
                                           int(speckle_range), d16))
        return d16

    def sgbm_dev(self, d_left: int, d_right: int, H: int, W: int, pitch: int, min_disp: int,
                 num_disp: int, block_size: int, d_out16: int, out_pitch: int, P1: int = None,
                 P2: int = None, disp12_max_diff: int = 1, pre_filter_cap: int = 63,
                 uniqueness_ratio: int = 10, speckle_window_size: int = 100,
                 speckle_range: int = 32, stream: int = 0):
        P1 = 8 * 3 * block_size * block_size if P1 is None else P1
        P2 = 32 * 3 * block_size * block_size if P2 is None else P2
        _check("sv_sgbm_dev", self.lib.sv_sgbm_dev(
            self._h, d_left, d_right, H, W, pitch, int(min_disp), int(num_disp), int(block_size),
            int(P1), int(P2), int(disp12_max_diff), int(pre_filter_cap), int(uniqueness_ratio),
            int(speckle_window_size), int(speckle_range), d_out16, out_pitch, stream or None))

    def filter_speckles(self, img: np.ndarray, new_val: int, max_speckle_size: int,
                        max_diff: int) -> np.ndarray:
        """cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on an int16 map; returns
        the filtered copy."""
        img = np.ascontiguousarray(img, np.int16).copy()
        if img.ndim != 2:
            raise ValueError("filter_speckles expects an H x W int16 map")
        H, W = img.shape
        _check("sv_filter_speckles", self.lib.sv_filter_speckles(
            self._h, img, H, W, int(new_val), int(max_speckle_size), int(max_diff)))
        return img

    def filter_speckles_dev(self, d_img: int, H: int, W: int, pitch: int, new_val: int,
                            max_speckle_size: int, max_diff: int, stream: int = 0):
        _check("sv_filter_speckles_dev", self.lib.sv_filter_speckles_dev(
            self._h, d_img, H, W, pitch, int(new_val), int(max_speckle_size), int(max_diff),
            stream or None))

    def disparity_rows(self, left, right, min_disp: int, num_disp: int, win: int, row0: int,
                       row1: int, cost="sad", out: np.ndarray | None = None) -> np.ndarray:
        """Rows [row0, row1) of the int16 x16 disparity (a row-tiled shard); other rows of
        ``out`` are left untouched."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        if out is None:
            out = np.zeros((H, W), np.int16)
        _check("sv_disparity_rows", self.lib.sv_disparity_rows(
            self._h, left, right, H, W, C, W * C, int(min_disp), int(num_disp), int(win),
            _cost(cost), int(row0), int(row1), out))
        return out

    # -- device buffers (torch-free zero-copy use) ------------------------------------
    def dev_alloc(self, nbytes: int) -> int:
        p = _vp()
        _check("sv_dev_alloc", self.lib.sv_dev_alloc(self._h, int(nbytes), ctypes.byref(p)))
        return p.value

    def dev_free(self, ptr: int):
        _check("sv_dev_free", self.lib.sv_dev_free(self._h, ptr))

    def to_device(self, ptr: int, a: np.ndarray, stream: int = 0):
        """Host array -> device; synchronous unless `stream` (then enqueued there: keep `a`
        alive, and page-locked for the copy to overlap device work)."""
        a = np.ascontiguousarray(a)
        _check("sv_copy_to_device", self.lib.sv_copy_to_device(self._h, ptr, a.ctypes.data, a.nbytes,
                                                                stream or None))

    def to_host(self, ptr: int, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        _check("sv_copy_to_host", self.lib.sv_copy_to_host(self._h, out.ctypes.data, ptr, out.nbytes, None))
        return out

    def median5(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float32)
        out = np.empty_like(a)
        _check("sv_median5_f32", self.lib.sv_median5_f32(self._h, a, a.shape[0], a.shape[1], out))
        return out

    def depth_post(self, disparity, min_depth: float, max_depth: float, min_disp_global=0):
        d = np.ascontiguousarray(disparity, np.float32)
        df = np.empty_like(d)
        nm = np.empty(d.shape, np.uint8)
        _check("sv_depth_post", self.lib.sv_depth_post(
            self._h, d, d.size, np.float32(min_depth), np.float32(max_depth),
            np.float32(float(max_depth) - float(min_depth)), np.float32(min_disp_global), df, nm))
        return df, nm

    def scaled_post(self, disparity, min_disp: int, num_disp: int):
        d = np.ascontiguousarray(disparity, np.float32)
        dn = np.empty_like(d)
        du = np.empty(d.shape, np.uint8)
        cf = np.empty_like(d)
        _check("sv_scaled_post", self.lib.sv_scaled_post(self._h, d, d.size, int(min_disp),
                                                         int(num_disp), dn, du, cf))
        return dn, du, cf

    def depth_map(self, left, right, min_disp: int, num_disp: int, win: int, min_depth: float,
                  max_depth: float, min_disp_global=None, cost="sad"):
        """Numeric body of depth_map.create_depth_map: (depth_final, disparity, depth_u8)."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        mdg = min_disp if min_disp_global is None else min_disp_global
        depth = np.empty((H, W), np.float32)
        disp = np.empty((H, W), np.float32)
        norm = np.empty((H, W), np.uint8)
        _check("sv_depth_map", self.lib.sv_depth_map(
            self._h, left, right, H, W, C, W * C, int(min_disp), int(num_disp), int(win),
            _cost(cost), np.float32(min_depth), np.float32(max_depth),
            np.float32(float(max_depth) - float(min_depth)), np.float32(mdg), depth, disp, norm))
        return depth, disp, norm

    def stereo_scaled(self, left, right, min_disp: int, num_disp: int, win: int, cost="sad"):
        """Numeric body of create_depth_map_stereo_scaled:
        (disparity_normalized f32, disparity f32, normalized u8, confidence f32)."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        dn = np.empty((H, W), np.float32)
        disp = np.empty((H, W), np.float32)
        du = np.empty((H, W), np.uint8)
        cf = np.empty((H, W), np.float32)
        _check("sv_stereo_scaled", self.lib.sv_stereo_scaled(
            self._h, left, right, H, W, C, W * C, int(min_disp), int(num_disp), int(win),
            _cost(cost), dn, disp, du, cf))
        return dn, disp, du, cf

    def depth_map_color(self, left, right, min_disp: int, num_disp: int, win: int,
                        min_depth: float, max_depth: float, cmap_bgr: np.ndarray,
                        min_disp_global=None, cost="sad", with_normalized: bool = False, out=None):
        """create_depth_map's outputs with the colormap computed on the GPU:
        (depth_final, disparity, depth_colormap HxWx3 BGR[, depth_normalized]).
        `out`: optional (depth, disparity, colormap) arrays to fill instead of new ones."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        lut = np.ascontiguousarray(cmap_bgr, np.uint8).reshape(256, 3)
        mdg = min_disp if min_disp_global is None else min_disp_global
        if out is not None:
            depth, disp, cmap = out
            if (depth.shape, disp.shape, cmap.shape) != ((H, W), (H, W), (H, W, 3)) or \
                    (depth.dtype, disp.dtype, cmap.dtype) != (np.float32, np.float32, np.uint8) or \
                    not all(a.flags.c_contiguous for a in out):
                raise ValueError("out arrays must be C-contiguous (H,W) f32, (H,W) f32, (H,W,3) u8")
        else:
            depth, disp, cmap = self.outputs((((H, W), np.float32), ((H, W), np.float32), ((H, W, 3), np.uint8)))
        norm = np.empty((H, W), np.uint8) if with_normalized else None
        _check("sv_depth_map_color", self.lib.sv_depth_map_color(
            self._h, left, right, H, W, C, W * C, int(min_disp), int(num_disp), int(win),
            _cost(cost), np.float32(min_depth), np.float32(max_depth),
            np.float32(float(max_depth) - float(min_depth)), np.float32(mdg), lut, depth, disp,
            norm, cmap))
        return (depth, disp, cmap, norm) if with_normalized else (depth, disp, cmap)

    def stereo_scaled_color(self, left, right, min_disp: int, num_disp: int, win: int,
                            cmap_bgr: np.ndarray, cost="sad", with_normalized: bool = False):
        """create_depth_map_stereo_scaled's outputs with the colormap on the GPU:
        (disparity_normalized, disparity, colormap HxWx3 BGR, confidence[, normalized u8])."""
        left, H, W, C = _image(left)
        right, H2, W2, C2 = _image(right)
        if (H, W, C) != (H2, W2, C2):
            raise ValueError("left/right shapes differ")
        lut = np.ascontiguousarray(cmap_bgr, np.uint8).reshape(256, 3)
        dn, disp, cf, cmap = self.outputs((((H, W), np.float32), ((H, W), np.float32), ((H, W), np.float32),
                                           ((H, W, 3), np.uint8)))
        du = np.empty((H, W), np.uint8) if with_normalized else None
        _check("sv_stereo_scaled_color", self.lib.sv_stereo_scaled_color(
            self._h, left, right, H, W, C, W * C, int(min_disp), int(num_disp), int(win),
            _cost(cost), lut, dn, disp, du, cf, cmap))
        return (dn, disp, cmap, cf, du) if with_normalized else (dn, disp, cmap, cf)

    def harris(self, gray: np.ndarray) -> np.ndarray:
        gray, H, W, C = _image(gray)
        if C != 1:
            raise ValueError("harris() expects a gray image")
        out = np.empty((H, W), np.float32)
        _check("sv_harris", self.lib.sv_harris(self._h, gray, H, W, W, out))
        return out

    def hog_hist(self, gray: np.ndarray, win: int) -> np.ndarray:
        """[9, H, W] uint16 window histograms (the device layout is [H][W][10])."""
        gray, H, W, C = _image(gray)
        if C != 1:
            raise ValueError("hog_hist() expects a gray image")
        out = np.empty((H, W, 10), np.uint16)
        _check("sv_hog_hist", self.lib.sv_hog_hist(self._h, gray, H, W, W, int(win), out))
        return np.ascontiguousarray(out[:, :, :9].transpose(2, 0, 1))

    # -- device-memory entry points (integer device pointers) ---------------------------
    def gray_dev(self, d_bgr: int, H: int, W: int, pitch: int, d_gray: int, stream: int = 0):
        _check("sv_gray_dev", self.lib.sv_gray_dev(self._h, d_bgr, H, W, pitch, d_gray,
                                                   stream or None))

    def disparity_dev(self, d_left: int, d_right: int, H: int, W: int, pitch: int,
                      min_disp: int, num_disp: int, win: int, cost, row0: int, row1: int,
                      d_out16: int, out_pitch: int, stream: int = 0):
        _check("sv_disparity_dev", self.lib.sv_disparity_dev(
            self._h, d_left, d_right, H, W, pitch, int(min_disp), int(num_disp), int(win),
            _cost(cost), int(row0), int(row1), d_out16, out_pitch, stream or None))

    def median_rows_dev(self, d_disp16: int, H: int, W: int, row0: int, row1: int, out: "MapOut",
                        min_disp: int = 0, num_disp: int = 0, cost="sad", stream: int = 0):
        """sv_median_rows_dev: median (+ post) of rows [row0, row1) into the outputs of `out`
        (:func:`map_out`), at full-frame offsets."""
        _check("sv_median_rows_dev", self.lib.sv_median_rows_dev(
            self._h, d_disp16, H, W, int(row0), int(row1), int(min_disp), int(num_disp), _cost(cost),
            ctypes.byref(out), stream or None))

    def median_post_dev(self, d_disp16: int, H: int, W: int, row0: int, row1: int, mode: int,
                        d_disparity: int, d_out_a: int = 0, d_out_u8: int = 0, d_out_b: int = 0,
                        min_depth=0.0, max_depth=0.0, min_disp_global=0.0, min_disp=0,
                        num_disp=0, stream: int = 0, cost="sad"):
        self.median_rows_dev(d_disp16, H, W, row0, row1,
                             map_out(mode, d_disparity, d_out_a, d_out_u8, d_out_b, min_depth=min_depth,
                                     max_depth=max_depth, min_disp_global=min_disp_global),
                             min_disp, num_disp, cost, stream)

    def median_post_m16_dev(self, d_disp16: int, H: int, W: int, row0: int, row1: int, mode: int,
                            d_disparity: int = 0, d_out_a: int = 0, d_out_u8: int = 0,
                            d_out_b: int = 0, d_med16: int = 0, min_depth=0.0, max_depth=0.0,
                            min_disp_global=0.0, min_disp=0, num_disp=0, stream: int = 0, cost="sad"):
        """Median of rows [row0, row1) plus (mode) the post outputs and/or the int16 x16
        medians d_med16 (full-frame offsets)."""
        self.median_rows_dev(d_disp16, H, W, row0, row1,
                             map_out(mode, d_disparity, d_out_a, d_out_u8, d_out_b, med16=d_med16,
                                     min_depth=min_depth, max_depth=max_depth,
                                     min_disp_global=min_disp_global),
                             min_disp, num_disp, cost, stream)

    def median_map_dev(self, d_disp16: int, H: int, W: int, row0: int, row1: int, d_map: int,
                       fmt="m16", min_disp: int = 0, num_disp: int = 0, stream: int = 0, cost="sad"):
        """Median of rows [row0, row1) written only as a gather map at full-frame offsets of
        d_map (``fmt`` "m16": int16 x16, "d8": u8 indices; d8 needs an integer cost)."""
        f = _map_format(fmt)
        self.median_rows_dev(d_disp16, H, W, row0, row1,
                             map_out(POST_NONE, med16=d_map if f == MAP_M16 else 0,
                                     d8=d_map if f == MAP_D8 else 0),
                             min_disp, num_disp, cost, stream)

    def post_m16_dev(self, d_med16: int, n: int, mode: int, d_disparity: int = 0, d_out_a: int = 0,
                     d_out_u8: int = 0, d_out_b: int = 0, min_depth=0.0, max_depth=0.0,
                     min_disp_global=0.0, min_disp=0, num_disp=0, stream: int = 0):
        """sv_post_m16_dev: n int16 x16 medians -> disparity (m / 16) and mode's outputs."""
        _check("sv_post_m16_dev", self.lib.sv_post_m16_dev(
            self._h, d_med16, int(n), int(mode), np.float32(min_depth), np.float32(max_depth),
            np.float32(float(max_depth) - float(min_depth)), np.float32(min_disp_global),
            int(min_disp), int(num_disp), d_disparity or None, d_out_a or None, d_out_u8 or None,
            d_out_b or None, stream or None))

    def median_post_color_dev(self, d_disp16: int, H: int, W: int, row0: int, row1: int, mode: int,
                              cmap_bgr: np.ndarray, d_disparity: int, d_out_a: int, d_out_u8: int,
                              d_bgr: int, d_out_b: int = 0, min_depth=0.0, max_depth=0.0,
                              min_disp_global=0.0, min_disp=0, num_disp=0, stream: int = 0, cost="sad"):
        if mode not in (POST_DEPTH, POST_SCALED):
            raise ValueError("the colormap epilogue needs POST_DEPTH or POST_SCALED")
        self.median_rows_dev(d_disp16, H, W, row0, row1,
                             map_out(mode, d_disparity, d_out_a, d_out_u8, d_out_b, bgr=d_bgr, cmap=cmap_bgr,
                                     min_depth=min_depth, max_depth=max_depth,
                                     min_disp_global=min_disp_global),
                             min_disp, num_disp, cost, stream)

    def depth_map_dev(self, d_left: int, d_right: int, H: int, W: int, pitch: int,
                      min_disp: int, num_disp: int, win: int, min_depth: float,
                      max_depth: float, d_depth: int, d_disp: int, d_norm: int, cost="sad",
                      min_disp_global=None, stream: int = 0):
        """Whole app-1 device path on one gray device frame pair (a batch of one)."""
        self.depth_map_batch_dev(d_left, d_right, 1, H, W, pitch, pitch * H, min_disp, num_disp, win,
                                 min_depth, max_depth, d_depth, d_disp, d_norm, cost=cost,
                                 min_disp_global=min_disp_global, stream=stream)

    # -- frame batches (one launch per kernel over all frames) ------------------------------
    def disparity_batch_dev(self, d_left: int, d_right: int, n_frames: int, H: int, W: int,
                            pitch: int, frame_stride: int, min_disp: int, num_disp: int,
                            win: int, cost, d_out16: int, out_pitch: int,
                            out_frame_stride: int, stream: int = 0):
        _check("sv_disparity_batch_dev", self.lib.sv_disparity_batch_dev(
            self._h, d_left, d_right, int(n_frames), H, W, pitch, int(frame_stride),
            int(min_disp), int(num_disp), int(win), _cost(cost), d_out16, out_pitch,
            int(out_frame_stride), stream or None))

    def median_post_batch_dev(self, d_disp16: int, n_frames: int, H: int, W: int, mode: int,
                              d_disparity: int, d_out_a: int = 0, d_out_u8: int = 0,
                              d_out_b: int = 0, min_depth=0.0, max_depth=0.0,
                              min_disp_global=0.0, min_disp=0, num_disp=0, stream: int = 0,
                              cost="sad", win: int = 1, d_med16: int = 0, d_d8: int = 0):
        """The median stage alone over n_frames int16 x16 maps (dense per frame): SV_STAGE_MEDIAN
        of sv_depth_map_batch_dev."""
        self.depth_map_batch_ex(0, 0, n_frames, H, W, W, H * W, min_disp, num_disp, win, cost, STAGE_MEDIAN,
                                d_disp16, map_out(mode, d_disparity, d_out_a, d_out_u8, d_out_b, med16=d_med16,
                                                  d8=d_d8, min_depth=min_depth, max_depth=max_depth,
                                                  min_disp_global=min_disp_global), stream)

    def depth_map_batch_ex(self, d_left: int, d_right: int, n_frames: int, H: int, W: int, pitch: int,
                           frame_stride: int, min_disp: int, num_disp: int, win: int, cost, stages: int,
                           d_disp16: int, out: "MapOut | None", stream: int = 0):
        """sv_depth_map_batch_dev as the C ABI has it: `stages` (STAGE_MATCH / STAGE_MEDIAN /
        STAGE_ALL), the int16 x16 maps in d_disp16 (0 with STAGE_ALL: the context's scratch) and
        the outputs of `out` (:func:`map_out`)."""
        _check("sv_depth_map_batch_dev", self.lib.sv_depth_map_batch_dev(
            self._h, d_left or None, d_right or None, int(n_frames), H, W, pitch, int(frame_stride),
            int(min_disp), int(num_disp), int(win), _cost(cost), int(stages), d_disp16 or None,
            ctypes.byref(out) if out is not None else None, stream or None))

    def depth_map_batch_dev(self, d_left: int, d_right: int, n_frames: int, H: int, W: int,
                            pitch: int, frame_stride: int, min_disp: int, num_disp: int,
                            win: int, min_depth: float, max_depth: float, d_depth: int,
                            d_disp: int, d_norm: int, cost="sad", min_disp_global=None,
                            stream: int = 0, d_med16: int = 0, d_harris: int = 0, d_d8: int = 0):
        """create_depth_map over a batch of device frame pairs.  d_med16 (optional): also the
        int16 x16 median maps (d_disp = d_med16 / 16 exactly).  d_d8 (optional): also the u8
        disparity indices d_disp - (min_disp - 1) (integer costs, num_disp <= 255).  d_harris
        (optional): also the Harris response of every left frame, computed inside the median
        launch."""
        mdg = min_disp if min_disp_global is None else min_disp_global
        out = map_out(POST_DEPTH, d_disp, d_depth, d_norm, med16=d_med16, d8=d_d8, harris=d_harris,
                      min_depth=min_depth, max_depth=max_depth, min_disp_global=mdg)
        self.depth_map_batch_ex(d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp, num_disp, win,
                                cost, STAGE_ALL, 0, out, stream)

    def harris_batch_dev(self, d_gray: int, n_frames: int, H: int, W: int, pitch: int,
                         frame_stride: int, d_out: int, stream: int = 0):
        _check("sv_harris_batch_dev", self.lib.sv_harris_batch_dev(
            self._h, d_gray, int(n_frames), H, W, pitch, int(frame_stride), d_out, stream or None))

    def harris_dev(self, d_gray: int, H: int, W: int, pitch: int, d_out: int, stream: int = 0):
        _check("sv_harris_dev", self.lib.sv_harris_dev(self._h, d_gray, H, W, pitch, d_out,
                                                       stream or None))

    def hog_hist_dev(self, d_gray: int, H: int, W: int, pitch: int, win: int, row0: int,
                     row1: int, d_out: int, stream: int = 0):
        _check("sv_hog_hist_dev", self.lib.sv_hog_hist_dev(self._h, d_gray, H, W, pitch, win,
                                                           row0, row1, d_out, stream or None))

    # -- rectification (initUndistortRectifyMap / remap) ------------------------------------
    @staticmethod
    def _map_params(K, dist, R, P):
        K = np.ascontiguousarray(np.asarray(K, np.float64).reshape(3, 3))
        d = None if dist is None else np.ascontiguousarray(np.asarray(dist, np.float64).ravel())
        nd = 0 if d is None else int(d.size)
        if nd == 0:
            d = None
        Rm = None if R is None else np.ascontiguousarray(np.asarray(R, np.float64).reshape(3, 3))
        Pm = None
        pc = 3
        if P is not None:
            Pm = np.asarray(P, np.float64)
            pc = Pm.size // 3
            Pm = np.ascontiguousarray(Pm.reshape(3, pc))
        return K, d, nd, Rm, Pm, pc

    def init_undistort_rectify_map(self, K, dist, R, P, width: int, height: int):
        """cv2.initUndistortRectifyMap(K, dist, R, P, (width, height), CV_16SC2) ->
        (map1 int16 [H, W, 2], map2 uint16 [H, W])."""
        K, d, nd, Rm, Pm, pc = self._map_params(K, dist, R, P)
        m1 = np.empty((height, width, 2), np.int16)
        m2 = np.empty((height, width), np.uint16)
        _check("sv_init_undistort_rectify_map", self.lib.sv_init_undistort_rectify_map(
            self._h, K, d, nd, Rm, Pm, pc, int(height), int(width), m1, m2))
        return m1, m2

    def init_undistort_rectify_map_dev(self, K, dist, R, P, width: int, height: int, d_map1: int,
                                       d_map2: int, stream: int = 0):
        K, d, nd, Rm, Pm, pc = self._map_params(K, dist, R, P)
        _check("sv_init_undistort_rectify_map_dev", self.lib.sv_init_undistort_rectify_map_dev(
            self._h, K, d, nd, Rm, Pm, pc, int(height), int(width), d_map1, d_map2, stream or None))

    def remap(self, src, map1, map2) -> np.ndarray:
        """cv2.remap(src, map1, map2, cv2.INTER_LINEAR) (BORDER_CONSTANT 0), uint8 gray/BGR."""
        src, sH, sW, C = _image(src)
        m1 = np.ascontiguousarray(map1, np.int16)
        if m1.ndim != 3 or m1.shape[2] != 2:
            raise ValueError(f"map1 must be HxWx2 int16 (CV_16SC2), got {m1.shape}")
        H, W = m1.shape[:2]
        m2 = None
        if map2 is not None and np.asarray(map2).size:
            m2 = np.ascontiguousarray(map2, np.uint16)
            if m2.shape != (H, W):
                raise ValueError(f"map2 shape {m2.shape} != {(H, W)}")
        out = np.empty((H, W, C) if C == 3 else (H, W), np.uint8)
        _check("sv_remap", self.lib.sv_remap(self._h, src, sH, sW, C, sW * C, m1, m2, H, W, out))
        return out

    def remap_dev(self, d_src: int, sH: int, sW: int, channels: int, src_pitch: int,
                  d_map1: int, d_map2: int, H: int, W: int, d_dst: int, dst_pitch: int,
                  gray_out: bool = False, n_frames: int = 1, src_frame_stride: int = 0,
                  dst_frame_stride: int = 0, stream: int = 0):
        _check("sv_remap_dev", self.lib.sv_remap_dev(
            self._h, d_src, sH, sW, channels, src_pitch, int(src_frame_stride), d_map1,
            d_map2 or None, H, W, 1 if gray_out else 0, d_dst, dst_pitch, int(dst_frame_stride),
            int(n_frames), stream or None))

    def resize(self, src, width: int, height: int) -> np.ndarray:
        """cv2.resize(src, (width, height)) with INTER_LINEAR, uint8 gray/BGR."""
        src, sH, sW, C = _image(src)
        if (sH, sW) == (height, width):
            return src.copy()
        out = np.empty((height, width, C) if C == 3 else (height, width), np.uint8)
        _check("sv_resize_linear", self.lib.sv_resize_linear(self._h, src, sH, sW, C, sW * C, out,
                                                             int(height), int(width)))
        return out

    def resize_dev(self, d_src: int, sH: int, sW: int, channels: int, src_pitch: int, d_dst: int,
                   dH: int, dW: int, dst_pitch: int, n_frames: int = 1, src_frame_stride: int = 0,
                   dst_frame_stride: int = 0, stream: int = 0):
        _check("sv_resize_linear_dev", self.lib.sv_resize_linear_dev(
            self._h, d_src, sH, sW, channels, src_pitch, int(src_frame_stride), d_dst, dH, dW,
            dst_pitch, int(dst_frame_stride), int(n_frames), stream or None))

    def resize_f32_dev(self, d_src: int, sH: int, sW: int, d_dst: int, dH: int, dW: int,
                       stream: int = 0):
        _check("sv_resize_linear_f32_dev", self.lib.sv_resize_linear_f32_dev(
            self._h, d_src, sH, sW, sW * 4, d_dst, dH, dW, dW * 4, stream or None))

    # -- reductions (occlusion statistics, percentile order statistics) ------------------
    def frame_stats(self, img0, img1=None):
        """Per-48x48-block (sum, sum of squares) and the 256-bin histogram of one gray/BGR
        image or a pair -> (block_sum [n, bh, bw], block_sq [n, bh, bw], hist [n, 256])."""
        img0, H, W, C = _image(img0)
        n = 1
        if img1 is not None:
            img1, H2, W2, C2 = _image(img1)
            if (H2, W2, C2) != (H, W, C):
                raise ValueError("frame_stats: the two images differ in shape")
            n = 2
        bh, bw = max(1, H // 48), max(1, W // 48)
        bs = np.empty((n, bh, bw), np.uint32)
        bq = np.empty((n, bh, bw), np.uint32)
        hist = np.empty((n, 256), np.uint32)
        _check("sv_frame_stats", self.lib.sv_frame_stats(
            self._h, img0, img1.ctypes.data if img1 is not None else None, H, W, C, W * C, bs, bq,
            hist))
        return bs, bq, hist

    def frame_stats_dev(self, d_img0: int, d_img1: int, H: int, W: int, channels: int, pitch: int,
                        d_block_sum: int, d_block_sq: int, d_hist: int, stream: int = 0):
        """One image or pair: the batch entry point with one frame."""
        self.frame_stats_batch_dev(d_img0, d_img1, 1, 0, H, W, channels, pitch, d_block_sum, d_block_sq,
                                   d_hist, stream)

    def frame_stats_batch_dev(self, d_img0: int, d_img1: int, n_frames: int, frame_stride: int, H: int,
                              W: int, channels: int, pitch: int, d_block_sum: int, d_block_sq: int,
                              d_hist: int, stream: int = 0):
        """detect_camera_occlusion's image statistics for a batch of frames (or pairs) in one
        launch: outputs dense per image (frame-major, img0 before img1)."""
        _check("sv_frame_stats_batch_dev", self.lib.sv_frame_stats_batch_dev(
            self._h, d_img0, d_img1 or None, int(n_frames), int(frame_stride), H, W, channels, pitch,
            d_block_sum, d_block_sq, d_hist, stream or None))

    def select_count(self, d_x: int, n: int, mask_mode: int = 0, d_mask: int = 0,
                     thr: float = 0.0) -> tuple[int, int]:
        sel, nan = self.select_count_batch(d_x, n, n, 1, mask_mode, d_mask, n, thr)
        return int(sel[0]), int(nan[0])

    def select_ranks(self, d_x: int, n: int, ranks, mask_mode: int = 0, d_mask: int = 0,
                     thr: float = 0.0) -> np.ndarray:
        r = np.asarray(ranks, np.int64).reshape(1, -1)
        return self.select_ranks_batch(d_x, n, n, r, mask_mode, d_mask, n, thr)[0]

    def select_count_batch(self, d_x: int, n: int, x_stride: int, n_arrays: int, mask_mode: int = 0,
                           d_mask: int = 0, mask_stride: int = 0, thr: float = 0.0):
        """select_count of n_arrays arrays (array y at d_x + 4 * y * x_stride) in one pass."""
        sel = np.zeros(n_arrays, np.int64)
        nan = np.zeros(n_arrays, np.int64)
        _check("sv_select_count_batch", self.lib.sv_select_count_batch(
            self._h, d_x, int(n), int(x_stride), int(n_arrays), int(mask_mode), d_mask or None,
            int(mask_stride), np.float32(thr), sel, nan))
        return sel, nan

    def select_ranks_batch(self, d_x: int, n: int, x_stride: int, ranks, mask_mode: int = 0,
                           d_mask: int = 0, mask_stride: int = 0, thr: float = 0.0) -> np.ndarray:
        """ranks: [n_arrays][nranks] -> values [n_arrays][nranks] (three passes for the batch)."""
        r = np.ascontiguousarray(np.asarray(ranks, np.int64))
        if r.ndim != 2:
            raise ValueError("ranks must be [n_arrays][nranks]")
        out = np.empty(r.shape, np.float32)
        _check("sv_select_ranks_batch", self.lib.sv_select_ranks_batch(
            self._h, d_x, int(n), int(x_stride), r.shape[0], int(mask_mode), d_mask or None,
            int(mask_stride), np.float32(thr), r.ravel(), r.shape[1], out.ravel()))
        return out

    def affine_f32_dev(self, d_x: int, n: int, mode: int, d_out: int, fa=0.0, fb=1.0, fc=0.0,
                       fd=0.0, ds=1.0, doff=0.0, stream: int = 0):
        _check("sv_affine_f32_dev", self.lib.sv_affine_f32_dev(
            self._h, d_x, int(n), int(mode), np.float32(fa), np.float32(fb), np.float32(fc),
            np.float32(fd), float(ds), float(doff), d_out, stream or None))

    def rectify_pair(self, dmaps, left, right):
        """Both remaps of apply_stereo_rectification with device-resident maps
        (``dmaps`` = (d_map1_l, d_map2_l, d_map1_r, d_map2_r, H, W))."""
        left, sH, sW, C = _image(left)
        right, sH2, sW2, C2 = _image(right)
        if (sH, sW, C) != (sH2, sW2, C2):
            raise ValueError("left/right shapes differ")
        m1l, m2l, m1r, m2r, H, W = dmaps
        shape = (H, W, C) if C == 3 else (H, W)
        ol = np.empty(shape, np.uint8)
        orr = np.empty(shape, np.uint8)
        _check("sv_rectify_pair", self.lib.sv_rectify_pair(
            self._h, m1l, m2l, m1r, m2r, H, W, left, right, sH, sW, C, sW * C, ol, orr))
        return ol, orr

    # -- profiling ------------------------------------------------------------------------
    def timer_begin(self, stream: int = 0):
        _check("sv_timer_begin", self.lib.sv_timer_begin(self._h, stream or None))

    def timer_end(self, stream: int = 0) -> float:
        """Device milliseconds since the matching timer_begin on the same stream."""
        ms = ctypes.c_double()
        _check("sv_timer_end", self.lib.sv_timer_end(self._h, stream or None, ctypes.byref(ms)))
        return ms.value

    def profile(self, on: bool = True):
        _check("sv_profile_enable", self.lib.sv_profile_enable(self._h, 1 if on else 0))

    def profile_region_begin(self, kernel: str | int, stream: int = 0):
        """Open a caller-delimited profiling region on `stream` (counted under `kernel`,
        e.g. "gather" around an RCCL gatherv this process enqueues); no-op unless profiling
        is on."""
        k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
        _check("sv_profile_region_begin", self.lib.sv_profile_region_begin(self._h, k, stream or None))

    def profile_region_end(self, stream: int = 0):
        _check("sv_profile_region_end", self.lib.sv_profile_region_end(self._h, stream or None))

    def profile_reset(self):
        _check("sv_profile_reset", self.lib.sv_profile_reset(self._h))

    def profile_read(self, kernel: str | int) -> tuple[float, int]:
        k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
        ms = ctypes.c_double()
        n = ctypes.c_longlong()
        _check("sv_profile_read", self.lib.sv_profile_read(self._h, k, ctypes.byref(ms),
                                                           ctypes.byref(n)))
        return ms.value, n.value


def multi_gpu_batch(engines, left, right, min_disp: int, num_disp: int, win: int,
                    min_depth: float, max_depth: float, min_disp_global=None, cost="sad"):
    """create_depth_map over a stack of frames (depth_map.py:837-946, once per frame),
    frame-sharded over the devices of `engines` from this one process (sv_multi_gpu_batch:
    one host thread + stream per device, contiguous shards).  left/right: F x H x W gray or
    F x H x W x 3 BGR uint8.  Returns (depth_final, disparity, depth_normalized), F x H x W."""
    engines = list(engines)
    if not engines:
        raise ValueError("no engines")
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    if left.shape != right.shape or left.ndim not in (3, 4) or (left.ndim == 4 and left.shape[3] != 3):
        raise ValueError(f"expected matching F x H x W (x 3) stacks, got {left.shape} / {right.shape}")
    F, H, W = left.shape[:3]
    C = 3 if left.ndim == 4 else 1
    mdg = min_disp if min_disp_global is None else min_disp_global
    depth = np.empty((F, H, W), np.float32)
    disp = np.empty((F, H, W), np.float32)
    norm = np.empty((F, H, W), np.uint8)
    hs = (_vp * len(engines))(*[e._h for e in engines])
    lib = engines[0].lib
    _check("sv_multi_gpu_batch", lib.sv_multi_gpu_batch(
        hs, len(engines), left, right, F, H, W, C, int(min_disp), int(num_disp), int(win),
        _cost(cost), np.float32(min_depth), np.float32(max_depth),
        np.float32(float(max_depth) - float(min_depth)), np.float32(mdg), depth, disp, norm))
    return depth, disp, norm


def _handles(items):
    items = list(items)
    return (_vp * len(items))(*[getattr(x, "_h", x) for x in items])


def _ptrs(values):
    values = [int(v) for v in values]
    return (_vp * len(values))(*values)


def multi_gpu_dev(engines, comms, shard: int, inputs: int, left, right, n_frames, H: int, W: int,
                  pitch: int, frame_stride: int, min_disp: int, num_disp: int, win: int, out: MapOut,
                  cost="sad"):
    """sv_multi_gpu_dev: one process driving the contexts of `engines` (SHARD_FRAMES: C4,
    SHARD_ROWS: C5 with INPUTS_RESIDENT / INPUTS_SCATTER / INPUTS_HOST), the root's outputs
    selected by `out` (:func:`map_out`).  `comms`: Communicator list (rank k on engines[k]'s
    device) or None (peer copies).  Enqueue only: synchronize engines[0] before reading."""
    engines = list(engines)
    nd = len(engines)
    lib = engines[0].lib
    ch = None if comms is None else _handles([c.handle for c in comms])
    nf = (_c_int * nd)(*[int(v) for v in n_frames]) if n_frames is not None else None
    _check("sv_multi_gpu_dev", lib.sv_multi_gpu_dev(
        _handles(engines), ch, nd, int(shard), int(inputs), _ptrs(left), _ptrs(right), nf, H, W, pitch,
        int(frame_stride), int(min_disp), int(num_disp), int(win), _cost(cost), ctypes.byref(out)))


def _full_out(min_depth, max_depth, min_disp, min_disp_global, d_depth, d_disp, d_norm) -> MapOut:
    mdg = min_disp if min_disp_global is None else min_disp_global
    return map_out(POST_DEPTH, d_disp, d_depth, d_norm, min_depth=min_depth, max_depth=max_depth,
                   min_disp_global=mdg)


def multi_gpu_depth_map_dev(engines, comms, d_left, d_right, n_frames, H: int, W: int, pitch: int,
                            frame_stride: int, min_disp: int, num_disp: int, win: int,
                            min_depth: float, max_depth: float, d_depth: int, d_disp: int,
                            d_norm: int, cost="sad", min_disp_global=None):
    """C4 on device-resident frames from ONE process: engine k runs create_depth_map over its
    n_frames[k] frames (its own device), and every output frame ends up on engines[0]'s device
    (d_depth/d_disp/d_norm, context order): the peers' int16 x16 medians cross over RCCL
    (`comms`) or peer copies (None), 2 B/px, and engines[0] expands them.  Enqueue only."""
    multi_gpu_dev(engines, comms, SHARD_FRAMES, INPUTS_RESIDENT, d_left, d_right, n_frames, H, W, pitch,
                  frame_stride, min_disp, num_disp, win,
                  _full_out(min_depth, max_depth, min_disp, min_disp_global, d_depth, d_disp, d_norm), cost)


MAP_M16, MAP_D8 = 1, 2   # SV_MAP_M16 / SV_MAP_D8
_MAP_FORMATS = {"m16": MAP_M16, "i16": MAP_M16, "d8": MAP_D8, "u8": MAP_D8}


def _map_format(fmt) -> int:
    if isinstance(fmt, str):
        if fmt not in _MAP_FORMATS:
            raise ValueError(f"map format must be one of {sorted(_MAP_FORMATS)}, got {fmt!r}")
        return _MAP_FORMATS[fmt]
    return int(fmt)


def _map_out(d_map: int, fmt) -> MapOut:
    f = _map_format(fmt)
    if f not in (MAP_M16, MAP_D8):
        raise ValueError(f"map format must be m16 or d8, got {fmt!r}")
    return map_out(POST_NONE, med16=d_map if f == MAP_M16 else 0, d8=d_map if f == MAP_D8 else 0)


def multi_gpu_m16_dev(engines, comms, d_left, d_right, n_frames, H: int, W: int, pitch: int,
                      frame_stride: int, min_disp: int, num_disp: int, win: int, d_med16: int,
                      cost="sad"):
    """C4 gather-only with int16 x16 maps (multi_gpu_map_dev with fmt "m16")."""
    multi_gpu_map_dev(engines, comms, d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp,
                      num_disp, win, d_med16, "m16", cost)


def multi_gpu_map_dev(engines, comms, d_left, d_right, n_frames, H: int, W: int, pitch: int,
                      frame_stride: int, min_disp: int, num_disp: int, win: int, d_map: int,
                      fmt="m16", cost="sad"):
    """C4 gather-only: engine k computes disparity + median over its n_frames[k] frames and
    only the median maps are gathered into d_map on engines[0]'s device (context order):
    ``fmt="m16"`` int16 x16 (2 B/px), ``"d8"`` u8 disparity indices median/16 - (min_disp - 1)
    (1 B/px; integer costs, num_disp <= 255).  Enqueue only."""
    multi_gpu_dev(engines, comms, SHARD_FRAMES, INPUTS_RESIDENT, d_left, d_right, n_frames, H, W, pitch,
                  frame_stride, min_disp, num_disp, win, _map_out(d_map, fmt), cost)


def _rows_inputs(scatter) -> int:
    if scatter in (False, None, 0):
        return INPUTS_RESIDENT
    if scatter in (True, 1, "scatter"):
        return INPUTS_SCATTER
    if scatter == "host":
        return INPUTS_HOST
    raise ValueError(f"scatter must be False, True/'scatter' or 'host', got {scatter!r}")


def _rows_ptrs(d_left, d_right, inputs):
    if inputs == INPUTS_RESIDENT:
        return d_left, d_right
    # one frame: a device pointer on the root (scatter) or a host array / pointer (host)
    def one(x):
        if isinstance(x, np.ndarray):
            if x.dtype != np.uint8 or not x.flags["C_CONTIGUOUS"]:
                raise ValueError("host frames must be C-contiguous uint8")
            return x.ctypes.data
        return int(x)
    return [one(d_left)], [one(d_right)]


def depth_map_rows_map(engines, comms, d_left, d_right, H: int, W: int, pitch: int, min_disp: int,
                       num_disp: int, win: int, d_map: int, fmt="m16", scatter=False, cost="sad"):
    """C5 gather-only: one frame row-tiled over the engines; the root (engines[0]) receives
    only the full-frame median map (int16 x16 or u8 indices) in d_map and expands nothing.
    ``scatter``: False — lists with the full frame on every engine's device; True — the root's
    device frame (one pointer each), the other engines receive just their bands' input rows
    over xGMI; "host" — a host frame (uint8 arrays, page-locked for overlap), every engine
    uploads its own band's rows over its own PCIe link.  Enqueue only."""
    inputs = _rows_inputs(scatter)
    L, R = _rows_ptrs(d_left, d_right, inputs)
    multi_gpu_dev(engines, comms, SHARD_ROWS, inputs, L, R, None, H, W, pitch, 0, min_disp, num_disp, win,
                  _map_out(d_map, fmt), cost)


def depth_map_rows_multi(engines, comms, d_left, d_right, H: int, W: int, pitch: int, min_disp: int,
                         num_disp: int, win: int, min_depth: float, max_depth: float, d_depth: int,
                         d_disp: int, d_norm: int, cost="sad", min_disp_global=None, scatter=False):
    """C5 from ONE process: one frame row-tiled over the engines, bands gathered to
    engines[0]'s device into the full-frame outputs (inputs as :func:`depth_map_rows_map`).
    Enqueue only."""
    inputs = _rows_inputs(scatter)
    L, R = _rows_ptrs(d_left, d_right, inputs)
    multi_gpu_dev(engines, comms, SHARD_ROWS, inputs, L, R, None, H, W, pitch, 0, min_disp, num_disp, win,
                  _full_out(min_depth, max_depth, min_disp, min_disp_global, d_depth, d_disp, d_norm), cost)


def depth_map_rows_scatter(engines, comms, d_left: int, d_right: int, H: int, W: int, pitch: int,
                           min_disp: int, num_disp: int, win: int, min_depth: float, max_depth: float,
                           d_depth: int, d_disp: int, d_norm: int, cost="sad", min_disp_global=None):
    """C5 with the frame resident on engines[0]'s device only: each other engine receives just
    the input rows of its band (+ halos, :func:`band_rows_in`), computes its band, and the bands
    are gathered back into the full-frame outputs on engines[0]'s device.  Enqueue only."""
    depth_map_rows_multi(engines, comms, d_left, d_right, H, W, pitch, min_disp, num_disp, win, min_depth,
                         max_depth, d_depth, d_disp, d_norm, cost, min_disp_global, scatter=True)


def band_rows_in(H: int, rank: int, world: int, win: int, cost="sad") -> dict:
    """Row bands of a `world`-way tiling (sv_band_rows_in): output rows r0:r1, disparity rows
    h0:h1 (with the median halo) and the input rows in0:in1 the band's kernels read."""
    out = (_c_int * 6)()
    _check("sv_band_rows_in", load_library().sv_band_rows_in(H, rank, world, win, _cost(cost), out))
    return dict(zip(("r0", "r1", "h0", "h1", "in0", "in1"), list(out)))


HOST_STAGES = ("prepare", "stage_issue", "wait_first", "expand", "wait_rest", "total")


def host_profile(enable: bool | None = None, reset: bool = False) -> dict:
    """Host-side stage timings of the host-buffer entry points (sv_host_profile_*):
    ``enable`` switches collection on/off; returns the mean ms per call of each stage in
    HOST_STAGES since the last reset (and resets when asked)."""
    lib = load_library()
    if enable is not None:
        lib.sv_host_profile_enable(int(bool(enable)))
    ms = (ctypes.c_double * 6)()
    n = ctypes.c_longlong()
    _check("sv_host_profile_read", lib.sv_host_profile_read(ms, ctypes.byref(n), int(reset)))
    calls = n.value
    return {"calls": calls, **{k: (ms[i] / calls if calls else None) for i, k in enumerate(HOST_STAGES)}}


class Communicator:
    """An RCCL communicator of libsvhip (sv_comm_*): rank `rank` of `nranks` on `device`."""

    def __init__(self, handle, lib):
        self._h = handle
        self.lib = lib
        r, n, d = _c_int(), _c_int(), _c_int()
        _check("sv_comm_rank", lib.sv_comm_rank(handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)))
        self.rank, self.nranks, self.device = r.value, n.value, d.value

    @staticmethod
    def available() -> bool:
        return bool(load_library().sv_comm_available())

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        _check("sv_comm_unique_id", load_library().sv_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def init_rank(cls, device: int, nranks: int, rank: int, uid: bytes, timeout: float = 120.0) -> "Communicator":
        """ncclCommInitRank, non-blocking with a deadline: if a peer fails during bootstrap
        this rank gets an error after `timeout` seconds (the half-built communicator aborted)
        instead of blocking forever."""
        lib = load_library()
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        h = _vp()
        _check("sv_comm_init_rank", lib.sv_comm_init_rank(device, nranks, rank, uid, float(timeout),
                                                          ctypes.byref(h)))
        return cls(h, lib)

    @classmethod
    def init_all(cls, devices) -> list["Communicator"]:
        lib = load_library()
        devices = [int(d) for d in devices]
        hs = (_vp * len(devices))()
        _check("sv_comm_init_all", lib.sv_comm_init_all(len(devices), (_c_int * len(devices))(*devices), hs))
        return [cls(_vp(h), lib) for h in hs]

    @property
    def handle(self):
        return self._h

    def close(self):
        for sets in getattr(self, "_recycle", {}).values():
            for arrs in sets:
                self._unregister(arrs)
        self._recycle = {}
        if getattr(self, "_h", None):
            self.lib.sv_comm_destroy(self._h)
            self._h = None

    def barrier(self):
        _check("sv_comm_barrier", self.lib.sv_comm_barrier(self._h))

    def allreduce_max(self, value: float) -> float:
        v = ctypes.c_double(float(value))
        _check("sv_comm_allreduce_max_f64", self.lib.sv_comm_allreduce_max_f64(self._h, ctypes.byref(v)))
        return v.value

    def gatherv(self, d_send: int, send_bytes: int, d_recv: int, offsets, sizes, root: int = 0,
                stream: int = 0):
        n = self.nranks
        off = (ctypes.c_uint64 * n)(*[int(v) for v in offsets])
        sz = (ctypes.c_uint64 * n)(*[int(v) for v in sizes])
        _check("sv_comm_gatherv", self.lib.sv_comm_gatherv(self._h, d_send or None, int(send_bytes),
                                                          d_recv or None, off, sz, int(root),
                                                          stream or None))

    def scatterv(self, d_send: int, offsets, sizes, d_recv: int, recv_bytes: int, root: int = 0,
                 stream: int = 0):
        n = self.nranks
        off = (ctypes.c_uint64 * n)(*[int(v) for v in offsets]) if offsets is not None else None
        sz = (ctypes.c_uint64 * n)(*[int(v) for v in sizes]) if sizes is not None else None
        _check("sv_comm_scatterv", self.lib.sv_comm_scatterv(self._h, d_send or None, off, sz,
                                                            d_recv or None, int(recv_bytes), int(root),
                                                            stream or None))

    def synchronize(self):
        _check("sv_comm_synchronize", self.lib.sv_comm_synchronize(self._h))

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def start_warmup(fn, name: str = "sv-warmup") -> threading.Event:
    """Run `fn` (engine creation + one pass of the kernels a drop-in will use, at its
    processing size) on a daemon thread; returns an Event set when it has finished.  The
    drop-in modules call this at import so the first frame of the reference's loop does not
    pay HIP initialisation, code-object loading and staging allocation inside its 0.5 s
    budget (fused_depth_map.py:2671).  Without a GPU (or library) the thread ends silently:
    the first real call then raises EngineUnavailable loudly.  The warm-up initialises the GPU
    in the importing process: a host application that forks or execs worker processes after
    importing the drop-ins sets SV_WARMUP_AT_IMPORT=0 (the first call then pays the start-up).
    Interpreter exit waits for an unfinished warm-up (at most 30 s)."""
    done = threading.Event()

    def run():
        try:
            fn()
        except Exception:  # no GPU here, or a failing warm-up: the real call reports it
            pass
        finally:
            done.set()

    t = threading.Thread(target=run, name=name, daemon=True)
    t.start()
    # a short-lived script must not tear the interpreter down while the warm-up is still
    # inside a HIP call: wait for it at exit (bounded)
    atexit.register(done.wait, 30.0)
    return done


_engines: dict[int, Engine] = {}
_engines_lock = threading.Lock()


def get_engine(device: int | None = None) -> Engine:
    """Process-wide cached Engine per device (SV_DEVICE env var picks the default)."""
    if device is None:
        device = int(os.environ.get("SV_DEVICE", "0"))
    with _engines_lock:
        eng = _engines.get(device)
        if eng is None:
            eng = Engine(device)
            _engines[device] = eng
        return eng
