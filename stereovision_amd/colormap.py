"""Display colormaps for the drop-in entry points (NOT part of the parity contract).

The reference colours its maps with ``cv2.applyColorMap`` (TURBO at depth_map.py:937,
JET at fused_depth_map.py:1013) and stamps text with ``cv2.putText``
(fused_depth_map.py:1016-1018).  When ``cv2`` is importable those exact calls are used.
Otherwise a built-in LUT is used: Turbo from its published polynomial approximation and
the classic piecewise-linear Jet; these are visually equivalent but not byte-identical
to OpenCV's tables, which is why colormaps are excluded from parity.
"""
from __future__ import annotations

import numpy as np

try:  # optional, display only
    import cv2  # type: ignore
except Exception:  # pragma: no cover - cv2 is absent in this image
    cv2 = None


def _turbo_lut() -> np.ndarray:
    x = np.linspace(0.0, 1.0, 256)
    r = 0.13572138 + x * (4.61539260 + x * (-42.66032258 + x * (132.13108234 + x * (-152.94239396 + x * 59.28637943))))
    g = 0.09140261 + x * (2.19418839 + x * (4.84296658 + x * (-14.18503333 + x * (4.27729857 + x * 2.82956604))))
    b = 0.10667330 + x * (12.64194608 + x * (-60.58204836 + x * (110.36276771 + x * (-89.90310912 + x * 27.34824973))))
    rgb = np.clip(np.stack([r, g, b], 1), 0.0, 1.0)
    return np.round(rgb[:, ::-1] * 255.0).astype(np.uint8)   # BGR


def _jet_lut() -> np.ndarray:
    x = np.linspace(0.0, 1.0, 256)
    r = np.clip(1.5 - np.abs(4.0 * x - 3.0), 0.0, 1.0)
    g = np.clip(1.5 - np.abs(4.0 * x - 2.0), 0.0, 1.0)
    b = np.clip(1.5 - np.abs(4.0 * x - 1.0), 0.0, 1.0)
    return np.round(np.stack([b, g, r], 1) * 255.0).astype(np.uint8)   # BGR


_LUTS = {"turbo": _turbo_lut(), "jet": _jet_lut()}
_TABLES: dict = {}


def table(name: str) -> np.ndarray:
    """The 256 x 3 BGR table of colormap `name` that the GPU epilogue applies: cv2's own
    (read back through cv2.applyColorMap on the 256 gray levels, byte-exact with the
    reference) when cv2 is importable, the built-in LUT otherwise."""
    t = _TABLES.get(name)
    if t is None:
        if cv2 is not None:
            code = cv2.COLORMAP_TURBO if name == "turbo" else cv2.COLORMAP_JET
            t = np.ascontiguousarray(cv2.applyColorMap(np.arange(256, dtype=np.uint8).reshape(256, 1),
                                                       code).reshape(256, 3))
        else:
            t = _LUTS[name]
        _TABLES[name] = t
    return t


def apply(u8: np.ndarray, name: str) -> np.ndarray:
    """HxW uint8 -> HxWx3 BGR uint8."""
    u8 = np.ascontiguousarray(u8, np.uint8)
    if cv2 is not None:
        code = cv2.COLORMAP_TURBO if name == "turbo" else cv2.COLORMAP_JET
        return cv2.applyColorMap(u8, code)
    return _LUTS[name][u8]


def put_text(img: np.ndarray, text: str, org=(10, 30)) -> np.ndarray:
    """cv2.putText(img, text, org, FONT_HERSHEY_COMPLEX, 0.7, white, 2) when cv2 exists."""
    if cv2 is not None:
        cv2.putText(img, text, org, cv2.FONT_HERSHEY_COMPLEX, 0.7, (255, 255, 255), 2)
    return img
