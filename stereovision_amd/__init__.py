"""stereovision_amd — MI355X-native (gfx950) stereo-disparity engine.

A drop-in for the disparity hot path of AlexGr5/StereoVision's ``depth_map.py`` and
``fused_depth_map.py``: the same Python entry points, computed by hand-written HIP kernels
through a C ABI (``include/stereovision_amd.h``, ``lib/libsvhip.so``).  See DESIGN.md.
"""
from .engine import (COSTS, Engine, EngineUnavailable, SVError, device_count, get_engine,
                     load_library, plan)

__all__ = ["COSTS", "Engine", "EngineUnavailable", "SVError", "device_count", "get_engine",
           "load_library", "plan"]
