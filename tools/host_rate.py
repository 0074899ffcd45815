#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer drop-in path: BGR frames in host
memory -> sv_depth_map (pinned staging, H2D, gray, disparity, median+post, D2H) -> NumPy
outputs, one call per frame as depth_map.create_depth_map does.  Not the bench metric."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereovision_amd.engine import get_engine  # noqa: E402
from stereovision_amd.synthetic import stereo_pair, to_bgr  # noqa: E402


def main():
    H, W, D, win = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (1080, 1920, 128, 9)))
    frames = []
    for s in range(4):
        L, R, _ = stereo_pair(H, W, D, seed=s)
        frames.append((to_bgr(L), to_bgr(R)))
    eng = get_engine(0)
    for i in range(5):
        eng.depth_map(*frames[i % 4], 0, D, win, 0.3, 2.0)
    n = 100
    t0 = time.perf_counter()
    for i in range(n):
        eng.depth_map(*frames[i % 4], 0, D, win, 0.3, 2.0)
    dt = time.perf_counter() - t0
    print(json.dumps({"path": "host BGR -> sv_depth_map -> host (PCIe-inclusive)",
                      "size": f"{W}x{H}", "D": D, "win": win, "frames": n,
                      "frames_per_s": round(n / dt, 1), "ms_per_frame": round(dt * 1e3 / n, 3),
                      "bytes_per_frame_h2d": 2 * 3 * H * W, "bytes_per_frame_d2h": 9 * H * W}))


if __name__ == "__main__":
    main()
