#!/usr/bin/env python3
"""HOG window-histogram diagnostics on the GPU box: the engine's histograms against the
oracle's at a given size / window, mismatches summarised by position (row, column, column
within a 496-column wave, lane, row within a 32-row strip) and bin.

Usage: python tools/hog_diag.py H W WIN [synthetic|synthetic_r|random] [SEED]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import sv_oracle as O  # noqa: E402
from stereovision_amd.engine import get_engine  # noqa: E402
from stereovision_amd.synthetic import stereo_pair  # noqa: E402


def main():
    H, W, win = (int(v) for v in sys.argv[1:4])
    kind = sys.argv[4] if len(sys.argv) > 4 else "synthetic"
    seed = int(sys.argv[5]) if len(sys.argv) > 5 else 55
    if kind in ("synthetic", "synthetic_r"):
        L, R, _ = stereo_pair(H, W, 256, seed=seed)
        g = L if kind == "synthetic" else R
    else:
        g = np.random.default_rng(seed).integers(0, 256, (H, W), dtype=np.uint8)
    got = get_engine(0).hog_hist(g, win)
    exp = O.hog_hist(g, win)
    bad = np.argwhere(got != exp)
    print(f"{H}x{W} win {win} {kind}: {len(bad)} mismatching entries of {got.size}", flush=True)
    if len(bad):
        b, y, x = bad[:, 0], bad[:, 1], bad[:, 2]
        xr = x % 496
        print("bins", np.bincount(b, minlength=9).tolist())
        print("rows", np.unique(y)[:40].tolist(), "... n", len(np.unique(y)))
        print("cols", np.unique(x)[:40].tolist(), "... n", len(np.unique(x)))
        print("col in wave", np.unique(xr)[:60].tolist())
        print("lane", np.unique(xr // 8 + 1).tolist())
        print("row in strip", np.unique(y % 32).tolist())
        for i in range(min(8, len(bad))):
            print("  at", bad[i].tolist(), "got", int(got[tuple(bad[i])]), "exp", int(exp[tuple(bad[i])]))


if __name__ == "__main__":
    main()


def disparity_dump(path, H=2160, W=3840, D=256, win=15, seed=55):
    """Child entry: the engine's HOG disparity of the synthetic pair, saved to `path` (.npy)."""
    L, R, _ = stereo_pair(H, W, D, seed=seed)
    np.save(path, get_engine(0).disparity(L, R, 0, D, win, "hog"))
