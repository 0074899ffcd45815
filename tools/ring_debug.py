#!/usr/bin/env python3
"""Mismatch locator for the SAD kernels (GPU box; a debugging aid): runs one case and prints
where the engine and the C oracle differ.  Usage: python tools/ring_debug.py D win min_disp pattern"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sv_oracle_c as C  # noqa: E402
from stereovision_amd.engine import get_engine  # noqa: E402


def pattern(name, H, W, seed=0):
    yy, xx = np.mgrid[0:H, 0:W]
    if name == "columns":
        L = np.tile(np.array([0, 255], np.uint8), (H, W // 2))
        return L, np.roll(L, 1, axis=1)
    if name == "checker":
        c = (((yy + xx) & 1) * 255).astype(np.uint8)
        return c, 255 - c
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    return L, np.roll(L, -7, axis=1)


def main():
    D, win, md = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    name = sys.argv[4] if len(sys.argv) > 4 else "random"
    H, W = (int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else (29, 448)
    L, R = pattern(name, H, W)
    eng = get_engine(0)
    got = eng.disparity(L, R, md, D, win, "sad")
    exp = C.disparity16(L, R, md, D, win, 0)
    bad = np.argwhere(got != exp)
    print(f"D={D} win={win} min_disp={md} {name} {H}x{W}: {len(bad)} mismatches")
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    print("rows", rows[:40])
    print("cols", cols[:80], "..." if len(cols) > 80 else "")
    for y, x in bad[:24]:
        print(f"  ({y},{x}) got {got[y, x] / 16} exp {exp[y, x] / 16}")


if __name__ == "__main__":
    main()
