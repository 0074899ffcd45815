#!/usr/bin/env python3
"""Regenerates tests/golden/golden_v1.npz from the NumPy oracle (oracle/sv_oracle.py).

The reference holds no fixtures or golden vectors for this path, so
these are the oracle's own outputs on small seeded synthetic pairs: they pin the oracle
against drift and give the GPU tests a committed target.  Inputs are stored alongside.
Usage: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import sv_oracle as O  # noqa: E402
from stereovision_amd.synthetic import stereo_pair, to_bgr  # noqa: E402

CASES = [  # name, H, W, min_disp, num_disp, win, seed
    ("a", 32, 96, 0, 16, 5, 1),
    ("b", 40, 160, 0, 32, 9, 2),
    ("c", 24, 120, -8, 48, 7, 3),
    ("d", 36, 200, 4, 64, 11, 4),
]


def main():
    out = {}
    for name, H, W, mn, D, win, seed in CASES:
        L, R, _ = stereo_pair(H, W, max(16, D), seed, max(0, mn))
        out[f"{name}_left"] = L
        out[f"{name}_right"] = R
        out[f"{name}_params"] = np.array([mn, D, win], np.int32)
        for cost, cname in ((O.COST_SAD, "sad"), (O.COST_SSD, "ssd"), (O.COST_HOG, "hog")):
            out[f"{name}_d16_{cname}"] = O.disparity16(L, R, mn, D, win, cost)
        disp = O.disparity_f32(out[f"{name}_d16_sad"])
        out[f"{name}_disparity"] = disp
        df, dn = O.depth_post(disp, 0.3, 2.0, mn)
        out[f"{name}_depth_final"] = df
        out[f"{name}_depth_norm"] = dn
        sn, su, sc = O.scaled_post(disp, mn, D)
        out[f"{name}_scaled_norm"] = sn
        out[f"{name}_scaled_conf"] = sc
        out[f"{name}_harris"] = O.harris(L)
        out[f"{name}_hog"] = O.hog_hist(L, win)
    bgr = np.random.default_rng(9).integers(0, 256, (17, 23, 3), dtype=np.uint8)
    out["gray_bgr"] = bgr
    out["gray_out"] = O.bgr_to_gray(bgr)
    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
