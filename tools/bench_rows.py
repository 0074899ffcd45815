#!/usr/bin/env python3
"""Per-row measurements of SURVEY.md §8(f) (rectification, calibration maps, resize,
occlusion statistics, percentile calibration, SGBM): device time from HIP events around
the kernels (inputs resident in HBM), the algorithmic-bytes HBM roofline of each, the
host-API wall time (PCIe-inclusive, one call as the reference makes it), and the CPU
restatement timed beside it on this host (the oracle modules, which for the reductions
are the reference's own NumPy code).  Prints one JSON line per row; --out writes them.

Run on the GPU box: python tools/bench_rows.py --out gpurun_out/rows.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime: torch first)
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from stereovision_amd import calib, fusion  # noqa: E402
from stereovision_amd.engine import get_engine  # noqa: E402
from stereovision_amd.synthetic import stereo_pair, synthetic_calibration, to_bgr  # noqa: E402

HBM_PEAK = 8000.0


def dev_time(eng, kernel: str, fn, reps: int = 20):
    fn()
    eng.synchronize()
    eng.profile_reset()
    eng.profile(True)
    for _ in range(reps):
        fn()
    eng.synchronize()
    eng.profile(False)
    ms, n = eng.profile_read(kernel)
    return ms / max(n, 1) * 1e3 * (n / reps)      # us per call (all launches of the call)


def wall(fn, reps: int = 5):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps * 1e6


def cpu(fn, budget: float = 3.0):
    t0 = time.perf_counter()
    n = 0
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= budget or n >= 20:
            return dt / n * 1e6


def roof(bytes_per_call, us):
    gbs = bytes_per_call / (us * 1e-6) / 1e9
    return {"bytes": int(bytes_per_call), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu-budget", type=float, default=3.0)
    args = ap.parse_args()
    import sv_fusion_oracle as FO
    import sv_rectify_oracle as RO
    import sv_sgbm_oracle as SG

    eng = get_engine(0)
    H, W = 1080, 1920
    rows = []

    def emit(d):
        rows.append(d)
        print(json.dumps(d), flush=True)

    # ---- rectification: remap BGR -> rectified gray, both cameras (row 1) ------------------
    from stereovision_amd.rectify import StereoRectifier
    c = synthetic_calibration(W, H)
    R1, R2, P1, P2, _, _, _ = calib.stereo_rectify(c["mtx_left"], c["dist_left"], c["mtx_right"],
                                                   c["dist_right"], (W, H), c["R"], c["T"], alpha=0)
    rect = StereoRectifier.from_calibration(c["mtx_left"], c["dist_left"], R1, P1, c["mtx_right"],
                                            c["dist_right"], R2, P2, (W, H), eng)
    L, R, _ = stereo_pair(H, W, 128, seed=1)
    bl, br = to_bgr(L), to_bgr(R)
    d_src = eng.upload("rows_src", np.stack([bl, br]))
    d_dst = eng.scratch("rows_dst", 2 * H * W)
    m1l, m2l, m1r, m2r, _, _ = rect.device_maps

    def remap_pair():
        eng.remap_dev(d_src, H, W, 3, 3 * W, m1l, m2l, H, W, d_dst, W, gray_out=True)
        eng.remap_dev(d_src + 3 * H * W, H, W, 3, 3 * W, m1r, m2r, H, W, d_dst + H * W, W, gray_out=True)
    us = dev_time(eng, "remap", remap_pair)
    lm1, lm2, rm1, rm2 = rect.host_maps()
    emit({"row": "rectify pair (remap INTER_LINEAR + BGR2GRAY, 2 x 1920x1080)", "gpu_us": round(us, 1),
          "roofline": roof(2 * 10 * H * W, us),
          "host_api_us": round(wall(lambda: rect.rectify(bl, br)), 1),
          "cpu_us": round(cpu(lambda: (RO.remap_gray(bl, lm1, lm2), RO.remap_gray(br, rm1, rm2)),
                              args.cpu_budget), 1),
          "cpu_kind": "port (NumPy oracle, 1 thread)"})

    # ---- calibration maps (row 2) ---------------------------------------------------------
    d_m1 = eng.scratch("rows_m1", 4 * H * W)
    d_m2 = eng.scratch("rows_m2", 2 * H * W)
    us = dev_time(eng, "undistort", lambda: eng.init_undistort_rectify_map_dev(
        c["mtx_left"], c["dist_left"], R1, P1, W, H, d_m1, d_m2))
    emit({"row": "initUndistortRectifyMap CV_16SC2 (1920x1080, f64)", "gpu_us": round(us, 1),
          "roofline": roof(6 * H * W, us),
          "host_api_us": round(wall(lambda: eng.init_undistort_rectify_map(c["mtx_left"], c["dist_left"], R1, P1, W, H)), 1),
          "cpu_us": round(cpu(lambda: RO.undistort_rectify_map(c["mtx_left"], c["dist_left"], R1, P1, W, H),
                              args.cpu_budget), 1),
          "cpu_kind": "port (NumPy oracle, 1 thread)",
          "stereo_rectify_host_us": round(wall(lambda: calib.stereo_rectify(
              c["mtx_left"], c["dist_left"], c["mtx_right"], c["dist_right"], (W, H), c["R"], c["T"], alpha=0)), 1)})

    # ---- resize to the processing scale (row 1, fused app) ----------------------------------
    pw, ph = int(W * 0.33), int(H * 0.33)
    d_rs = eng.scratch("rows_rs", 3 * pw * ph)
    us = dev_time(eng, "resize", lambda: eng.resize_dev(d_src, H, W, 3, 3 * W, d_rs, ph, pw, 3 * pw))
    emit({"row": f"resize INTER_LINEAR 1920x1080 BGR -> {pw}x{ph}", "gpu_us": round(us, 1),
          "roofline": roof(3 * (ph * pw) * 5, us),
          "host_api_us": round(wall(lambda: eng.resize(bl, pw, ph)), 1),
          "cpu_us": round(cpu(lambda: RO.resize_linear(bl, pw, ph), args.cpu_budget), 1),
          "cpu_kind": "port (NumPy oracle, 1 thread)"})

    # ---- occlusion statistics (row 4) ---------------------------------------------------------
    nb = max(1, H // 48) * max(1, W // 48)
    d_st = eng.scratch("rows_st", 4 * 2 * (2 * nb + 256))
    us = dev_time(eng, "stats", lambda: eng.frame_stats_dev(d_dst, d_dst + H * W, H, W, 1, W, d_st,
                                                             d_st + 8 * nb, d_st + 16 * nb))
    emit({"row": "detect_camera_occlusion statistics (pair 1920x1080 gray)", "gpu_us": round(us, 1),
          "roofline": roof(2 * H * W, us),
          "host_api_us": round(wall(lambda: fusion.detect_camera_occlusion(bl, br)), 1),
          "cpu_us": round(cpu(lambda: FO.detect_camera_occlusion(bl, br), args.cpu_budget), 1),
          "cpu_kind": "reference NumPy code (cv2 calls restated), 1 thread"})

    # ---- percentile calibration (row 4) ---------------------------------------------------------
    rng = np.random.default_rng(0)
    disp = (rng.integers(0, 128, (H, W)) + rng.random((H, W))).astype(np.float32)
    conf = (rng.random((H, W)) > 0.2).astype(np.float32)
    midas = (rng.random((H, W)) * 255).astype(np.float32)
    emit({"row": "calibrate_midas_to_stereo (1920x1080 f32, reliable branch)",
          "host_api_us": round(wall(lambda: fusion.calibrate_midas_to_stereo(midas, disp, conf)), 1),
          "cpu_us": round(cpu(lambda: FO.calibrate_midas_to_stereo(midas, disp, conf), args.cpu_budget), 1),
          "cpu_kind": "reference NumPy code, 1 thread",
          "select_pass_gpu_us": round(dev_time(eng, "select", lambda: eng.select_count(
              eng.upload("rows_d", disp), H * W, 1)), 1),
          "select_pass_roofline": None})
    rows[-1]["select_pass_roofline"] = roof(4 * H * W, rows[-1]["select_pass_gpu_us"])
    emit({"row": "normalize_to_stereo_range (1920x1080 f32)",
          "host_api_us": round(wall(lambda: fusion.normalize_to_stereo_range(midas, disp)), 1),
          "cpu_us": round(cpu(lambda: FO.normalize_to_stereo_range(midas, disp), args.cpu_budget), 1),
          "cpu_kind": "reference NumPy code, 1 thread"})

    # ---- SGBM-3WAY mode (row 3) ---------------------------------------------------------------
    for D, win in ((128, 9), (320, 7)):
        d_l = eng.upload("rows_l", L)
        d_r = eng.upload("rows_r", R)
        d_o = eng.scratch("rows_o", 2 * H * W)
        us = dev_time(eng, "sgbm", lambda: eng.sgbm_dev(d_l, d_r, H, W, W, 0, D, win, d_o, W), reps=5)
        sp = dev_time(eng, "speckle", lambda: eng.sgbm_dev(d_l, d_r, H, W, W, 0, D, win, d_o, W), reps=5)
        rows_cpu = 32
        t_strip = cpu(lambda: SG.sgbm(L[:rows_cpu], R[:rows_cpu], 0, D, win), args.cpu_budget)
        emit({"row": f"SGBM-3WAY 1920x1080 D={D} win={win}", "gpu_us": round(us + sp, 1),
              "fps": round(1e6 / (us + sp), 1),
              "cpu_us": round(t_strip * H / rows_cpu, 1),
              "cpu_kind": f"port (NumPy oracle on {rows_cpu}-row strips, scaled to the frame), 1 thread"})
    rect.close()
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
