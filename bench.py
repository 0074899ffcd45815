#!/usr/bin/env python3
"""bench.py — disparity frames/s of the MI355X engine (BASELINE.json metric).  No PyTorch.

Workload (BASELINE.json metric): 1920x1080 rectified synthetic pairs, D=128, 9x9 SAD
window, the whole device path of depth_map.create_depth_map per frame:
    disparity (k_match) -> medianBlur 5 + depth post (k_median_i16, fused)
Inputs are gray u8 pairs already resident in HBM (16 distinct frames per GPU, cycled);
outputs are depth f32, disparity f32 and depth u8 per frame.  One step = one batch of
--batch frame pairs (default 16) through sv_depth_map_batch_dev: one k_match and one
k_median_i16 launch over the batch (grid.z = frame).  --batch 1 = one call per frame.

Multi-GPU (frames mode = C4, weak scaling; rowtile mode = C5, strong scaling):
  * under `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` (the
    driver's launch; only the launcher is torch's): one process per GPU, RANK/WORLD_SIZE/
    LOCAL_RANK from the environment, barrier + max-over-ranks through RCCL
    (stereovision_amd.distributed: file rendezvous + sv_comm_* of libsvhip);
  * `python bench.py --gpus N` without a launcher: ONE process drives N devices
    (sv_multi_gpu_dev when gathering).
value = frames of all GPUs / max wall time of the timed region.

Extra JSON fields:
  roofline      k_match against the HBM roofline with SURVEY.md §8(d)'s algorithmic bytes
                (6 B/px: 2 u8 images read + the f32 disparity map); launch times from HIP
                events inside the timed region; `traffic` and `valu` from rocprofv3 PMC passes
                run live by this script on this box (separate --pmc passes, a child process
                each; --no-live-pmc skips them)
  host_path     the drop-in create_depth_map (BGR NumPy in -> NumPy out, one frame per call,
                PCIe-inclusive) and its pipelined form (several frames in flight)
  cpu_baseline  the C oracle (oracle/sv_oracle.c, OpenMP over every core of this process's
                affinity) on full frames
"""
from __future__ import annotations

import argparse
import csv
import faulthandler
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from stereovision_amd.engine import (POST_DEPTH, STAGE_MATCH, STAGE_MEDIAN, Communicator,  # noqa: E402
                                     Engine, depth_map_rows_map, depth_map_rows_multi,
                                     depth_map_rows_scatter, device_count, get_engine, map_out,
                                     multi_gpu_depth_map_dev, multi_gpu_map_dev)
from stereovision_amd.synthetic import stereo_batch, stereo_pair, synthetic_calibration, to_bgr  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
N_SIMD = 1024                        # 256 CU x 4 SIMD
VALU_ISSUE_PEAK = N_SIMD * 2.4e9 / 2   # one wave64 VALU instr per 2 cycles per SIMD


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """(cores this process may run on, os.cpu_count()): the affinity set, capped by a cgroup
    CPU quota when one is set (a GPU box's per-GPU CPU share)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            aff = max(1, min(aff, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return aff, os.cpu_count() or aff


# ---- CPU baseline (the oracle: test infrastructure, timed only here) ------------------------
def cpu_baseline_sgbm(H, W, D, win, seconds):
    """SGBM mode: the NumPy SGBM-3WAY oracle (single process) on horizontal strips of the
    frame (full width, the whole disparity range), scaled to frames/s by the strip share."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sv_sgbm_oracle as SG  # test infrastructure, used here only as the CPU baseline
    L, R = stereo_batch(1, H, W, D, seed=4242)
    rows = max(8, min(H, 64))
    n, t0 = 0, time.perf_counter()
    while True:
        y0 = (n * rows) % max(1, H - rows + 1)
        SG.sgbm(L[0, y0:y0 + rows], R[0, y0:y0 + rows], 0, D, win)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or n >= 50:
            break
    fps = n * rows / H / dt
    return {"value": round(fps, 4), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} strips of {rows}x{W} (D={D}, win={win}) of the NumPy SGBM-3WAY oracle "
                      f"in {dt:.1f} s, scaled by {rows}/{H} rows to frames/s; single process"}


def cpu_baseline(H, W, D, win, cost, seconds, harris=False):
    """The C oracle (the port of the engine's semantics; the reference's own CPU path is
    OpenCV StereoSGBM, not importable on this image) timed on this host: the whole app-1
    path per frame (+ the Harris response of the left frame for C2), OpenMP over all cores of
    the process's affinity; plus the single-thread rate of the same port."""
    if cost == "sgbm":
        return cpu_baseline_sgbm(H, W, D, win, seconds)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes
    import sv_oracle_c as C  # test infrastructure, used here only as the CPU baseline
    lib = C.lib()
    aff, ncpu = host_cores()
    L, R = stereo_batch(2, H, W, D, seed=4242)
    depth = np.empty((H, W), np.float32)
    disp = np.empty((H, W), np.float32)
    norm = np.empty((H, W), np.uint8)
    costi = {"sad": 0, "ssd": 1, "hog": 2}[cost]
    f32 = ctypes.c_float
    lib.svo_depth_map.argtypes = [C._u8p, C._u8p, C._i, C._i, C._i, C._i, C._i, C._i, f32, f32,
                                  f32, C._f32p, C._f32p, C._u8p, C._i]
    lib.svo_depth_map.restype = C._i

    def one(i, threads):
        lib.svo_depth_map(np.ascontiguousarray(L[i % 2]), np.ascontiguousarray(R[i % 2]), H, W,
                          0, D, win, costi, np.float32(0.3), np.float32(2.0),
                          np.float32(2.0 - 0.3), depth, disp, norm, threads)
        if harris:
            C.harris(np.ascontiguousarray(L[i % 2]))

    def rate(threads, budget, cap):
        one(0, threads)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            one(n, threads)
            n += 1
            dt = time.perf_counter() - t0
            if dt >= budget or n >= cap:
                return n, dt

    n, dt = rate(aff, seconds, 400)
    n1, dt1 = rate(1, max(1.0, seconds / 4), 20)
    # the NumPy oracle (BASELINE.md's planned single-process baseline), on strips of 64
    # output rows (+ the window's halo rows) of the same frame, scaled by the strip share
    import sv_oracle as NO  # test infrastructure, used here only as the CPU baseline
    r = win // 2
    rows, ns, t0 = 64, 0, time.perf_counter()
    while True:
        y0 = (ns * rows) % max(1, H - rows - 2 * r)
        NO.disparity16(L[0, y0:y0 + rows + 2 * r], R[0, y0:y0 + rows + 2 * r], 0, D, win, costi)
        ns += 1
        dts = time.perf_counter() - t0
        if dts >= max(1.0, seconds / 4) or ns >= 40:
            break
    numpy_fps = ns * min(rows, H) / H / dts
    return {
        "numpy_oracle_value": round(numpy_fps, 4),
        "numpy_oracle_sample": f"{ns} strips of {rows}+{2 * r} rows x {W} (disparity only) of the "
                               f"NumPy oracle (oracle/sv_oracle.py) in {dts:.1f} s, single process, "
                               f"scaled by {rows}/{H} rows to frames/s",
        "value": round(n / dt, 3), "unit": "frames/s", "cores": aff, "kind": "port",
        "cpu_count": ncpu, "affinity_cores": aff,
        "single_thread_value": round(n1 / dt1, 4),
        "sample": f"{n} full {W}x{H} frames (D={D}, win={win}, {cost}: disparity + median5 + "
                  f"depth post{' + Harris (1 thread)' if harris else ''}) of the C oracle "
                  f"(oracle/sv_oracle.c, the engine's semantics; the reference's cv2.StereoSGBM "
                  f"is not installed), OpenMP {aff} threads = every core this process may use "
                  f"(affinity set, capped by the cgroup CPU quota; os.cpu_count() {ncpu}), "
                  f"{dt:.1f} s; single thread: {n1} frames "
                  f"in {dt1:.1f} s",
    }


# ---- helpers -------------------------------------------------------------------------------
class DevArena:
    """Device buffers of one engine, freed together."""

    def __init__(self, eng):
        self.eng, self.ptrs = eng, []

    def alloc(self, nbytes):
        p = self.eng.dev_alloc(max(256, int(nbytes)))
        self.ptrs.append(p)
        return p

    def upload(self, a):
        a = np.ascontiguousarray(a)
        p = self.alloc(a.nbytes)
        self.eng.to_device(p, a)
        return p

    def free(self):
        for p in self.ptrs:
            self.eng.dev_free(p)
        self.ptrs = []


def make_rectifier(eng, W, H):
    """Device-resident CV_16SC2 maps of a synthetic calibration (stereoRectify alpha=0)."""
    from stereovision_amd import calib
    from stereovision_amd.rectify import StereoRectifier
    c = synthetic_calibration(W, H)
    R1, R2, P1, P2, _, _, _ = calib.stereo_rectify(c["mtx_left"], c["dist_left"], c["mtx_right"],
                                                   c["dist_right"], (W, H), c["R"], c["T"], alpha=0)
    return StereoRectifier.from_calibration(c["mtx_left"], c["dist_left"], R1, P1, c["mtx_right"],
                                            c["dist_right"], R2, P2, (W, H), eng)


def hbm_entry(name, bytes_per_launch, ms, n):
    if not n:
        return None
    s = ms / n * 1e-3
    gbs = bytes_per_launch / s / 1e9
    return {"kernel": name, "bound": "hbm", "avg_launch_us": round(s * 1e6, 2),
            "bytes_per_launch": bytes_per_launch, "achieved": round(gbs, 1), "unit": "GB/s",
            "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4), "launches": n}


def aux_kernels(eng, H, W, B, med_ms, med_n, reps=20, blocker=None, frames=None, maps=None):
    """HBM rooflines of the memory-bound kernels around k_match, measured after the timed
    region (not part of `value`): k_median_i16 from the timed steps, k_remap (the
    rectify+gray stage in front of the path) over a batch of B raw BGR frames, the occlusion
    statistics of a pair and one radix-select pass.  The small kernels are timed as a run of
    `reps` back-to-back calls between two stream events (sv_timer_*), enqueued behind a
    `blocker` (one step of the path) so they run back to back on the device: device time
    per call, without host launch latency or per-launch event overhead.  `frames` = (left,
    right) device stacks of >= B gray frames and `maps` = a device stack of >= B f32 disparity
    maps from the path: the occlusion statistics run on the camera frames and the selects on
    the disparity maps, as the reference applies them (fused_depth_map.py:131-301,
    1169-1257); without them, uniform random data."""
    out = {"k_median_i16": hbm_entry("k_median_i16", 11 * H * W * B, med_ms, med_n)}
    arena = DevArena(eng)

    def timed(fn):
        for _ in range(3):
            fn()
        eng.synchronize()
        if blocker is not None:
            blocker()
        eng.timer_begin()
        for _ in range(reps):
            fn()
        return eng.timer_end(), reps
    try:
        Bs = max(2, B)
        rect = make_rectifier(eng, W, H)
        rng = np.random.default_rng(7)
        src = arena.upload(rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8))
        dst = arena.alloc(Bs * H * W)
        m1, m2 = rect.device_maps[0], rect.device_maps[1]

        def remap():
            eng.remap_dev(src, H, W, 3, 3 * W, m1, m2, H, W, dst, W, gray_out=True, n_frames=B,
                          src_frame_stride=3 * H * W, dst_frame_stride=H * W)
        ms, n = timed(remap)
        # algorithmic bytes per output pixel: 6 (map1 + map2) + 3 (BGR source) + 1 (gray out)
        out["k_remap_bgr2gray"] = hbm_entry("k_remap<3,gray>", 10 * H * W * B, ms, n)
        rect.close()
        # occlusion statistics of a rectified gray pair (1 B/px per image read once; the
        # histogram fold runs in the same launch)
        nb = max(1, H // 48) * max(1, W // 48)
        st = arena.alloc(4 * 2 * (2 * nb + 256))
        f0, f1 = frames if frames else (dst, dst + H * W)
        ms, n = timed(lambda: eng.frame_stats_dev(f0, f1, H, W, 1, W, st, st + 8 * nb, st + 16 * nb))
        out["k_frame_stats"] = hbm_entry("k_frame_stats", 2 * H * W, ms, n)
        # the same statistics for a batch of B pairs in one launch + one fold
        # (sv_frame_stats_batch_dev): the queued-frames form
        if frames:
            g0, g1, gfs = frames[0], frames[1], H * W
        else:
            gpair = arena.upload(rng.integers(0, 256, (B, 2, H, W), dtype=np.uint8))
            g0, g1, gfs = gpair, gpair + H * W, 2 * H * W
        stb = arena.alloc(4 * 2 * B * (2 * nb + 256))
        ms, n = timed(lambda: eng.frame_stats_batch_dev(g0, g1, B, gfs, H, W, 1, W, stb, stb + 8 * B * nb,
                                                        stb + 16 * B * nb))
        out["k_frame_stats_batch"] = hbm_entry(f"k_frame_stats ({B} pairs per launch)", 2 * H * W * B, ms, n)
        # one radix-select pass over a float32 disparity map (4 B/px).  select_count returns
        # its counts to the host (a synchronising call), so this one is timed per launch by
        # the context's kernel events
        d = maps if maps else arena.upload(rng.random((H, W), dtype=np.float32))
        eng.profile_reset()
        eng.profile(True)
        for _ in range(reps):
            eng.select_count(d, H * W, 1)
        eng.profile(False)
        ms, n = eng.profile_read("select")
        out["k_select_hist"] = hbm_entry("k_select_hist", 4 * H * W, ms, n)
        # one pass over a batch of B maps per launch (sv_select_count_batch: grid.y = map)
        Bm = min(B, 16)
        dm = maps if maps else arena.upload(rng.random((Bm, H, W), dtype=np.float32))
        eng.select_count_batch(dm, H * W, H * W, Bm, 1)
        eng.profile_reset()
        eng.profile(True)
        for _ in range(reps):
            eng.select_count_batch(dm, H * W, H * W, Bm, 1)
        eng.profile(False)
        ms, n = eng.profile_read("select")
        out["k_select_hist_batch"] = hbm_entry(f"k_select_hist ({Bm} maps per launch)", 4 * H * W * Bm, ms, n)
    finally:
        arena.free()
    return out


def host_path(H, W, D, win, seconds=3.0):
    """PCIe-inclusive rate of the drop-in path the reference actually calls (depth_map.py:
    1181-1183): BGR NumPy frames -> depth_map.create_depth_map -> (depth, disparity,
    colormap) NumPy arrays, one frame per call; and the pipelined form of the same calls
    (stereovision_amd.pipeline: several frames in flight, as fused_depth_map.py:2591-2598
    submits frames to a worker pool)."""
    from stereovision_amd import depth_map as DM
    frames = []
    for s in range(4):
        L, R, _ = stereo_pair(H, W, D, seed=900 + s)
        frames.append((to_bgr(L), to_bgr(R)))
    DM.NUM_DISP, DM.WINDOW_SIZE, DM.MIN_DISP = D, win, 0
    for i in range(3):
        DM.create_depth_map(*frames[i % 4])
    n, t0 = 0, time.perf_counter()
    while True:
        DM.create_depth_map(*frames[n % 4])
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or n >= 2000:
            break
    out = {"unit": "frames/s", "frames": n, "value": round(n / dt, 1),
           "ms_per_call": round(dt * 1e3 / n, 3),
           "path": "BGR uint8 NumPy pair -> depth_map.create_depth_map -> (depth f32, disparity "
                   "f32, colormap u8x3) NumPy, one synchronous call per frame",
           "bytes_h2d_per_frame": 6 * H * W}
    try:
        out["per_call"] = host_path_stages(DM, frames, H, W)
    except Exception as e:  # reported, never required
        out["per_call"] = {"error": str(e)}
    try:
        from stereovision_amd.pipeline import DepthMapPipeline, max_in_flight
    except ImportError:
        return out
    pipe = DepthMapPipeline(D, win, depth=max_in_flight())
    try:
        # every context warmed several times: its first frames pay one-time costs (page-locked
        # staging buffers, first touch — profiles/r06_pipeline/sweep.txt)
        for i in range(5 * pipe.depth):
            pipe.submit(*frames[i % 4]).result()
        futs, n, t0 = [], 0, time.perf_counter()
        while True:
            futs.append(pipe.submit(*frames[n % 4]))
            n += 1
            if len(futs) > pipe.depth:
                futs.pop(0).result()
            dt = time.perf_counter() - t0
            if dt >= seconds or n >= 4000:
                break
        for f in futs:
            f.result()
        dt = time.perf_counter() - t0
        out["pipelined"] = {"value": round(n / dt, 1), "frames": n, "in_flight": pipe.depth,
                            "path": "the same calls through DepthMapPipeline.submit (futures)"}
    finally:
        pipe.close()
    return out


def host_path_stages(DM, frames, H, W, calls=300, seconds=1.5):
    """Where a synchronous create_depth_map call's time goes (a separate, profiled run of the
    same calls): device events around each image upload (SV_K_H2D), the kernels and the
    outputs' download (SV_K_D2H) on the engine's stream, and the host stages of the call
    (sv_host_profile_*).  Device spans are per call (both images for h2d / gray); their sum
    against the wall time shows what bounds the call."""
    from stereovision_amd.engine import host_profile
    eng = get_engine()
    host_profile(enable=True, reset=True)
    eng.profile(True)
    eng.profile_reset()
    m, t0 = 0, time.perf_counter()
    try:
        while m < calls and time.perf_counter() - t0 < seconds:
            DM.create_depth_map(*frames[m % len(frames)])
            m += 1
        wall = time.perf_counter() - t0
    finally:
        eng.profile(False)
        hp = host_profile(enable=False, reset=True)
    dev = {k: eng.profile_read(k) for k in ("h2d", "gray", "match", "median", "d2h")}
    eng.profile_reset()
    us = {f"{k}_us": round(ms * 1e3 / m, 1) for k, (ms, _) in dev.items()}
    kernel_us = us["gray_us"] + us["match_us"] + us["median_us"]
    # the outputs that cross PCIe: registered output arrays come back by DMA (depth f32 +
    # disparity f32 + colormap BGR = 11 B/px), else the int16 medians (2 B/px) + host expansion
    dma = hp["expand"] is not None and hp["expand"] < 0.01
    d2h_bytes = 11 * H * W if dma else 2 * H * W
    regs = getattr(eng, "_registered", {})
    return {"calls": m, "wall_us": round(wall * 1e6 / m, 1), **us,
            "outputs_registered": len(regs),
            "output_registration": "off (default: int16 download + host expansion measured faster; "
                                   "SV_REGISTER_OUTPUTS=1 enables the DMA path)" if getattr(eng, "_noreg", False) else "on",
            "kernel_us": round(kernel_us, 1),
            "device_sum_us": round(us["h2d_us"] + kernel_us + us["d2h_us"], 1),
            "h2d_GBps": round(6 * H * W / (us["h2d_us"] * 1e-6) / 1e9, 1) if us["h2d_us"] else None,
            "d2h_bytes": d2h_bytes,
            "d2h_path": ("registered output arrays filled by DMA" if dma else
                         "int16 medians + host expansion"),
            "d2h_GBps": round(d2h_bytes / (us["d2h_us"] * 1e-6) / 1e9, 1) if us["d2h_us"] else None,
            "host_ms": {k: (round(v, 3) if v is not None else None) for k, v in hp.items() if k != "calls"},
            "note": "device spans from HIP events on the call's stream (h2d: both BGR images from the "
                    "caller's pageable arrays, staged by the HIP runtime); host_ms = sv_host_profile stages"}


# ---- live PMC (rocprofv3 passes over a short child run of this script) -----------------------
PMC_PASSES = [("sq", ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"]),
              ("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"])]


def kernel_busy(tmp, tag):
    """Union of the dispatch intervals of the kernels named `tag` in the kernel trace under
    `tmp`: with launches of two streams in flight together, each launch's own duration counts
    the time it shares the device with the other, so per-launch bytes / duration undercounts
    the kernel's throughput; bytes of all launches / the time any of them runs does not."""
    spans = []
    for f in glob.glob(os.path.join(tmp, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if tag in r.get("Kernel_Name", ""):
                spans.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if len(spans) < 4:
        return {}
    spans.sort()
    spans = spans[len(spans) // 4:]   # past the warm-up
    busy, cur_s, cur_e = 0, spans[0][0], spans[0][1]
    for a, b in spans[1:]:
        if a > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    busy += cur_e - cur_s
    return {"busy_launches": len(spans), "busy_us_per_launch": round(busy / len(spans) / 1e3, 2),
            "busy_overlap": round(sum(b - a for a, b in spans) / busy, 3) if busy else None}


def live_pmc(args, kernel_tags=("k_match",), timeout=150):
    """rocprofv3 over short child runs of this script with the same workload: one kernel-trace
    pass (average duration of the match kernel and the median, to set beside the HIP-event
    launch times of the timed region) and the PMC passes.  The first of `kernel_tags` found in
    the trace names the match kernel (SSD: k_ssd_mfma where it runs, else k_match)."""
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rocprof):
        return {"error": "rocprofv3 not found"}
    tmp = tempfile.mkdtemp(prefix="sv_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--warmup", "2",
             "--height", str(args.height), "--width", str(args.width), "--num-disp", str(args.num_disp),
             "--win", str(args.win), "--cost", args.cost, "--batch", str(args.batch),
             "--frames", str(args.frames), "--streams", str(args.streams)]
    agg, trace = {}, {}
    kernel_tag = kernel_tags[0]
    try:
        cmd = [rocprof, "--kernel-trace", "--stats", "--output-format", "csv", "-d",
               os.path.join(tmp, "trace"), "-o", "trace", "--", *child, "--steps", "60", "--warmup-seconds", "1.0"]
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=tmp,
                             start_new_session=True, env=dict(os.environ, TMPDIR=tmp))
        try:
            _, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            err = b"timed out"
        # a failed trace pass is reported in `trace` and the PMC passes still run
        if p.returncode != 0:
            trace["error"] = f"rocprofv3 kernel-trace pass rc={p.returncode}: {err.decode(errors='replace')[-300:]}"
        stats = []
        for f in glob.glob(os.path.join(tmp, "trace", "**", "*kernel_stats.csv"), recursive=True):
            stats += list(csv.DictReader(open(f)))
        for tag in kernel_tags:
            rows = [r for r in stats if tag in r["Name"]]
            if rows:
                kernel_tag = tag
                r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
                trace["kernel"] = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                trace["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
                trace["calls"] = int(r["Calls"])
                break
        med = [r for r in stats if "k_median" in r["Name"]]
        if med:
            trace["median_avg_us"] = round(float(med[0]["AverageNs"]) / 1e3, 2)
        if trace.get("kernel"):
            trace.update(kernel_busy(tmp, kernel_tag))
        for name, counters in PMC_PASSES:
            cmd = [rocprof, "--pmc", *counters, "--output-format", "csv", "-d",
                   os.path.join(tmp, name), "-o", name, "--", *child, "--steps", "6"]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=tmp,
                                 start_new_session=True, env=dict(os.environ, TMPDIR=tmp))
            try:
                _, err = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return {"error": f"rocprofv3 pass {name} timed out", "trace": trace}
            if p.returncode != 0:
                return {"error": f"rocprofv3 pass {name} rc={p.returncode}: "
                                 f"{err.decode(errors='replace')[-300:]}", "trace": trace}
            for f in glob.glob(os.path.join(tmp, name, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if kernel_tag in r["Kernel_Name"]:
                        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    res = {k: sum(v) / len(v) for k, v in agg.items()}
    res["dispatches"] = max((len(v) for v in agg.values()), default=0)
    res["trace"] = trace
    return res


# ---- verification of the timed outputs (after the timed region) --------------------------
class Verifier:
    """Bit-exact check of maps the timed steps produced against the C oracle
    (oracle/sv_oracle.c, the engine's semantics; test infrastructure used here only as the
    checker): (depth_final, disparity, depth_normalized) of create_depth_map per frame
    (depth_map.py:909-936), the Harris response within 1e-4 (north_star)."""

    def __init__(self, D, win, cost, threads):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import sv_oracle_c as C  # test infrastructure: the checker only
        self.C, self.D, self.win, self.threads = C, D, win, threads
        self.cost = {"sad": 0, "ssd": 1, "hog": 2}[cost]
        self.checked, self.failed = [], []

    def frame(self, tag, L, R, got_depth, got_disp, got_norm):
        e_depth, e_disp, e_norm = self.C.depth_map(L, R, 0, self.D, self.win, self.cost, 0.3, 2.0,
                                                   self.threads)
        ok = (np.array_equal(got_disp, e_disp) and np.array_equal(got_depth, e_depth)
              and np.array_equal(got_norm, e_norm))
        self.checked.append(tag)
        if not ok:
            bad = int((got_disp != e_disp).sum())
            self.failed.append(f"{tag}: {bad} disparity pixels differ")
        return ok

    def disparity(self, tag, L, R, got_disp):
        _, e_disp, _ = self.C.depth_map(L, R, 0, self.D, self.win, self.cost, 0.3, 2.0, self.threads)
        self.checked.append(tag)
        if not np.array_equal(got_disp, e_disp):
            self.failed.append(f"{tag}: {int((got_disp != e_disp).sum())} disparity pixels differ")

    def harris(self, tag, L, got):
        exp = self.C.harris(L)
        err = float(np.max(np.abs(got.astype(np.float64) - exp))) if exp.size else 0.0
        self.checked.append(tag + " harris")
        if not err <= 1e-4:
            self.failed.append(f"{tag}: Harris max |diff| {err:.3g} > 1e-4")

    def result(self):
        return not self.failed


def fetch_maps(eng, d_depth, d_disp, d_norm, index, n_px, H, W):
    """Frame `index` of dense per-frame output stacks -> host (depth, disparity, norm)."""
    return (eng.to_host(d_depth + 4 * n_px * index, (H, W), np.float32),
            eng.to_host(d_disp + 4 * n_px * index, (H, W), np.float32),
            eng.to_host(d_norm + n_px * index, (H, W), np.uint8))


def map_to_disp(eng, d_map, index, n_px, H, W, u8):
    """Frame `index` of a dense stack of gathered maps -> the f32 disparity it encodes: u8
    indices d8 + min_disp - 1 (min_disp 0 here) or int16 x16 / 16."""
    if u8:
        return eng.to_host(d_map + n_px * index, (H, W), np.uint8).astype(np.float32) - np.float32(1.0)
    return eng.to_host(d_map + 2 * n_px * index, (H, W), np.int16).astype(np.float32) / np.float32(16.0)


def init_comms(devices, required: bool):
    """One process, N devices: an RCCL group (ncclCommInitAll) -> (comms, "").  When it
    cannot start: (None, reason) — the caller gathers with hipMemcpyPeerAsync
    and names the fallback in the line — or SystemExit with --require-rccl.
    SV_RCCL_INIT_FAIL=1 makes the init fail as ncclCommInitAll would (the fallback's test)."""
    try:
        if os.environ.get("SV_RCCL_INIT_FAIL", "") not in ("", "0"):
            raise RuntimeError("ncclCommInitAll: forced failure (SV_RCCL_INIT_FAIL)")
        return Communicator.init_all(devices), ""
    except Exception as ex:
        reason = f"ncclCommInitAll failed: {ex}"
        if required:
            raise SystemExit(f"RCCL group over devices {devices} unavailable ({ex}) and --require-rccl given")
        log(f"RCCL group unavailable ({ex}); gathering with peer copies (hipMemcpyPeerAsync)")
        return None, reason


def agreed_extra_warmup(pg, spent_s: float, steps_done: int, warmup_seconds: float) -> int:
    """Warm-up steps every rank runs after its first W (one-process-per-GPU launches): each
    rank estimates how many more steps fill --warmup-seconds at its own rate, and all take the
    max over ranks, so ranks whose steps hold a collective stay in lock step (a rank that
    decided on its own clock ran one warm-up step more than its peers and waited in a gather
    the others never entered)."""
    per = spent_s / max(1, steps_done)
    left = max(0.0, warmup_seconds - spent_s)
    mine = min(100000, int(left / max(per, 1e-6)) + 1) if left > 0 else 0
    return int(pg.allreduce_max(float(mine)))


def dist_summary(ngpu, launched, pg=None, comms=None, gather=False, rowtile=False,
                 gather_ms=0.0, gather_n=0, scatter_ms=0.0, scatter_n=0, gather_wall_s=0.0,
                 steps=0, gather_bytes=0, scatter_bytes=0, reason="", gathered_maps=None,
                 expand_ms=0.0, expand_n=0, root_outputs=None):
    """The multi-GPU fields of the bench line (None for one GPU): the backend the run used,
    how many ranks the RCCL communicator saw (0 + the reason when it fell back), and the
    gather / scatter time per step from HIP events on the root's stream (these include the
    wait for the slowest rank's maps)."""
    if ngpu <= 1:
        return None
    if launched:
        backend = pg.backend
        rccl_ranks = pg.rccl_ranks
        why = pg.reason
    else:
        backend = "rccl" if comms else "peer"
        rccl_ranks = len(comms) if comms else 0
        why = "" if comms else (reason or "RCCL group not requested")
    out = {"backend": backend, "rccl_ranks": rccl_ranks, "rccl_reason": why or None,
           "process_model": "one process per GPU" if launched else "one process, all devices",
           "gather": bool(gather or rowtile),
           "gathered_maps": gathered_maps,
           "gather_us_per_step": round(gather_ms * 1e3 / gather_n, 2) if gather_n else None,
           "gather_events": gather_n,
           "gather_bytes_per_step": gather_bytes or None,
           "gather_wall_us_per_step": (round(gather_wall_s * 1e6 / steps, 2)
                                       if (gather_wall_s and steps) else None)}
    if out["gather_us_per_step"] and gather_bytes:
        out["gather_GBps"] = round(gather_bytes / (gather_ms * 1e-3 / gather_n) / 1e9, 1)
    out["root_outputs"] = root_outputs
    # the root's k_post_m16 launches (peers' medians -> create_depth_map outputs), HIP events
    out["root_expand_us_per_step"] = round(expand_ms * 1e3 / expand_n, 2) if expand_n else None
    if rowtile:
        out["scatter_us_per_step"] = round(scatter_ms * 1e3 / scatter_n, 2) if scatter_n else None
        out["scatter_bytes_per_step"] = scatter_bytes or None
        out["inputs"] = "band-only: each rank receives its band + halo rows from rank 0 inside the step"
    return out


# ---- main ----------------------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-seconds", type=float, default=1.0,
                    help="keep warming up (untimed steps) until at least this long has passed "
                         "and --warmup steps ran: the GPU needs tens of ms of load to reach its "
                         "steady clocks, so 5 steps (3 ms) time the clock ramp, not the kernels")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--num-disp", type=int, default=128)
    ap.add_argument("--win", type=int, default=9)
    ap.add_argument("--cost", default="sad", choices=["sad", "ssd", "hog", "sgbm"],
                    help="sad/ssd/hog: the north_star WTA engine; sgbm: the SGBM-3WAY mode")
    ap.add_argument("--frames", type=int, default=None,
                    help="distinct resident frames per GPU (default: the batch)")
    ap.add_argument("--batch", type=int, default=None,
                    help="frames mode: frames per step and GPU, one launch per kernel over the "
                         "batch (sv_depth_map_batch_dev); 1 = one frame per call (latency mode). "
                         "Default 16; 26 for 1920x1080 (not SGBM): the metric config's k_match grid "
                         "is 1,890 waves per frame, 26 frames = 49,140 waves = 24.0 rounds of the "
                         "2,048 wave slots (16 frames = 14.8 rounds, a last round 77%% full): +0.9%% "
                         "frames/s, C3 (win 11) +1.1%% (profiles/r05ag, r05ai)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no HIP events in the timed loop")
    ap.add_argument("--profile-every", type=int, default=4,
                    help="bracket the kernels of every N-th timed step with HIP events (each "
                         "event record costs a few us of queue time; 1 = every step)")
    ap.add_argument("--mode", default="frames", choices=["frames", "rowtile"],
                    help="frames: independent frames per GPU (C4, weak scaling); rowtile: one "
                         "frame row-tiled across GPUs, band inputs scattered from GPU 0 and the "
                         "bands gathered back (C5, strong scaling)")
    ap.add_argument("--gather", action="store_true",
                    help="(default for --gpus N > 1) gather every step's output maps to GPU 0")
    ap.add_argument("--no-gather", action="store_true",
                    help="frames mode, N > 1: no gather (the compute-only weak-scaling curve)")
    ap.add_argument("--full-frame-inputs", action="store_true",
                    help="rowtile: every GPU holds the full frame (no input scatter in the step)")
    ap.add_argument("--band-inputs", default="scatter", choices=["scatter", "host"],
                    help="rowtile, N > 1: where each GPU's band rows come from inside a step — "
                         "scatter: from GPU 0's HBM over xGMI (RCCL send/recv; launched: on a "
                         "communicator and stream of its own, so frame i+1's scatter runs beside "
                         "frame i's gather in the opposite link direction); host: every GPU uploads "
                         "its own band's rows from page-locked host memory over its own PCIe link "
                         "(no xGMI scatter; the step is then PCIe-inclusive, so the line says so)")
    ap.add_argument("--require-rccl", action="store_true",
                    help="N distinct devices: exit non-zero when RCCL cannot start (default: one "
                         "process gathers with hipMemcpyPeerAsync, one process per GPU through the "
                         "file store, and the line names the fallback: backend + rccl_reason)")
    ap.add_argument("--root-outputs", default="m16", choices=["m16", "full"],
                    help="N > 1 (frames and rowtile): what GPU 0 holds after each step's gather — "
                         "m16: the disparity rows only (north_star's 'gather of the final "
                         "disparity rows', --gather-format), nothing expanded on GPU 0; full: also "
                         "create_depth_map's depth f32 / disparity f32 / u8, expanded on GPU 0 from "
                         "the gathered int16 medians (k_post_m16, 11 B/px of GPU 0's HBM per peer "
                         "pixel)")
    ap.add_argument("--gather-format", default="auto", choices=["auto", "i16", "u8"],
                    help="--root-outputs m16: the gathered disparity rows as int16 x16 (2 B/px) or "
                         "as u8 disparity indices d - min_disp + 1 (1 B/px: SAD/SSD/HOG disparities "
                         "are whole pixels, exact for num_disp <= 255); auto: u8 where exact")
    ap.add_argument("--rehearse", action="store_true",
                    help="one process: run --gpus N logical GPUs on the visible devices (logical "
                         "GPU k on device k %% devices: own context, stream and buffers; gathers "
                         "as device copies) — the 1-GPU rehearsal of the N-GPU one-process path")
    ap.add_argument("--rectify", action="store_true",
                    help="camera pipeline: raw BGR frames resident in HBM -> rectify+gray "
                         "(k_remap, calibrated CV_16SC2 maps) -> disparity -> median/post")
    ap.add_argument("--streams", type=int, default=0,
                    help="frames mode: contexts (HIP streams) per GPU that consecutive steps "
                         "alternate over, so one step overlaps the next (separate output buffers "
                         "per stream); 0 = auto: 3 for frames of <= 1 MP (a 16-frame VGA batch "
                         "leaves most of the chip idle between its launches), else 1")
    ap.add_argument("--schedule", default="lanes", choices=["split", "lanes"],
                    help="frames mode, one GPU: split = the match launch of batch i on one stream "
                         "and the median launch of batch i-1 on a second (SV_STAGE_MATCH / "
                         "SV_STAGE_MEDIAN of sv_depth_map_batch_dev: the HBM-bound median beside "
                         "the VALU-bound match, k_match launches never overlapping each other); "
                         "lanes (default) = --streams contexts alternating whole steps.  split "
                         "measured slower at 1080p (29.8k vs 29.7k one stream / 30.6k two lanes) and "
                         "4K (2.88k vs 3.14k): the median's sorting network competes with the match "
                         "for VALU issue, so it does not hide behind it (profiles/r06b)")
    ap.add_argument("--no-aux", action="store_true", help="skip the aux-kernel rooflines")
    ap.add_argument("--harris", action="store_true",
                    help="C2: also compute the Harris response of every left frame (k_harris)")
    ap.add_argument("--dist-backend", default=None, choices=["auto", "rccl", "host"],
                    help="one-process-per-GPU launch: RCCL or the node-local file store (auto: "
                         "RCCL unless ranks share a GPU).  Default: auto, and RCCL is then "
                         "required whenever the ranks are on distinct devices and a step has "
                         "a collective (the gather / the row-tile scatter)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the bit-exact check of the timed steps' outputs")
    ap.add_argument("--no-live-pmc", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host_path measurement")
    ap.add_argument("--hang-timeout", type=float, default=900.0,
                    help="dump every thread's stack and exit non-zero when the run takes longer "
                         "than this many seconds (a rank stuck in a collective fails loudly)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    full_hd = (args.height, args.width) == (1080, 1920) and args.cost != "sgbm"
    one_gpu = args.gpus <= 1 and int(os.environ.get("WORLD_SIZE", "1")) <= 1
    lanes2 = full_hd and args.mode == "frames" and one_gpu and not (args.rectify or args.harris)
    if args.batch is None:
        # 1080p frames on one GPU: 8-frame steps alternating over 2 streams (the second lane's
        # match fills the first one's tail waves: 29.7k -> 30.6-30.7k frames/s, profiles/r06b);
        # N > 1: 26 (whole rounds of k_match waves, one stream beside the gather stream)
        args.batch = (8 if lanes2 and args.streams in (0, 2) else 26) if full_hd and args.mode == "frames" else 16
    if args.streams == 0 and lanes2 and args.schedule != "split":
        args.streams = 2
    if args.frames is None:
        args.frames = args.batch * (2 if args.streams == 2 and lanes2 else 1)
    if args.pmc_child:
        args.no_cpu_baseline = args.no_aux = args.no_live_pmc = args.no_host_path = True
        args.no_profile = args.no_verify = True
        # the PMC passes count per dispatch (no warm-up needed); the kernel-trace pass times
        # kernels and passes its own --warmup-seconds (after this flag) to reach steady clocks
        if "--warmup-seconds" not in sys.argv:
            args.warmup_seconds = 0.0
    return args


def main():
    args = parse_args()
    if args.hang_timeout > 0:
        faulthandler.dump_traceback_later(args.hang_timeout, exit=True)
    launched = int(os.environ.get("WORLD_SIZE", "1")) > 1
    rowtile = args.mode == "rowtile"
    pg = None
    if launched:
        from stereovision_amd.distributed import init_process_group
        world_env = int(os.environ["WORLD_SIZE"])
        collective = rowtile or (world_env > 1 and not args.no_gather)
        backend = args.dist_backend or "auto"
        pg = init_process_group(backend=backend, strict=collective and args.require_rccl)
        rank, world = pg.rank, pg.world
        devices = [pg.device]
    else:
        rank, world = 0, 1
        n = max(1, args.gpus)
        nd = device_count()
        if n > nd and not args.rehearse:
            raise SystemExit(f"--gpus {n} but only {nd} device(s) are visible (--rehearse runs "
                             "them as contexts of the visible devices)")
        devices = [k % max(1, nd) for k in range(n)] if args.rehearse else list(range(n))
    ngpu = world * len(devices)
    # one context per logical GPU (the rehearsal puts several on one device)
    engines = [get_engine(d) if k == devices.index(d) else Engine(d) for k, d in enumerate(devices)]
    shared_devices = len(set(devices)) < len(devices)
    eng = engines[0]

    H, W, D, win = args.height, args.width, args.num_disp, args.win
    F = max(1, args.frames)
    B = max(1, min(args.batch, F))
    F = (F // B) * B
    rectify = args.rectify and not rowtile
    if rectify and len(devices) > 1:
        raise SystemExit("--rectify runs one GPU per process (use the torch.distributed.run launch)")
    harris = args.harris and not rowtile
    n_px = H * W
    arenas = [DevArena(e) for e in engines]
    gather_on = (not rowtile) and ngpu > 1 and not args.no_gather
    band_inputs = rowtile and ngpu > 1 and not args.full_frame_inputs
    host_bands = band_inputs and args.band_inputs == "host"

    # resident inputs: F distinct frames per GPU (rowtile: ONE frame, on GPU 0 only unless
    # --full-frame-inputs; the other GPUs receive their band rows inside each step)
    dL, dR, hostL, hostR = [], [], [], []
    for k, (e, a) in enumerate(zip(engines, arenas)):
        if rowtile:
            L, R = stereo_batch(1, H, W, D, seed=4242)
        else:
            L, R = stereo_batch(F, H, W, D, seed=1000 * (rank * len(devices) + k))
        hostL.append(L)
        hostR.append(R)
        if host_bands:   # every GPU reads its band rows from page-locked host memory
            if k == 0:
                for a_ in (L, R):
                    if e.lib.sv_host_register(a_.ctypes.data, a_.nbytes) != 0:
                        raise SystemExit("--band-inputs host: sv_host_register failed")
            dL.append(0)
            dR.append(0)
            continue
        if band_inputs and (rank if launched else k) != 0:
            dL.append(0)
            dR.append(0)
            continue
        if rectify:
            L, R = np.repeat(L[..., None], 3, axis=3), np.repeat(R[..., None], 3, axis=3)
        dL.append(a.upload(L))
        dR.append(a.upload(R))
    gather_all = (gather_on or rowtile) and not launched and len(engines) > 1
    root_full = args.root_outputs == "full"
    # u8 disparity indices over xGMI (1 B/px) where they are exact: integer-disparity costs,
    # num_disp <= 255, and GPU 0 holds the gathered maps only (no expansion from int16 medians);
    # frames and rowtile, launched and one-process alike
    gather_u8 = (args.gather_format != "i16" and not root_full and args.cost != "sgbm" and D <= 255)
    if args.gather_format == "u8" and not gather_u8:
        raise SystemExit("--gather-format u8 needs --root-outputs m16, an integer cost and num_disp <= 255")
    gel = 1 if gather_u8 else 2     # bytes per gathered pixel
    gather_desc = "u8 disparity index" if gather_u8 else "int16 x16"
    out_frames = 1 if rowtile else B * (len(engines) if gather_all else 1)
    depth = [a.alloc(4 * n_px * out_frames) for a in arenas]
    disp = [a.alloc(4 * n_px * out_frames) for a in arenas]
    norm = [a.alloc(n_px * out_frames) for a in arenas]
    # --streams S: S-1 extra contexts per GPU (own stream, own outputs) that steps alternate over
    # default: 3 streams for frames <= 1 MP (launch-bound); 2 for HOG and for 4K frames (the
    # write-bound histograms / the median of one stream's batch beside the VALU-bound match of
    # the other's: C5 HOG 1,564 -> 1,637-1,651, C5 SAD 2,920 -> 3,035 frames/s,
    # profiles/r05h_hog); 1 otherwise (1080p SAD: 2 streams +2.0%, 2 x 8-frame batches +2.9%,
    # left at one stream so the roofline's launch times stay those of a launch alone)
    # --schedule split (default above 1 MP): the match of batch i on the compute stream beside
    # the median of batch i-1 on a median stream (own context), int16 maps double-buffered
    split = args.schedule == "split" and not (rowtile or rectify or gather_on or harris or len(engines) > 1 or B == 1)
    req_streams = args.streams if args.streams > 0 else (
        3 if n_px <= 1_000_000 else 2 if (args.cost == "hog" or n_px >= 4_000_000) else 1)
    nstreams = max(1, req_streams) if not (rowtile or args.rectify or gather_on or split) else 1
    lanes = [(engines, depth, disp, norm)]
    for _ in range(nstreams - 1):
        lanes.append(([Engine(d) for d in devices], [a.alloc(4 * n_px * out_frames) for a in arenas],
                      [a.alloc(4 * n_px * out_frames) for a in arenas], [a.alloc(n_px * out_frames) for a in arenas]))
    all_engines = [e for ln in lanes for e in ln[0]]
    if rectify:
        rect = make_rectifier(eng, W, H)
        gL, gR = arenas[0].alloc(B * n_px), arenas[0].alloc(B * n_px)
        m1l, m2l, m1r, m2r, _, _ = rect.device_maps
    if harris:   # per stream lane: its own Harris maps
        hmaps_l = [[a.alloc(4 * n_px * B) for a in arenas] for _ in range(nstreams)]
        hmaps = hmaps_l[0]
    meng, sd16 = None, None
    if split:
        meng = Engine(devices[0])
        all_engines.append(meng)
        sd16 = [arenas[0].alloc(2 * n_px * B) for _ in range(2)]
        sout = map_out(POST_DEPTH, disp[0], depth[0], norm[0], min_depth=0.3, max_depth=2.0,
                       min_disp_global=0)
    tile = tiles = None
    rt = {"t": 0, "primed": False, "last": 0, "n": 0}
    if rowtile and launched:
        from stereovision_amd.distributed import RowTiledDepthMap
        # two tiles (band inputs, medians, outputs each) alternate over consecutive frames, so
        # the band scatter of frame i+1 and the gather of frame i run on a communication stream
        # while frame i+1 computes
        tiles = [RowTiledDepthMap(H, W, D, win, cost=args.cost, device=devices[0], rank=rank,
                                  world=world, engine=eng) for _ in range(2 if world > 1 else 1)]
        tile = tiles[0]
    comms, comm_reason = None, ""
    forced_fail = os.environ.get("SV_RCCL_INIT_FAIL", "") not in ("", "0")
    if shared_devices and not forced_fail:
        comm_reason = "rehearsal: logical GPUs share a device (device copies, no RCCL)"
    elif not launched and len(engines) > 1 and (gather_on or rowtile):
        # one process, N devices: an RCCL group, or — when ncclCommInitAll fails — the gather
        # by hipMemcpyPeerAsync (SURVEY.md §5's fallback), named in the line (backend "peer",
        # rccl_reason) instead of ending the run
        comms, comm_reason = init_comms(devices, args.require_rccl)
    # one process, N devices, gather: two lanes of contexts (own streams, scratch, RCCL
    # group and root outputs each) that consecutive steps alternate over, so one step's
    # gather overlaps the next step's kernels
    glanes = None
    if gather_all:
        comms2 = None
        if comms is not None:
            comms2, why2 = init_comms(devices, args.require_rccl)
            if comms2 is None:   # both lanes gather the same way
                for c in comms:
                    c.close()
                comms, comm_reason = None, why2
        engines2 = [Engine(d) for d in devices]
        all_engines.extend(engines2)
        glanes = [(engines, comms, depth[0], disp[0], norm[0], arenas[0].alloc(2 * n_px * out_frames)),
                  (engines2, comms2, arenas[0].alloc(4 * n_px * out_frames), arenas[0].alloc(4 * n_px * out_frames),
                   arenas[0].alloc(n_px * out_frames), arenas[0].alloc(2 * n_px * out_frames))]
    # launched frames mode with the gather: every step's disparity maps go to rank 0 as int16
    # x16 (OpenCV's fixed-point disparity, written by the median epilogue beside the f32 map,
    # which is exactly it / 16: half the xGMI bytes of the f32 map) on a communication stream
    # of their own, double-buffered, so step i's gather overlaps step i+1's kernels; rank 0
    # receives them into one stack per buffer (rank-major).  Event slots of `eng`: 2s = set s
    # computed, 2s+1 = set s gathered.
    gathered, ceng, cstream, expanded = None, None, 0, None
    if launched and gather_on:
        ceng = Engine(devices[0])
        cstream = ceng.stream
        all_engines.append(ceng)
        gset = [(depth[0], disp[0], norm[0], arenas[0].alloc(gel * n_px * B)),
                (arenas[0].alloc(4 * n_px * B), arenas[0].alloc(4 * n_px * B), arenas[0].alloc(n_px * B),
                 arenas[0].alloc(gel * n_px * B))]
        gathered = [arenas[0].alloc(gel * n_px * B * world) if rank == 0 else 0 for _ in range(2)]
        # --root-outputs full: rank 0 expands the peers' gathered medians into create_depth_map's
        # outputs (its own frames already have them), double-buffered like the gathers
        nexp = n_px * B * (world - 1)
        expanded = ([(arenas[0].alloc(4 * nexp), arenas[0].alloc(4 * nexp), arenas[0].alloc(nexp))
                     for _ in range(2)] if (root_full and rank == 0) else None)
    geng, gstream, pg2 = None, 0, None
    if tiles is not None and world > 1:
        # scatter (root -> peers) on ceng's stream over pg's communicator; the gather (peers ->
        # root) on geng's stream over a second communicator (pg.dup), so frame i+1's scatter and
        # frame i's gather use opposite link directions at once
        ceng = Engine(devices[0])
        cstream = ceng.stream
        geng = Engine(devices[0])
        gstream = geng.stream
        all_engines += [ceng, geng]
        pg2 = pg.dup("gather")
    gather_wall = [0.0]

    def step(i):
        f = (i * B) % F
        if rowtile:
            if launched and world == 1:
                tile.compute(dL[0], dR[0])
            elif launched:
                # pipelined over the two tiles (event slots of `eng`: 4+t = tile t's band inputs
                # in place, 6+t = tile t computed, 8+t = tile t's medians gathered): compute(i) on
                # the compute stream; frame i+1's band inputs into the other tile on the scatter
                # stream (after that tile's previous compute), frame i's medians to the root on the
                # gather stream (after compute(i)) — two streams, two communicators
                t = rt["t"]
                u = (t + 1) % len(tiles)
                # gather-only (--root-outputs m16): every rank, the root included, writes only its
                # band of the map (int16 x16 or u8 indices); full: the root's band is expanded by
                # its own epilogue and the peers' int16 bands after the gather
                bo = ("full" if rank == 0 else "m16") if root_full else ("d8" if gather_u8 else "m16")

                def bands_into(x):
                    if rt["n"] >= 2:   # the tile's previous frame has been computed
                        eng.stream_wait_event(6 + x, cstream)
                    ceng.profile_region_begin("h2d" if host_bands else "scatter", cstream)
                    if host_bands:
                        tiles[x].upload(hostL[0][0], hostR[0][0], stream=cstream)
                    else:
                        tiles[x].scatter(pg, dL[0], dR[0], stream=cstream)
                    ceng.profile_region_end(cstream)
                    eng.event_record(4 + x, cstream)
                if rt["n"] >= 2:       # tile t's medians of two frames ago have left
                    eng.stream_wait_event(8 + t, eng.stream)
                if band_inputs:
                    if not rt["primed"]:
                        bands_into(t)
                        rt["primed"] = True
                    eng.stream_wait_event(4 + t, eng.stream)
                    tiles[t].compute(band_outputs=bo)
                else:
                    tiles[t].compute(dL[0], dR[0], band_outputs=bo)
                eng.event_record(6 + t, eng.stream)
                rt["n"] += 1
                if band_inputs:
                    bands_into(u)
                eng.stream_wait_event(6 + t, gstream)
                geng.profile_region_begin("gather", gstream)
                tiles[t].gather(pg2, stream=gstream, expand=root_full, check=rt["n"] == 1)
                geng.profile_region_end(gstream)
                eng.event_record(8 + t, gstream)
                rt["last"], rt["t"] = t, u
            else:   # one process: two lanes of contexts alternate, so frame i+1's scatter and
                    # kernels overlap frame i's gather and expansion
                le, lc, ldep, ldis, lnor, lmap = glanes[i % 2]
                if host_bands:      # every context uploads its band from host memory
                    if root_full:
                        depth_map_rows_multi(le, lc, hostL[0][0], hostR[0][0], H, W, W, 0, D, win, 0.3, 2.0,
                                             ldep, ldis, lnor, cost=args.cost, scatter="host")
                    else:
                        depth_map_rows_map(le, lc, hostL[0][0], hostR[0][0], H, W, W, 0, D, win, lmap,
                                           fmt="d8" if gather_u8 else "m16", scatter="host", cost=args.cost)
                elif not root_full:   # gather-only: the full map on device 0, nothing expanded
                    depth_map_rows_map(le, lc, dL[0] if band_inputs else dL, dR[0] if band_inputs else dR,
                                       H, W, W, 0, D, win, lmap, fmt="d8" if gather_u8 else "m16",
                                       scatter=band_inputs, cost=args.cost)
                elif band_inputs:
                    depth_map_rows_scatter(le, lc, dL[0], dR[0], H, W, W, 0, D, win, 0.3, 2.0,
                                           ldep, ldis, lnor, cost=args.cost)
                else:
                    depth_map_rows_multi(le, lc, dL, dR, H, W, W, 0, D, win, 0.3, 2.0,
                                         ldep, ldis, lnor, cost=args.cost)
                rt["last"] = i % 2
            return
        if split:   # event slots of `eng`: k = d16[k] written, 2+k = d16[k] read by its median
            k = i % 2
            if i >= 2:
                eng.stream_wait_event(2 + k, eng.stream)
            eng.depth_map_batch_ex(dL[0] + f * n_px, dR[0] + f * n_px, B, H, W, W, n_px, 0, D, win, args.cost,
                                   STAGE_MATCH, sd16[k], None, stream=eng.stream)
            eng.event_record(k, eng.stream)
            eng.stream_wait_event(k, meng.stream)
            meng.depth_map_batch_ex(0, 0, B, H, W, W, n_px, 0, D, win, args.cost, STAGE_MEDIAN, sd16[k], sout,
                                    stream=meng.stream)
            eng.event_record(2 + k, meng.stream)
            return
        if gather_all:     # one process, N devices, maps gathered on device 0 (1 or 2 B/px)
            le, lc, ldep, ldis, lnor, lmap = glanes[i % 2]
            if root_full:
                multi_gpu_depth_map_dev(le, lc, [p + f * n_px for p in dL],
                                        [p + f * n_px for p in dR], [B] * len(le), H, W, W, n_px,
                                        0, D, win, 0.3, 2.0, ldep, ldis, lnor, cost=args.cost)
            else:
                multi_gpu_map_dev(le, lc, [p + f * n_px for p in dL], [p + f * n_px for p in dR],
                                  [B] * len(le), H, W, W, n_px, 0, D, win, lmap,
                                  fmt="d8" if gather_u8 else "m16", cost=args.cost)
            return
        engs, depth_o, disp_o, norm_o = lanes[i % nstreams]
        med_o = 0
        if gathered is not None:   # double-buffered output sets; set s free once its gather ran
            gs = i % 2
            if i >= 2:
                eng.stream_wait_event(2 * gs + 1, eng.stream)
            depth_o, disp_o, norm_o = [gset[gs][0]], [gset[gs][1]], [gset[gs][2]]
            med_o = gset[gs][3]
        for k, e in enumerate(engs):
            if rectify:
                for src, m1, m2, g in ((dL[k], m1l, m2l, gL), (dR[k], m1r, m2r, gR)):
                    e.remap_dev(src + f * 3 * n_px, H, W, 3, 3 * W, m1, m2, H, W, g, W,
                                gray_out=True, n_frames=B, src_frame_stride=3 * n_px,
                                dst_frame_stride=n_px)
                e.depth_map_batch_dev(gL, gR, B, H, W, W, n_px, 0, D, win, 0.3, 2.0, depth[k],
                                      disp[k], norm[k], cost=args.cost)
            elif B == 1 and not med_o:
                e.depth_map_dev(dL[k] + f * n_px, dR[k] + f * n_px, H, W, W, 0, D, win, 0.3, 2.0,
                                depth_o[k], disp_o[k], norm_o[k], cost=args.cost)
            elif harris and not rectify and not med_o:   # Harris blocks inside the median launch
                e.depth_map_batch_dev(dL[k] + f * n_px, dR[k] + f * n_px, B, H, W, W, n_px, 0, D, win,
                                      0.3, 2.0, depth_o[k], disp_o[k], norm_o[k], cost=args.cost,
                                      d_harris=hmaps_l[i % nstreams][k])
            else:
                e.depth_map_batch_dev(dL[k] + f * n_px, dR[k] + f * n_px, B, H, W, W, n_px, 0, D, win,
                                      0.3, 2.0, depth_o[k], disp_o[k], norm_o[k], cost=args.cost,
                                      d_med16=0 if gather_u8 else med_o, d_d8=med_o if gather_u8 else 0)
            if harris and (rectify or med_o or B == 1):   # one launch over the batch's left frames
                e.harris_batch_dev(gL if rectify else dL[k] + f * n_px, B, H, W, W, n_px,
                                   hmaps_l[i % nstreams][k])
        if gathered is not None:   # every rank's disparity maps -> rank 0 (RCCL over xGMI)
            from stereovision_amd.distributed import gather_frames
            t_g = time.perf_counter()
            eng.event_record(2 * gs, eng.stream)        # set gs computed
            eng.stream_wait_event(2 * gs, cstream)      # the gather follows it
            ceng.profile_region_begin("gather", cstream)
            gather_frames(pg, gset[gs][3], B, gathered[gs], gel * n_px, stream=cstream)
            ceng.profile_region_end(cstream)
            if expanded is not None:   # the peers' frames, after the gather on the same stream
                xd, xp, xu = expanded[gs]
                ceng.post_m16_dev(gathered[gs] + 2 * n_px * B, nexp, POST_DEPTH, d_disparity=xp,
                                  d_out_a=xd, d_out_u8=xu, min_depth=0.3, max_depth=2.0,
                                  min_disp_global=0, min_disp=0, num_disp=D, stream=cstream)
            eng.event_record(2 * gs + 1, cstream)       # set gs free again
            gather_wall[0] += time.perf_counter() - t_g

    def sync_all():
        for e in all_engines:
            e.synchronize()

    t_w = time.perf_counter()
    n_warm = 0
    if pg is None:
        while n_warm < args.warmup or (time.perf_counter() - t_w < args.warmup_seconds and n_warm < 100000):
            step(n_warm)
            n_warm += 1
            if n_warm >= args.warmup and n_warm % 8 == 0:
                sync_all()    # the time test sees device progress, not just enqueued steps
    else:
        # launched: a step may hold a collective (the gather, the row-tile scatter), so every
        # rank must run the same number of warm-up steps — the W steps, then the extra steps
        # the slowest rank needs to fill --warmup-seconds (agreed through a max over ranks)
        for _ in range(max(1, args.warmup)):
            step(n_warm)
            n_warm += 1
        sync_all()
        extra = agreed_extra_warmup(pg, time.perf_counter() - t_w, n_warm, args.warmup_seconds)
        for _ in range(extra):
            step(n_warm)
            n_warm += 1
            if n_warm % 8 == 0:
                sync_all()
    sync_all()
    warm_s = time.perf_counter() - t_w
    for pe in ([eng] + ([ceng] if ceng is not None else []) + ([glanes[1][0][0]] if glanes else [])
               + ([meng] if meng is not None else []) + ([geng] if geng is not None else [])):
        pe.profile(False)
        pe.profile_reset()
    gather_wall[0] = 0.0
    every = max(1, args.profile_every)

    if pg is not None:
        pg.barrier()
    sync_all()
    t0 = time.perf_counter()
    prof_engs = ([eng] + ([ceng] if ceng is not None else []) + ([glanes[1][0][0]] if glanes else [])
                 + ([meng] if meng is not None else []) + ([geng] if geng is not None else []))
    for i in range(args.steps):
        for pe in prof_engs:
            if not args.no_profile and every > 1:
                pe.profile(i % every == 0)        # host-side toggle, no GPU work
            elif i == 0:
                pe.profile(not args.no_profile)
        step(i)
    sync_all()
    elapsed = time.perf_counter() - t0     # this rank's; the max over ranks is the run's
    if pg is not None:
        pg.barrier()

    for pe in prof_engs:
        pe.profile(False)
    match_ms, match_n = eng.profile_read("sgbm" if args.cost == "sgbm" else "match")
    med_ms, med_n = (meng or eng).profile_read("median")
    remap_ms, remap_n = eng.profile_read("remap")
    harris_ms, harris_n = eng.profile_read("harris")
    gath_ms, gath_n = (geng or ceng or eng).profile_read("gather")
    if glanes:   # the second lane's root context times its own gathers
        m2, n2 = glanes[1][0][0].profile_read("gather")
        gath_ms, gath_n = gath_ms + m2, gath_n + n2
    scat_ms, scat_n = (ceng or eng).profile_read("h2d" if host_bands and launched else "scatter")
    if glanes:
        m2, n2 = glanes[1][0][0].profile_read("scatter")
        scat_ms, scat_n = scat_ms + m2, scat_n + n2
    exp_ms, exp_n = (ceng or eng).profile_read("post")
    if ceng is not None and rowtile:   # the tiles' expansion runs on the compute context's engine
        m2, n2 = eng.profile_read("post")
        exp_ms, exp_n = exp_ms + m2, exp_n + n2
    if glanes:
        m2, n2 = glanes[1][0][0].profile_read("post")
        exp_ms, exp_n = exp_ms + m2, exp_n + n2
    k_name = "sgbm pipeline (k_sgbm_*)" if args.cost == "sgbm" else "k_match"
    if pg is not None:
        elapsed = pg.allreduce_max(elapsed)

    frames = args.steps if rowtile else ngpu * args.steps * B
    value = frames / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    if args.pmc_child:
        print(json.dumps({"pmc_child": True, "value": value}), flush=True)
        return

    # ---- the timed steps' own outputs, checked bit-exactly (outside the timed region) ----
    verified, verify_info = None, None
    if not args.no_verify and args.cost != "sgbm":
        t_v = time.perf_counter()
        ver = Verifier(D, win, args.cost, host_cores()[0])
        last = args.steps - 1 if args.steps > 0 else max(0, n_warm - 1)
        f0 = (last * B) % F
        zs = sorted({0, B - 1})
        if rowtile:
            where = "rank 0" if launched else "device 0"
            if launched and rank == 0:
                tl = tiles[rt["last"]]
                if root_full:
                    ver.frame("full frame gathered on rank 0", hostL[0][0], hostR[0][0],
                              eng.to_host(tl.out_a, (H, W), np.float32),
                              eng.to_host(tl.disp, (H, W), np.float32),
                              eng.to_host(tl.out_u8, (H, W), np.uint8))
                else:
                    ver.disparity(f"full-frame map gathered on rank 0 ({gather_desc})", hostL[0][0],
                                  hostR[0][0], map_to_disp(eng, tl.m16, 0, n_px, H, W, gather_u8))
            elif not launched:
                if root_full or not glanes:
                    od, op, on = (glanes[rt["last"]][2:5] if glanes else (depth[0], disp[0], norm[0]))
                    ver.frame(f"full frame gathered on {where}", hostL[0][0], hostR[0][0],
                              *fetch_maps(eng, od, op, on, 0, n_px, H, W))
                else:
                    ver.disparity(f"full-frame map gathered on {where} ({gather_desc})", hostL[0][0],
                                  hostR[0][0], map_to_disp(eng, glanes[rt["last"]][5], 0, n_px, H, W,
                                                           gather_u8))
        elif gather_all:
            _, _, ldep, ldis, lnor, lmap = glanes[last % 2]
            for k in range(len(engines)):
                for z in zs:
                    tag = f"device {k} frame {f0 + z} (gathered on device 0)"
                    if root_full:
                        ver.frame(tag, hostL[k][f0 + z], hostR[k][f0 + z],
                                  *fetch_maps(eng, ldep, ldis, lnor, k * B + z, n_px, H, W))
                    else:
                        ver.disparity(f"{tag} {gather_desc}", hostL[k][f0 + z], hostR[k][f0 + z],
                                      map_to_disp(eng, lmap, k * B + z, n_px, H, W, gather_u8))
        else:
            engs, depth_o, disp_o, norm_o = lanes[last % nstreams]
            if gathered is not None:
                gs = last % 2
                depth_o, disp_o, norm_o = [gset[gs][0]], [gset[gs][1]], [gset[gs][2]]
            for k, e in enumerate(engs):
                for z in zs:
                    Lz, Rz = hostL[k][f0 + z], hostR[k][f0 + z]
                    if rectify:
                        sys.path.insert(0, os.path.join(ROOT, "oracle"))
                        import sv_rectify_oracle as RO  # test infrastructure: the checker only
                        lm1, lm2, rm1, rm2 = rect.host_maps()
                        Lz = RO.remap_gray(np.repeat(Lz[..., None], 3, axis=2), lm1, lm2)
                        Rz = RO.remap_gray(np.repeat(Rz[..., None], 3, axis=2), rm1, rm2)
                    ver.frame(f"rank {rank} device {k} frame {f0 + z}", Lz, Rz,
                              *fetch_maps(e, depth_o[k], disp_o[k], norm_o[k], z, n_px, H, W))
                    if harris:
                        ver.harris(f"rank {rank} device {k} frame {f0 + z}", Lz,
                                   e.to_host(hmaps_l[last % nstreams][k] + 4 * n_px * z, (H, W),
                                             np.float32))
            if gathered is not None and rank == 0:
                from stereovision_amd.synthetic import stereo_pair
                for r in range(world):
                    for z in zs:
                        if r == 0:
                            Lz, Rz = hostL[0][f0 + z], hostR[0][f0 + z]
                        else:   # rank r's inputs, regenerated from its seed
                            Lz, Rz, _ = stereo_pair(H, W, D, seed=1000 * r + f0 + z)
                        got = map_to_disp(eng, gathered[last % 2], r * B + z, n_px, H, W, gather_u8)
                        ver.disparity(f"rank {r} frame {f0 + z} (gathered on rank 0)", Lz, Rz, got)
                        if expanded is not None and r > 0:
                            xd, xp, xu = expanded[last % 2]
                            ver.frame(f"rank {r} frame {f0 + z} (expanded on rank 0)", Lz, Rz,
                                      *fetch_maps(eng, xd, xp, xu, (r - 1) * B + z, n_px, H, W))
        ok = ver.result()
        if pg is not None:
            ok = pg.allreduce_max(0.0 if ok else 1.0) == 0.0
        verified = bool(ok)
        verify_info = {"checked": ver.checked if rank == 0 else len(ver.checked),
                       "failures": ver.failed or None,
                       "against": "oracle/sv_oracle.c (the engine's semantics), bit-exact"
                                  + (" + Harris within 1e-4" if harris else ""),
                       "when": "after the timed region: maps of the LAST timed step",
                       "seconds": round(time.perf_counter() - t_v, 2)}
    elif args.cost == "sgbm":
        verify_info = {"skipped": "SGBM mode: the NumPy SGBM-3WAY oracle takes ~15 s per 1080p "
                                  "frame; tests/test_sgbm.py checks the kernels bit-exactly"}
    # the collectives are over: from here on every phase (rocprofv3 passes, host path, CPU
    # baseline) has its own time limit, so the whole-run hang guard stands down
    if args.hang_timeout > 0:
        faulthandler.cancel_dump_traceback_later()

    # pixels of one k_match launch: the batch (frames) or this GPU's band + median halo
    npx = n_px * B
    if rowtile:
        from stereovision_amd.distributed import band_rows, median_halo
        r0, r1 = band_rows(H, 0, ngpu)
        h0, h1 = median_halo(r0, r1, H)
        npx = (h1 - h0) * W
    k_avg_s = (match_ms / match_n) * 1e-3 if match_n else None
    k_bytes = 6 * npx         # 2 u8 images read + the f32 disparity map
    k_bytes_kernel = 4 * npx  # what k_match itself moves: 2 u8 images in, int16 map out
    frame_bytes = 11 * n_px   # 2 u8 in; depth f32 + disparity f32 + u8 out
    if harris:
        frame_bytes += 4 * n_px
    if rectify:
        frame_bytes = 11 * n_px + 2 * 10 * n_px   # + per camera: map 6 B, BGR 3 B, gray 1 B
    roofline = None
    pmc = {}
    if k_avg_s:
        if rank == 0 and not args.no_live_pmc and not launched and len(engines) == 1 and not rowtile:
            t_p = time.perf_counter()
            pmc = live_pmc(args, ("sgbm",) if args.cost == "sgbm" else
                           ("k_ssd_mfma", "k_match") if args.cost == "ssd" else ("k_match",))
            pmc["seconds"] = round(time.perf_counter() - t_p, 1)
        ktrace = pmc.pop("trace", None) or {}
        achieved = k_bytes / k_avg_s / 1e9
        insts = pmc.get("SQ_INSTS_VALU")
        fetch = pmc.get("FETCH_SIZE")
        write = pmc.get("WRITE_SIZE")
        # gfx950: FETCH_SIZE tallies 128-B fabric reads at 64 B (MI355X_MICROARCH.md, HBM /
        # rocprofv3): x2.  Calibrated on k_match's own dword reads: with the XCD tile order
        # every input byte is fetched once, and FETCH_SIZE reads 0.49 x the 66.4 MB of input
        traffic = (round((2 * fetch + write) * 1024) if fetch is not None and write is not None
                   else None)
        roofline = {
            # bound: what limits the kernel (VALU issue); achieved/peak/frac stay
            # the contract's HBM figures (algorithmic bytes by SURVEY.md §8(d)), the VALU
            # roofline is the `valu` object below
            "kernel": k_name, "bound": "valu" if args.cost != "sgbm" else "hbm",
            "frac_basis": "hbm", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "bytes_per_launch": k_bytes,
            "bytes_rule": "SURVEY.md §8(d): 6 B/px (2 u8 images + f32 disparity) x pixels per launch",
            "achieved_note": "algorithmic bytes over the live launch time (HIP events), not a counter-"
                             f"observed HBM rate: the {F} resident frames ({2 * F * n_px / 1e6:.0f} MB of "
                             "inputs) live in the 256 MB Infinity Cache; the kernel's limiter is VALU "
                             "issue (see `valu`)",
            "kernel_bytes_per_launch": k_bytes_kernel,
            "frac_kernel_bytes": round(k_bytes_kernel / k_avg_s / 1e9 / HBM_PEAK_GBS, 5),
            "avg_launch_us": round(k_avg_s * 1e6, 2), "launches": match_n,
            # with S > 1 streams (frames <= 1 MP) lane 0's launches share the device
            # with the other lanes' kernels, so these launch times are contended ones
            "launch_concurrency": ("split schedule: k_match launches back to back on the compute "
                                   "stream, each timed while the previous batch's median runs on the "
                                   "median stream (HIP events on the compute stream; the rocprofv3 "
                                   "kernel trace of the same command gives the same durations)"
                                   if split else
                                   f"{nstreams} streams: lane 0's launches timed while the other "
                                   f"{nstreams - 1} lanes' kernels share the device (not comparable "
                                   "with single-stream launch times)" if nstreams > 1 else "one stream"),
            # what actually bounds k_match: VALU issue.  SQ_INSTS_VALU per
            # launch from the live rocprofv3 pass over the live launch time, against the
            # full-rate issue peak (1 wave64 instruction / 2 cycles / SIMD); v_sad_u8 and the
            # other VOP3 integer ops issue at half that rate (profiles/r01_valu_rate.txt).
            "valu": {"bound": "valu", "unit": "wave-instr/s",
                     "achieved": round(insts / k_avg_s) if insts else None,
                     "peak": VALU_ISSUE_PEAK,
                     "frac": round(insts / k_avg_s / VALU_ISSUE_PEAK, 4) if insts else None,
                     "insts_per_launch": round(insts) if insts else None,
                     "insts_per_wave_cell": (round(insts / (npx * D / 64), 3) if insts else None),
                     "cells_per_s": round(npx * D / k_avg_s),
                     # the issue rate against the valu_rate microbenchmark at the kernel's 2 waves
                     # per SIMD (independent chains): the VOP3 integer ops k_match issues (v_sad_*,
                     # v_min3, DPP mins) sustain 2.06-2.22 ns per wave-instruction per SIMD, a mixed
                     # v_sad_u8 + v_min_u32 stream 1.88 ns, v_add 1.37 ns
                     "ns_per_wave_instr_per_simd": (round(N_SIMD * k_avg_s / insts * 1e9, 3) if insts else None),
                     "microbench_ns_per_wave_instr": {"v_sad_u8/v_sad_hi_u8/v_sad_u32": 2.2, "v_min3_u32/v_min_u32_dpp": 2.15,
                                                      "mixed v_sad_u8 + v_min_u32": 1.88, "v_add_u32": 1.37,
                                                      "source": "profiles/r05a/valu_rate_wps2.txt"}},
            "pmc": {"source": "rocprofv3 --pmc, 3 separate passes over a 6-step child run of this "
                              "script on this box (mean per k_match dispatch)",
                    "traffic_note": "traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024): the guide's "
                                    "gfx950 x2 FETCH correction, calibrated on k_match's own reads "
                                    "(XCD tile order: each input byte fetched once = 2 x FETCH_SIZE); "
                                    "inputs stay resident in the 256 MB Infinity Cache, whose hits "
                                    "the counter includes",
                    **{k: (round(v, 1) if isinstance(v, float) else v) for k, v in pmc.items()}},
            "median_post_avg_us": round(med_ms / med_n * 1e3, 2) if med_n else None,
        }
        if ktrace.get("avg_us"):
            # the same figures from the rocprofv3 kernel trace of a 60-step child run of this
            # command: per-kernel GPU durations, independent of HIP events
            ta = ktrace["avg_us"] * 1e-6
            roofline["trace"] = {
                "source": "rocprofv3 --kernel-trace --stats over a 60-step child run of this command (1 s warm-up)",
                "kernel": ktrace["kernel"], "calls": ktrace["calls"], "avg_launch_us": ktrace["avg_us"],
                "achieved": round(k_bytes / ta / 1e9, 2), "frac": round(k_bytes / ta / 1e9 / HBM_PEAK_GBS, 5),
                "median_avg_us": ktrace.get("median_avg_us"),
                "events_vs_trace": round(k_avg_s / ta, 4)}
            if ktrace.get("busy_us_per_launch"):
                # all launches' bytes over the time any of them runs (union of the dispatch
                # intervals): the kernel's throughput when the lanes' launches overlap
                tb = ktrace["busy_us_per_launch"] * 1e-6
                roofline["trace"].update({
                    "busy_us_per_launch": ktrace["busy_us_per_launch"], "busy_launches": ktrace["busy_launches"],
                    "launch_overlap": ktrace["busy_overlap"],
                    "achieved_busy": round(k_bytes / tb / 1e9, 2),
                    "frac_busy": round(k_bytes / tb / 1e9 / HBM_PEAK_GBS, 5)})
            roofline["kernel"] = ktrace["kernel"]
        elif ktrace.get("error"):
            roofline["trace"] = {"error": ktrace["error"]}

    # per step: bytes received by the root (N-1 peers' maps; rowtile: N-1 bands of the three
    # outputs) and, rowtile with band inputs, bytes sent from the root (both images' rows)
    gbytes = sbytes = 0
    if ngpu > 1:
        if rowtile:
            from stereovision_amd.distributed import band_layout
            for k in range(1, ngpu):
                b = band_layout(H, k, ngpu, win)
                gbytes += gel * (b["r1"] - b["r0"]) * W    # int16 x16 median rows or u8 indices
                if band_inputs and not host_bands:
                    sbytes += 2 * (b["in1"] - b["in0"]) * W
        elif gather_on:   # the disparity maps: u8 indices (launched, where exact) or int16 x16
            gbytes = gel * n_px * B * (ngpu - 1)
    dist = dist_summary(ngpu, launched, pg, comms, gather=gather_on, rowtile=rowtile,
                        gather_ms=gath_ms, gather_n=gath_n, scatter_ms=scat_ms, scatter_n=scat_n,
                        gather_wall_s=gather_wall[0], steps=args.steps, gather_bytes=gbytes,
                        scatter_bytes=sbytes, reason=comm_reason, expand_ms=exp_ms, expand_n=exp_n,
                        root_outputs=("full" if root_full else "m16") if (gather_on or rowtile) else None,
                        gathered_maps=(("row bands of the disparity" if rowtile else "disparity of every frame")
                                       + (" as u8 indices d - min_disp + 1 (whole-pixel disparities: exact; "
                                          "the f32 map is d8 + min_disp - 1)" if gather_u8 else
                                          " as int16 x16 (OpenCV's fixed point; the f32 map is it / 16 exactly)")
                                       + (", expanded on GPU 0 into depth f32 + disparity f32 + depth u8"
                                          if root_full else ", nothing expanded on GPU 0")
                                       + (", overlapped with the next step (communication stream, "
                                          "double-buffered)" if launched else
                                          ", two context lanes so a step's gather overlaps the next step"))
                        if (gather_on or rowtile) else None)
    if dist is not None and (gather_on or rowtile):
        dist["gather_format"] = gather_desc
    if dist is not None and rowtile:
        b0 = __import__("stereovision_amd.distributed", fromlist=["band_layout"]).band_layout(H, 0, ngpu, win)
        dist["band_inputs"] = ("full frame resident on every GPU (no input transfer in the step)"
                               if not band_inputs else
                               "host: every GPU uploads its band + halo rows from page-locked host memory "
                               "over its own PCIe link inside the step (no xGMI scatter; PCIe-inclusive)"
                               if host_bands else
                               "scatter: each GPU receives its band + halo rows from GPU 0's HBM over xGMI "
                               "inside the step")
        dist["inputs"] = dist["band_inputs"]
        if host_bands:
            dist["h2d_bytes_per_step_per_gpu"] = 2 * (b0["in1"] - b0["in0"]) * W
            dist["scatter_us_per_step"] = None
            dist["h2d_us_per_step"] = round(scat_ms * 1e3 / scat_n, 2) if scat_n else None
        if launched and ngpu > 1:
            dist["comm_streams"] = ("band inputs on a stream of their own " +
                                    ("(host uploads)" if host_bands else "(RCCL scatter, communicator 1)") +
                                    "; the band gather on a second stream over communicator 2 (pg.dup): "
                                    "frame i+1's inputs travel while frame i's medians leave, in opposite "
                                    "link directions")
    parallelism = (f"row-tiled x{ngpu}" + ((" (band inputs uploaded from host memory by every GPU)" if host_bands
                                            else " (band inputs scattered from GPU 0)") if band_inputs else "")
                   + " + band gather" if rowtile else
                   f"frame-sharded x{ngpu}" + (" + gather to GPU 0" if gather_on else ""))
    if ngpu > 1:
        parallelism += (f" ({'one process per GPU, ' + pg.backend if launched else 'one process, ' + ('RCCL group' if comms else 'peer copies')})")
    result = {
        "metric": "disparity frames/sec + HBM GB/s, 1920x1080 D=128 win=9, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "frames/s", "n_gpus": ngpu, "steps": args.steps,
        "warmup": args.warmup, "warmup_steps_run": n_warm, "warmup_seconds": round(warm_s, 3),
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if rowtile else "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic rectified pairs (stereovision_amd.synthetic, distinct seeds per GPU)",
        "config": {"workload": (f"{W}x{H} D={D} win={win} {args.cost.upper()} camera pipeline: "
                                "raw BGR frames resident in HBM -> rectify+gray (k_remap) -> "
                                "disparity -> median5 + depth post" if rectify else
                                f"{W}x{H} D={D} win={win} {args.cost.upper()} depth_map path "
                                "(disparity + median5 + depth post" + (" + Harris response"
                                                                        if harris else "") +
                                "), gray inputs resident in HBM"),
                   "harris": harris,
                   "height": H, "width": W, "num_disp": D, "win": win, "cost": args.cost,
                   "frames_resident_per_gpu": 1 if rowtile else F,
                   "frames_per_step_per_gpu": 1 if rowtile else B,
                   "streams_per_gpu": 2 if split else nstreams,
                   "schedule": "split (match stream + median stream)" if split else
                               (f"lanes ({nstreams} contexts alternating steps)" if nstreams > 1 else "one stream"),
                   "parallelism": parallelism},
        "verified": verified,
        "verify": verify_info,
        "distributed": dist,
        "hbm_gbs_frame_path": round(frame_bytes * value / 1e9, 2),
        # BASELINE.md's fixed roofline formulas, per GPU: 6*H*W algorithmic bytes and
        # H*W*D*win^2 SAD taps per frame against 8.0e12 B/s and 157.3e12 taps/s.  The
        # taps fraction exceeds 1 because running window sums do O(1) work per tap column.
        "baseline_roofline": {
            "fps_per_gpu": round(value / ngpu, 2),
            "achieved_hbm_frac": round(6 * n_px * value / ngpu / 8.0e12, 5),
            "achieved_valu_frac": round(n_px * D * win * win * value / ngpu / 157.3e12, 4)},
        "roofline": roofline,
        "aux_kernels": None,
        "host_path": None,
        "cpu_baseline": None,
    }
    solo = rank == 0 and ngpu == 1
    if rectify and remap_n:
        result["aux_kernels"] = {
            "k_remap_bgr2gray": hbm_entry("k_remap<3,gray>", 10 * n_px * B, remap_ms, remap_n)}
        rect.close()
    elif solo and not rowtile and not args.no_aux:
        try:
            result["aux_kernels"] = aux_kernels(eng, H, W, B, med_ms, med_n, blocker=lambda: step(0),
                                                frames=(dL[0], dR[0]), maps=disp[0])
            result["aux_kernels"]["inputs"] = ("occlusion statistics on the bench's gray frame pairs, "
                                               "selects (mask disparity > 0) on the path's disparity maps")
        except Exception as e:  # reported, never required
            log(f"aux kernels failed: {e}")
    if harris and harris_n:     # 1 B/px gray read + 4 B/px f32 response written
        result["aux_kernels"] = dict(result["aux_kernels"] or {})
        result["aux_kernels"]["k_harris"] = hbm_entry("k_harris_dpp", 5 * n_px * B, harris_ms,
                                                       harris_n)
    elif harris:
        result["aux_kernels"] = dict(result["aux_kernels"] or {})
        result["aux_kernels"]["k_harris"] = {
            "fused": "Harris blocks inside the k_median_i16 launch (sv_depth_map_batch_dev, out.harris): "
                     "median_post_avg_us includes them"}
    if solo and not args.no_host_path and args.cost != "sgbm" and not rectify:
        try:
            result["host_path"] = host_path(H, W, D, win)
        except Exception as e:  # reported, never required
            log(f"host path failed: {e}")
    if solo and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(H, W, D, win, args.cost, args.cpu_seconds,
                                                  harris=harris)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu baseline failed: {e}")
    if rank == 0:
        print(json.dumps(result), flush=True)
    for tl in tiles or []:
        tl.close()
    for a in arenas:
        a.free()
    if comms:
        for c in comms:
            c.close()
    if glanes and glanes[1][1]:
        for c in glanes[1][1]:
            c.close()
    if pg2 is not None:
        pg2.close()
    if pg is not None:
        pg.close()
    if verified is False:
        log("bench outputs do NOT match the oracle: " + "; ".join(verify_info["failures"] or ["(other rank)"]))
        sys.exit(3)


if __name__ == "__main__":
    main()
