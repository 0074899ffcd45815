#!/usr/bin/env python3
"""bench.py — disparity frames/s of the MI355X engine (BASELINE.json metric).

Workload (BASELINE.json metric): 1920x1080 rectified synthetic pairs, D=128, 9x9 SAD
window, the whole device path of depth_map.create_depth_map per frame:
    disparity (k_match) -> medianBlur 5 + depth post (k_median_i16, fused)
Inputs are gray u8 pairs already resident in HBM (8 distinct frames per rank, cycled);
outputs are depth f32, disparity f32 and depth u8 per frame.  One step = one batch of
--batch frame pairs (default 8) through sv_depth_map_batch_dev: one k_match and one
k_median_i16 launch over the whole batch (grid.z = frame), which keeps all 256 CUs busy
instead of leaving a partial last wave of blocks per frame.  --batch 1 = one call per frame.

Multi-GPU: one process per GPU (torch.distributed.run), frames sharded across ranks with
no collective in the data path (weak scaling); value = frames of all ranks / max time.

Extra JSON fields: `roofline` for the dominant kernel (k_match; HIP-event durations
measured inside the timed region) with the VALU-tap figure beside the HBM one, and
`cpu_baseline` = the C oracle (oracle/sv_oracle.c, OpenMP) on this host's cores.

torch is imported BEFORE the engine library so libsvhip binds to torch's HIP runtime
(both ship libamdhip64.so.7; see DESIGN.md "One HIP runtime per process").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch  # noqa: E402  (must precede the engine library load)
import torch.distributed as dist
import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from stereovision_amd.engine import get_engine  # noqa: E402
from stereovision_amd.synthetic import stereo_batch, synthetic_calibration  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 2   # 256 CU x 4 SIMD, one wave64 VALU instr per 2 cycles


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    """C oracle (the port) timed on this host: whole app-1 path per frame (+ the Harris
    response of the left frame for C2)."""
    if cost == "sgbm":
        return cpu_baseline_sgbm(H, W, D, win, seconds)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sv_oracle_c as C  # test infrastructure, used here only as the CPU baseline
    lib = C.lib()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))
    L, R = stereo_batch(2, H, W, D, seed=4242)
    depth = np.empty((H, W), np.float32)
    disp = np.empty((H, W), np.float32)
    norm = np.empty((H, W), np.uint8)
    costi = {"sad": 0, "ssd": 1, "hog": 2}[cost]

    def one(i):
        lib.svo_depth_map(np.ascontiguousarray(L[i % 2]), np.ascontiguousarray(R[i % 2]), H, W,
                          0, D, win, costi, np.float32(0.3), np.float32(2.0),
                          np.float32(2.0 - 0.3), depth, disp, norm, threads)
        if harris:
            C.harris(np.ascontiguousarray(L[i % 2]))

    import ctypes
    f32 = ctypes.c_float
    lib.svo_depth_map.argtypes = [C._u8p, C._u8p, C._i, C._i, C._i, C._i, C._i, C._i, f32, f32,
                                  f32, C._f32p, C._f32p, C._u8p, C._i]
    lib.svo_depth_map.restype = C._i
    one(0)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        one(n)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or n >= 200:
            break
    return {
        "value": round(n / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port",
        "sample": f"{n} full {W}x{H} frames (D={D}, win={win}, {cost}: disparity + median5 + "
                  f"depth post{' + Harris (1 thread)' if harris else ''}) of the C oracle, "
                  f"OpenMP {threads} threads, {dt:.1f} s",
    }


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


def aux_kernels(eng, dev, H, W, B, stream, med_ms, med_n, reps=20):
    """HBM rooflines of the memory-bound kernels around k_match, measured after the timed
    region (not part of `value`): k_median_i16 from the timed steps, and k_remap (the
    rectify+gray stage in front of the path) over a batch of B raw 1080p BGR frames."""
    out = {"k_median_i16": hbm_entry("k_median_i16", 11 * H * W * B, med_ms, med_n)}
    rect = make_rectifier(eng, W, H)
    src = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=f"cuda:{dev}")
    dst = torch.empty((B, H, W), dtype=torch.uint8, device=f"cuda:{dev}")
    m1, m2 = rect.device_maps[0], rect.device_maps[1]
    for _ in range(3):
        eng.remap_dev(src.data_ptr(), H, W, 3, 3 * W, m1, m2, H, W, dst.data_ptr(), W,
                      gray_out=True, n_frames=B, src_frame_stride=3 * H * W,
                      dst_frame_stride=H * W, stream=stream)
    torch.cuda.synchronize()
    eng.profile_reset()
    eng.profile(True)
    for _ in range(reps):
        eng.remap_dev(src.data_ptr(), H, W, 3, 3 * W, m1, m2, H, W, dst.data_ptr(), W,
                      gray_out=True, n_frames=B, src_frame_stride=3 * H * W,
                      dst_frame_stride=H * W, stream=stream)
    torch.cuda.synchronize()
    eng.profile(False)
    ms, n = eng.profile_read("remap")
    # algorithmic bytes per output pixel: 6 (map1 + map2) + 3 (BGR source) + 1 (gray out)
    out["k_remap_bgr2gray"] = hbm_entry("k_remap<3,gray>", 10 * H * W * B, ms, n)
    rect.close()
    # occlusion statistics of a rectified gray pair (1 B/px per image read once)
    nb = max(1, H // 48) * max(1, W // 48)
    st = torch.zeros(2 * (2 * nb + 256), dtype=torch.int32, device=f"cuda:{dev}")
    p0 = dst[0].data_ptr()
    p1 = dst[1].data_ptr()
    sp = st.data_ptr()
    eng.profile_reset()
    eng.profile(True)
    for _ in range(reps):
        eng.frame_stats_dev(p0, p1, H, W, 1, W, sp, sp + 8 * nb, sp + 16 * nb, stream=stream)
    torch.cuda.synchronize()
    eng.profile(False)
    ms, n = eng.profile_read("stats")
    out["k_frame_stats"] = hbm_entry("k_frame_stats", 2 * H * W, ms, n)
    # one radix-select pass over a float32 disparity map (4 B/px)
    d = torch.rand((H, W), dtype=torch.float32, device=f"cuda:{dev}")
    eng.profile_reset()
    eng.profile(True)
    for _ in range(reps):
        eng.select_count(d.data_ptr(), H * W, 1)
    eng.profile(False)
    ms, n = eng.profile_read("select")
    out["k_select_hist"] = hbm_entry("k_select_hist", 4 * H * W, ms, n)
    return out


def pmc_entry(workload_key):
    """k_match PMC figures per launch from the committed rocprofv3 summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload_key, {})
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--num-disp", type=int, default=128)
    ap.add_argument("--win", type=int, default=9)
    ap.add_argument("--cost", default="sad", choices=["sad", "ssd", "hog", "sgbm"],
                    help="sad/ssd/hog: the north_star WTA engine; sgbm: the SGBM-3WAY mode")
    ap.add_argument("--frames", type=int, default=16, help="distinct resident frames per rank")
    ap.add_argument("--batch", type=int, default=16,
                    help="frames mode: frames per step, one launch per kernel over the batch "
                         "(sv_depth_map_batch_dev); 1 = one frame per call (latency mode)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no HIP events in the timed loop")
    ap.add_argument("--profile-every", type=int, default=4,
                    help="bracket the kernels of every N-th timed step with HIP events (each "
                         "event record costs a few us of queue time; 1 = every step)")
    ap.add_argument("--mode", default="frames", choices=["frames", "rowtile"],
                    help="frames: independent frames per rank (C4, weak scaling); rowtile: "
                         "one frame row-tiled across ranks + RCCL row gather (C5, strong)")
    ap.add_argument("--gather", action="store_true",
                    help="frames mode: gather every step's disparity maps to rank 0 (RCCL)")
    ap.add_argument("--rectify", action="store_true",
                    help="camera pipeline: raw BGR frames resident in HBM -> rectify+gray "
                         "(k_remap, calibrated CV_16SC2 maps) -> disparity -> median/post")
    ap.add_argument("--no-aux", action="store_true", help="skip the aux-kernel rooflines")
    ap.add_argument("--harris", action="store_true",
                    help="C2: also compute the Harris response of every left frame (k_harris)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo rehearses N>1 with several ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = local % max(1, ndev) if world > 1 else 0
    torch.cuda.set_device(dev)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    comm_dev = "cpu" if gloo else f"cuda:{dev}"

    H, W, D, win = args.height, args.width, args.num_disp, args.win
    F = max(1, args.frames)
    B = max(1, min(args.batch, F))
    F = (F // B) * B
    L, R = stereo_batch(F, H, W, D, seed=1000 * rank)
    dL = torch.from_numpy(L).to(f"cuda:{dev}")
    dR = torch.from_numpy(R).to(f"cuda:{dev}")
    depth = torch.empty((B, H, W), dtype=torch.float32, device=f"cuda:{dev}")
    disp = torch.empty((B, H, W), dtype=torch.float32, device=f"cuda:{dev}")
    norm = torch.empty((B, H, W), dtype=torch.uint8, device=f"cuda:{dev}")
    torch.cuda.synchronize()

    eng = get_engine(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    pL = [dL[i].data_ptr() for i in range(F)]
    pR = [dR[i].data_ptr() for i in range(F)]
    rowtile = args.mode == "rowtile"
    rectify = args.rectify and not rowtile
    if rectify:      # raw camera frames: BGR, unrectified; gray intermediates per batch
        rect = make_rectifier(eng, W, H)
        bL = torch.from_numpy(np.repeat(L[..., None], 3, axis=3)).to(f"cuda:{dev}")
        bR = torch.from_numpy(np.repeat(R[..., None], 3, axis=3)).to(f"cuda:{dev}")
        gL = torch.empty((B, H, W), dtype=torch.uint8, device=f"cuda:{dev}")
        gR = torch.empty((B, H, W), dtype=torch.uint8, device=f"cuda:{dev}")
        m1l, m2l, m1r, m2r, _, _ = rect.device_maps
        torch.cuda.synchronize()
    if rowtile:
        from stereovision_amd.distributed import RowTiledDepthMap, gather_rows
        L0, R0 = stereo_batch(1, H, W, D, seed=4242)      # the SAME frame on every rank
        dL = torch.from_numpy(L0).to(f"cuda:{dev}")
        dR = torch.from_numpy(R0).to(f"cuda:{dev}")
        tile = RowTiledDepthMap(H, W, D, win, cost=args.cost, device=dev,
                                rank=rank, world=world)

    harris = args.harris and not rowtile
    if harris:
        hmap = torch.empty((B, H, W), dtype=torch.float32, device=f"cuda:{dev}")

    def gather(t):
        if world == 1:
            return
        src = t.to(comm_dev) if gloo else t
        if rowtile:
            gather_rows(src, H)
        else:
            out = torch.empty((world,) + tuple(src.shape), dtype=src.dtype, device=src.device)
            dist.all_gather_into_tensor(out, src.unsqueeze(0).contiguous())

    def step(i):
        if rowtile:
            band_disp, _, _, _ = tile.compute(dL[0], dR[0])
            gather(band_disp)
            return
        f = (i * B) % F
        if rectify:
            for src, m1, m2, g in ((bL, m1l, m2l, gL), (bR, m1r, m2r, gR)):
                eng.remap_dev(src[f].data_ptr(), H, W, 3, 3 * W, m1, m2, H, W, g.data_ptr(), W,
                              gray_out=True, n_frames=B, src_frame_stride=3 * H * W,
                              dst_frame_stride=H * W, stream=stream)
            eng.depth_map_batch_dev(gL.data_ptr(), gR.data_ptr(), B, H, W, W, H * W, 0, D, win,
                                    0.3, 2.0, depth.data_ptr(), disp.data_ptr(), norm.data_ptr(),
                                    cost=args.cost, stream=stream)
        elif B == 1:
            eng.depth_map_dev(pL[f], pR[f], H, W, W, 0, D, win, 0.3, 2.0, depth.data_ptr(),
                              disp.data_ptr(), norm.data_ptr(), cost=args.cost, stream=stream)
        else:
            eng.depth_map_batch_dev(pL[f], pR[f], B, H, W, W, H * W, 0, D, win, 0.3, 2.0,
                                    depth.data_ptr(), disp.data_ptr(), norm.data_ptr(),
                                    cost=args.cost, stream=stream)
        if harris:      # one launch over the batch's left frames
            eng.harris_batch_dev(gL.data_ptr() if rectify else pL[f], B, H, W, W, H * W,
                                 hmap.data_ptr(), stream=stream)
        if args.gather:
            gather(disp)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    eng.profile(False)
    eng.profile_reset()
    every = max(1, args.profile_every)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if not args.no_profile and every > 1:
            eng.profile(i % every == 0)        # host-side toggle, no GPU work
        elif i == 0:
            eng.profile(not args.no_profile)
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    eng.profile(False)
    match_ms, match_n = eng.profile_read("sgbm" if args.cost == "sgbm" else "match")
    med_ms, med_n = eng.profile_read("median")
    remap_ms, remap_n = eng.profile_read("remap")
    harris_ms, harris_n = eng.profile_read("harris")
    k_name = "sgbm pipeline (k_sgbm_*)" if args.cost == "sgbm" else "k_match"

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames = args.steps if rowtile else world * args.steps * B
    value = frames / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    npx = H * W * (1 if rowtile else B)
    if rowtile:       # per-launch work is one band (+ median halo rows) of the frame
        npx = (tile.h1 - tile.h0) * W
    k_avg_s = (match_ms / match_n) * 1e-3 if match_n else None
    k_bytes = 4 * npx                          # 2 u8 images read + int16 map written
    frame_bytes = 11 * H * W                   # 2 u8 in; depth f32 + disparity f32 + u8 out
    if harris:
        frame_bytes += 4 * H * W               # + the f32 Harris response
    if rectify:
        frame_bytes = 11 * H * W + 2 * 10 * H * W   # + per camera: map 6 B, BGR 3 B, gray 1 B
    roofline = None
    if k_avg_s:
        achieved = k_bytes / k_avg_s / 1e9
        pmc = pmc_entry(f"{W}x{H}_D{D}_w{win}_{args.cost}" + (f"_b{B}" if B > 1 and not rowtile else ""))
        insts = pmc.get("valu_insts_per_launch")
        roofline = {
            "kernel": k_name, "bound": "hbm", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc.get("hbm_bytes_per_launch"),
            "bytes_per_launch": k_bytes, "avg_launch_us": round(k_avg_s * 1e6, 2),
            "launches": match_n,
            # what actually bounds k_match: VALU issue.  SQ_INSTS_VALU per
            # launch (rocprofv3 PMC, profiles/) over the live launch time, against the
            # full-rate issue peak (1 wave64 instruction / 2 cycles / SIMD); v_sad_u8 and the
            # other VOP3 integer ops issue at half that rate (profiles/r01_valu_rate.txt).
            "valu": {"unit": "wave-instr/s",
                     "achieved": round(insts / k_avg_s) if insts else None,
                     "peak": VALU_ISSUE_PEAK,
                     "frac": round(insts / k_avg_s / VALU_ISSUE_PEAK, 4) if insts else None,
                     "insts_per_launch": insts,
                     "cells_per_s": round(npx * D / k_avg_s)},
            "median_post_avg_us": round(med_ms / med_n * 1e3, 2) if med_n else None,
        }

    result = {
        "metric": "disparity frames/sec + HBM GB/s, 1920x1080 D=128 win=9, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if rowtile else "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic rectified pairs (stereovision_amd.synthetic, seeds per rank)",
        "config": {"workload": (f"{W}x{H} D={D} win={win} {args.cost.upper()} camera pipeline: "
                                "raw BGR frames resident in HBM -> rectify+gray (k_remap) -> "
                                "disparity -> median5 + depth post" if rectify else
                                f"{W}x{H} D={D} win={win} {args.cost.upper()} depth_map path "
                                "(disparity + median5 + depth post" + (" + Harris response"
                                                                        if harris else "") +
                                "), gray inputs resident in HBM"),
                   "harris": harris,
                   "height": H, "width": W, "num_disp": D, "win": win, "cost": args.cost,
                   "frames_resident_per_rank": 1 if rowtile else F,
                   "frames_per_step": 1 if rowtile else B,
                   "parallelism": (f"row-tiled x{world} + RCCL row gather" if rowtile else
                                   f"frame-sharded x{world}" + (" + RCCL gather" if args.gather else "")),
                   "dist_backend": args.dist_backend if world > 1 else None},
        "hbm_gbs_frame_path": round(frame_bytes * value / 1e9, 2),
        # BASELINE.md's fixed roofline formulas, per GPU: 6*H*W algorithmic bytes and
        # H*W*D*win^2 SAD taps per frame against 8.0e12 B/s and 157.3e12 taps/s.  The
        # taps fraction exceeds 1 because running window sums do O(1) work per tap column.
        "baseline_roofline": {
            "fps_per_gpu": round(value / world, 2),
            "achieved_hbm_frac": round(6 * H * W * value / world / 8.0e12, 5),
            "achieved_valu_frac": round(H * W * D * win * win * value / world / 157.3e12, 4)},
        "roofline": roofline,
        "aux_kernels": None,
        "cpu_baseline": None,
    }
    if rectify and remap_n:
        result["aux_kernels"] = {
            "k_remap_bgr2gray": hbm_entry("k_remap<3,gray>", 10 * H * W * B, remap_ms, remap_n)}
        rect.close()
    elif rank == 0 and world == 1 and not rowtile and not args.no_aux:
        try:
            result["aux_kernels"] = aux_kernels(eng, dev, H, W, B, stream, med_ms, med_n)
        except Exception as e:  # reported, never required
            log(f"aux kernels failed: {e}")
    if harris and harris_n:     # 1 B/px gray read + 4 B/px f32 response written
        result["aux_kernels"] = dict(result["aux_kernels"] or {})
        result["aux_kernels"]["k_harris"] = hbm_entry("k_harris_lds", 5 * H * W * B, harris_ms,
                                                       harris_n)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(H, W, D, win, args.cost, args.cpu_seconds,
                                                  harris=harris)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu baseline failed: {e}")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
