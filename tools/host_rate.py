#!/usr/bin/env python3
"""PCIe-inclusive rates of the host-buffer drop-in path and where the time
goes: BGR frames in host memory -> engine -> NumPy outputs, one call per frame as
depth_map.create_depth_map does, plus the pipelined form.  Not the bench metric."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereovision_amd import colormap, depth_map as DM  # noqa: E402
from stereovision_amd.engine import get_engine, host_profile  # noqa: E402
from stereovision_amd.pipeline import DepthMapPipeline  # noqa: E402
from stereovision_amd.synthetic import stereo_pair, to_bgr  # noqa: E402


def rate(fn, n=60, warm=3):
    for i in range(warm):
        fn(i)
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    dt = time.perf_counter() - t0
    return round(n / dt, 1), round(dt * 1e3 / n, 3)


def main():
    H, W, D, win = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (1080, 1920, 128, 9)))
    frames = []
    for s in range(4):
        L, R, _ = stereo_pair(H, W, D, seed=s)
        frames.append((to_bgr(L), to_bgr(R)))
    eng = get_engine(0)
    t = colormap.table("turbo")
    DM.NUM_DISP, DM.WINDOW_SIZE, DM.MIN_DISP = D, win, 0
    out = {"size": f"{W}x{H}", "D": D, "win": win}
    out["engine.depth_map"] = rate(lambda i: eng.depth_map(*frames[i % 4], 0, D, win, 0.3, 2.0))
    out["engine.depth_map_color"] = rate(lambda i: eng.depth_map_color(*frames[i % 4], 0, D, win, 0.3, 2.0, t))
    bufs = (np.zeros((H, W), np.float32), np.zeros((H, W), np.float32), np.zeros((H, W, 3), np.uint8))
    out["engine.depth_map_color reused outputs"] = rate(
        lambda i: eng.depth_map_color(*frames[i % 4], 0, D, win, 0.3, 2.0, t, out=bufs))
    out["create_depth_map"] = rate(lambda i: DM.create_depth_map(*frames[i % 4]))
    u8 = np.random.default_rng(0).integers(0, 256, (H, W), dtype=np.uint8)
    out["host colormap.apply"] = rate(lambda i: colormap.apply(u8, "turbo"), n=10)
    out["host alloc+touch 22.8MB outputs"] = rate(
        lambda i: (np.empty((H, W), np.float32).fill(0), np.empty((H, W), np.float32).fill(0),
                   np.empty((H, W, 3), np.uint8).fill(0)), n=30)
    a = np.random.default_rng(1).integers(0, 256, 6 * H * W, dtype=np.uint8)
    b = np.empty_like(a)
    out["host memcpy 12.4MB warm"] = rate(lambda i: np.copyto(b, a), n=30)
    # the in-flight sweep: uncapped depths (cap=False) with the host-side stage times per call
    # (sv_host_profile: prepare, stage+issue, wait for the first piece, expand, wait for the
    # rest, total), and the capped pipeline a caller gets for the same request
    # the in-flight sweep: uncapped depths (cap=False) and the capped pipeline a caller gets for
    # the same request; per configuration 40 warm-up frames, then 3 timed runs of 300 frames
    # (frames/s of each and their median) with the host-side stage times per call
    # (sv_host_profile: prepare, stage+issue, wait for the first piece, expand, wait for the
    # rest, total) over the three
    depths = [int(v) for v in os.environ.get("SV_DEPTHS", "1,2,3,4,5,6,8").split(",")]
    for depth in depths:
        for cap in ((False, True) if depth > 4 else (False,)):
            pipe = DepthMapPipeline(D, win, depth=depth, cap=cap)
            try:
                def run(n):
                    futs = []
                    t0 = time.perf_counter()
                    for i in range(n):
                        futs.append(pipe.submit(*frames[i % 4]))
                        if len(futs) > pipe.depth:
                            futs.pop(0).result()
                    for f in futs:
                        f.result()
                    return n / (time.perf_counter() - t0)
                run(40)
                host_profile(enable=True, reset=True)
                reps = [round(run(300), 1) for _ in range(3)]
                st = host_profile(enable=False, reset=True)
                key = f"pipeline depth {depth}" + (f" capped to {pipe.depth}" if cap else "")
                out[key] = {"frames_per_s": sorted(reps)[1], "runs": reps,
                            "ms_per_frame": round(1e3 / sorted(reps)[1], 3),
                            "per_call_ms": {k: (round(v, 3) if v is not None else None)
                                            for k, v in st.items() if k != "calls"}}
            finally:
                pipe.close()
    out["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    out["cpu_count"] = os.cpu_count()
    out["affinity"] = len(os.sched_getaffinity(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
