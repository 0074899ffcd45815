#!/usr/bin/env python3
"""A/B on the GPU box: the metric config's step as one depth_map_batch_dev call (k_match then
the median on one stream) against a split pipeline — k_match of every step on context A's
stream into one of two int16 buffers, the median + post of that step on context B's stream
(event-ordered), so a step's median runs beside the next step's k_match while k_match
launches never overlap each other.  Prints frames/s, k_match / median launch times (context
events, every 4th step) and whether the two forms' outputs are bit-identical.

Usage: python tools/split_ab.py [--steps 200] [--rounds 2]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from stereovision_amd.engine import Engine, POST_DEPTH  # noqa: E402
from stereovision_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--win", type=int, default=9)
    ap.add_argument("--B", type=int, default=16)
    a = ap.parse_args()
    H, W, D, win, B = a.H, a.W, a.D, a.win, a.B
    n = H * W
    e, em = Engine(0), Engine(0)
    Ls, Rs = [], []
    for f in range(B):
        L, R, _ = stereo_pair(H, W, D, seed=100 + f)
        Ls.append(L)
        Rs.append(R)
    dL, dR = e.dev_alloc(B * n), e.dev_alloc(B * n)
    e.to_device(dL, np.stack(Ls))
    e.to_device(dR, np.stack(Rs))
    outs = [(e.dev_alloc(4 * n * B), e.dev_alloc(4 * n * B), e.dev_alloc(n * B)) for _ in range(2)]
    d16 = [e.dev_alloc(2 * n * B) for _ in range(2)]

    def step_one(i):
        dep, dis, nor = outs[0]
        e.depth_map_batch_dev(dL, dR, B, H, W, W, n, 0, D, win, 0.3, 2.0, dep, dis, nor, cost="sad")

    def step_split(i):
        s = i % 2
        dep, dis, nor = outs[1]
        if i >= 2:
            em.stream_wait_event(s, e.stream)          # buffer s: its median (step i-2) is done
        e.disparity_batch_dev(dL, dR, B, H, W, W, n, 0, D, win, "sad", d16[s], W, n, stream=e.stream)
        e.event_record(s, e.stream)
        e.stream_wait_event(s, em.stream)
        em.median_post_batch_dev(d16[s], B, H, W, POST_DEPTH, dis, d_out_a=dep, d_out_u8=nor,
                                 min_depth=0.3, max_depth=2.0, min_disp_global=0, min_disp=0,
                                 num_disp=D, stream=em.stream)
        em.event_record(s, em.stream)

    def run(step, name):
        for i in range(a.warmup):
            step(i)
        e.synchronize()
        em.synchronize()
        for x in (e, em):
            x.profile_reset()
        t0 = time.perf_counter()
        for i in range(a.steps):
            for x in (e, em):
                x.profile(i % 4 == 0)
            step(a.warmup + i)
        e.synchronize()
        em.synchronize()
        dt = time.perf_counter() - t0
        for x in (e, em):
            x.profile(False)
        mm, mn = e.profile_read("match")
        md, dn = (em if name == "split" else e).profile_read("median")
        print(f"{name:>6}: {a.steps * B / dt:9.1f} frames/s  {dt * 1e3 / a.steps:.4f} ms/step  "
              f"k_match {mm * 1e3 / max(mn, 1):.1f} us/launch ({mn})  median {md * 1e3 / max(dn, 1):.1f} us ({dn})",
              flush=True)

    for r in range(a.rounds):
        run(step_one, "one")
        run(step_split, "split")
    got = [e.to_host(p, (B, H, W), t) for p, t in zip(outs[1], (np.float32, np.float32, np.uint8))]
    exp = [e.to_host(p, (B, H, W), t) for p, t in zip(outs[0], (np.float32, np.float32, np.uint8))]
    same = all(np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(got, exp))
    print("outputs bit-identical:", same, flush=True)


if __name__ == "__main__":
    main()
