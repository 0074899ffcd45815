#!/usr/bin/env python3
"""A/B of the host-buffer drop-in path under environment variants (GPU box).

Usage: python tools/host_ab.py [--rounds 2] VAR=val[,VAR=val] ... ("-" = no extra env)

Each variant runs bench.host_path (create_depth_map one call per frame, its per-call stage
times, and DepthMapPipeline with 4 frames in flight) in a child process; variants alternate
for --rounds rounds so box drift hits all of them alike."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = ("import sys, json; sys.path.insert(0, {root!r}); import bench; "
         "print('@@' + json.dumps(bench.host_path({H}, {W}, {D}, {win})))")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--size", default="1080,1920,128,9")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    H, W, D, win = (int(v) for v in a.size.split(","))
    for r in range(a.rounds):
        for v in a.variants:
            env = dict(os.environ)
            for kv in ([] if v == "-" else v.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val
            p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, H=H, W=W, D=D, win=win)],
                               capture_output=True, text=True, timeout=240, env=env)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("@@")]
            if p.returncode != 0 or not line:
                print(f"{v}: rc={p.returncode} {p.stderr[-500:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[-1][2:])
            pc = d.get("per_call", {})
            print(f"round {r} {v:>40}: single {d['value']:7.1f}/s  pipelined {d.get('pipelined', {}).get('value')}/s  "
                  f"wall {pc.get('wall_us')} us  h2d {pc.get('h2d_us')}  kernels {pc.get('kernel_us')}  "
                  f"d2h {pc.get('d2h_us')} ({pc.get('d2h_path')})  host {pc.get('host_ms')}", flush=True)


if __name__ == "__main__":
    main()
