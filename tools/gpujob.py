#!/usr/bin/env python3
"""One parametrised GPU-box job runner (replaces the per-lease tools/gpu_*.sh scripts).

Usage (on the GPU box, from the repo root):
    python tools/gpujob.py TAG STEP [STEP ...]

Every STEP runs as a child process under its own time limit, with its output in
gpurun_out/TAG/<n>_<name>.log; the job stops at the first step that fails (a GPU fault, an
abort, a time limit or a failing test ends the call: nothing more touches the GPU).  Steps:

    tests[=PYTEST_ARGS]        pytest -m gpu (default: the whole GPU suite)
    smoke                      __graft_entry__.smoke()
    bench[=ARGS]               python bench.py ARGS            (summary line printed)
    trace[=ARGS]               rocprofv3 --kernel-trace --stats over bench.py ARGS
    pmc=C1,C2,..[@ARGS]        one rocprofv3 --pmc pass over bench.py ARGS (counters summed
                               per kernel, mean per dispatch printed)
                               (trace / pmc ARGS may start with NAME=VALUE environment tokens)
    ab=ENV1|ENV2|..[@ARGS]     alternating bench runs under env variants ("-" = none)
    valu[=WPS,..]              tools/microbench/valu_rate at each waves-per-SIMD count
    cmd=SHELL                  any command (bash -c)

A step name may carry a time limit: bench:300=ARGS (seconds; defaults per kind).  ARGS are
split like a shell line.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shlex
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH_QUIET = ["--no-cpu-baseline", "--no-live-pmc", "--no-host-path"]
LIMITS = {"tests": 900, "smoke": 180, "bench": 400, "trace": 400, "pmc": 240, "ab": 900, "valu": 240,
          "cmd": 600}


def run(cmd, log, limit, env=None, cwd=ROOT):
    t0 = time.time()
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, cwd=cwd, env=env,
                             start_new_session=True)
        try:
            rc = p.wait(timeout=limit)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            rc = 124
    return rc, time.time() - t0


def tail(log, n=3, width=400):
    try:
        lines = open(log, errors="replace").read().splitlines()
    except OSError:
        return ""
    return "\n".join(ln[:width] for ln in lines[-n:])


def bench_summary(log):
    for line in reversed(open(log, errors="replace").read().splitlines()):
        if line.startswith("{"):
            d = json.loads(line)
            r = d.get("roofline") or {}
            dist = d.get("distributed") or {}
            out = (f"{d['value']:.1f} {d['unit']}  ms/step {d['ms_per_step']}  k_match "
                   f"{r.get('avg_launch_us')} us  median {r.get('median_post_avg_us')} us  "
                   f"verified {d.get('verified')}")
            if dist:
                out += (f"  backend {dist.get('backend')} gather {dist.get('gather_format')} "
                        f"{dist.get('gather_bytes_per_step')} B/step  gather_us {dist.get('gather_us_per_step')}  "
                        f"expand_us {dist.get('root_expand_us_per_step')}")
            if d.get("host_path"):
                out += f"  host_path {json.dumps(d['host_path'])[:300]}"
            return out
    return "(no bench line)"


def pmc_summary(outdir):
    agg = {}
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            k = (name.split("(")[0][:60], r["Counter_Name"])
            agg.setdefault(k, []).append(float(r["Counter_Value"]))
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:24]
    return "\n".join(f"  {k[0]:<60} {k[1]:<22} mean {sum(v) / len(v):.4g}  n {len(v)}" for k, v in rows)


def split_env(env, args):
    """Leading NAME=VALUE tokens of ARGS -> (env with them set, the remaining args)."""
    toks = shlex.split(args)
    e2 = dict(env)
    while toks and "=" in toks[0] and not toks[0].startswith("-"):
        k, _, v = toks.pop(0).partition("=")
        e2[k] = v
    return e2, toks


def main():
    if len(sys.argv) < 3:
        print(__doc__)
        sys.exit(2)
    tag, steps = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")
    for i, step in enumerate(steps):
        head, _, arg = step.partition("=")
        kind, _, lim = head.partition(":")
        limit = int(lim) if lim else LIMITS.get(kind, 600)
        log = os.path.join(out, f"{i:02d}_{kind}.log")
        extra = ""
        if kind == "tests":
            cmd = [sys.executable, "-u", "-m", "pytest", "-m", "gpu", "-q", "-x", "-p", "no:cacheprovider",
                   "--timeout", "300", "--timeout-method", "thread"] + (shlex.split(arg) if arg else ["tests"])
            rc, dt = run(cmd, log, limit, env)
        elif kind == "smoke":
            rc, dt = run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], log, limit, env)
        elif kind == "bench":
            rc, dt = run([sys.executable, "bench.py"] + shlex.split(arg), log, limit, env)
            if rc == 0:
                extra = bench_summary(log)
        elif kind == "trace":
            d = os.path.join(out, f"{i:02d}_trace")
            e2, bargs = split_env(env, arg)
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "trace",
                   "--", sys.executable, os.path.join(ROOT, "bench.py")] + BENCH_QUIET + ["--no-aux"] + bargs
            rc, dt = run(cmd, log, limit, e2, cwd="/tmp")
            for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
                extra = "\n".join(ln[:160] for ln in open(f).read().splitlines()[:12])
        elif kind == "pmc":
            counters, _, bargs = arg.partition("@")
            d = os.path.join(out, f"{i:02d}_pmc")
            e2, bl = split_env(env, bargs)
            cmd = (["rocprofv3", "--pmc"] + counters.split(",") + ["--output-format", "csv", "-d", d, "-o", "pmc",
                    "--", sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child"] + bl)
            rc, dt = run(cmd, log, limit, e2, cwd="/tmp")
            if rc == 0:
                extra = pmc_summary(d)
        elif kind == "ab":
            variants, _, bargs = arg.partition("@")
            rc, dt, lines = 0, 0.0, []
            for j, v in enumerate(variants.split("|")):
                e2 = dict(env)
                for kv in ([] if v == "-" else v.split()):
                    k, _, val = kv.partition("=")
                    e2[k] = val
                lg = os.path.join(out, f"{i:02d}_ab{j}.log")
                rc, t = run([sys.executable, "bench.py"] + BENCH_QUIET + shlex.split(bargs), lg, limit // 4, e2)
                dt += t
                if rc != 0:
                    lines.append(f"  {v}: rc={rc} {tail(lg)}")
                    break
                lines.append(f"  {v:>28}: {bench_summary(lg)}")
            extra = "\n".join(lines)
        elif kind == "valu":
            rc, dt, text = 0, 0.0, []
            for w in (arg.split(",") if arg else ["1", "2", "3", "4"]):
                e2 = dict(env, WPS=w)
                lg = os.path.join(out, f"{i:02d}_valu_wps{w}.log")
                rc, t = run([os.path.join(ROOT, "tools", "microbench", "valu_rate")], lg, 60, e2)
                dt += t
                if rc != 0:
                    break
            extra = f"  logs in {out}/{i:02d}_valu_wps*.log"
        elif kind == "cmd":
            rc, dt = run(["bash", "-c", arg], log, limit, env)
        else:
            print(f"unknown step kind {kind!r}")
            sys.exit(2)
        print(f"== [{i}] {kind} rc={rc} {dt:.0f}s  {arg[:120]}", flush=True)
        if extra:
            print(extra, flush=True)
        elif rc != 0 or kind in ("tests", "smoke", "cmd"):
            print(tail(log), flush=True)
        if rc != 0:
            print(f"stopping after step {i} ({kind}, rc={rc})", flush=True)
            sys.exit(rc if 0 < rc < 256 else 1)


if __name__ == "__main__":
    main()
