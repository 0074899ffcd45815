#!/usr/bin/env python3
"""PMC A/B of the disparity kernel under environment variants (GPU box; a diagnostic aid).

Usage: python tools/pmc_ab.py [--kernel k_match] [--args "..."] VAR=val[,VAR=val] ... ("-" = none)

Each variant runs one separate rocprofv3 --pmc pass per counter group over a short bench.py
child (6 steps), every pass time-limited; prints the mean per dispatch of each counter for
kernels whose name contains --kernel.  SQ_* cycle counters count quad-cycles on gfx950.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"],
    ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"],
]


def run_variant(envs, kernel, bench_args, timeout):
    env = dict(os.environ)
    for kv in envs:
        k, v = kv.split("=", 1)
        env[k] = v
    tmp = tempfile.mkdtemp(prefix="sv_pmcab_", dir=os.environ.get("TMPDIR", "/tmp"))
    env["TMPDIR"] = tmp
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--steps", "6", "--warmup", "2",
             *bench_args]
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    agg = {}
    try:
        for gi, counters in enumerate(GROUPS):
            d = os.path.join(tmp, f"g{gi}")
            cmd = [rocprof, "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", f"g{gi}", "--", *child]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=tmp,
                                 start_new_session=True, env=env)
            try:
                _, err = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return {"error": f"pass {gi} timed out"}
            if p.returncode != 0:
                return {"error": f"pass {gi} rc={p.returncode}: {err.decode(errors='replace')[-400:]}"}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if kernel in r["Kernel_Name"]:
                        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_match")
    ap.add_argument("--args", default="")
    ap.add_argument("--timeout", type=int, default=90)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    for v in a.variants:
        envs = [] if v == "-" else v.split(",")
        res = run_variant(envs, a.kernel, a.args.split(), a.timeout)
        if "error" in res:
            print(f"{v}: {res['error']}", flush=True)
            sys.exit(1)
        w = res.get("SQ_WAVES", 1) or 1
        line = {"variant": v, **{k: round(x) for k, x in res.items()}}
        if "SQ_WAVE_CYCLES" in res:
            wc = res["SQ_WAVE_CYCLES"]
            line["frac"] = {k[3:]: round(res[k] / wc, 3) for k in res
                            if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) and wc}
            line["wave_cycles_per_wave"] = round(4 * wc / w)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
