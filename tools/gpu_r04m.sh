#!/bin/bash
# HOG strip rows per wave (SV_HOG_ROWS) sweep at C5 HOG, rocprofv3 per variant
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
B="--height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20 --warmup 3"
for v in 32 48 64 96 128; do
  SV_HOG_ROWS=$v bash tools/prof_kernels.sh hogrows$v $B > gpurun_out/hogrows$v.txt 2>&1 || exit $?
  python3 - $v <<'PY'
import csv, sys, json
v = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof_hogrows{v}/hogrows{v}_kernel_stats.csv")):
    if "hog_hist" in r["Name"]:
        print(v, "hist avg us", float(r["AverageNs"]) / 1000)
for line in open(f"gpurun_out/prof_hogrows{v}/bench.log"):
    if line.startswith("{"):
        print(v, "frames/s", json.loads(line)["value"])
PY
done
