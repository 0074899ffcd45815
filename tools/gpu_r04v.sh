#!/bin/bash
# HOG histograms: two rows per step with LDS vertical sums (SV_HOG_RP=2) vs one; HOG tests with RP=2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
SV_HOG_RP=2 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "hog or HOG" > gpurun_out/r04v_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04v_pytest.log; [ $rc -ne 0 ] && exit $rc
B="--height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20 --warmup 3"
for v in 1 2; do
  SV_HOG_RP=$v bash tools/prof_kernels.sh hogrp$v $B > gpurun_out/hogrp$v.txt 2>&1 || exit $?
  python3 - $v <<'PY'
import csv, sys, json
v = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof_hogrp{v}/hogrp{v}_kernel_stats.csv")):
    if "hog_hist" in r["Name"]:
        print("RP", v, "hist avg us", float(r["AverageNs"]) / 1000)
for line in open(f"gpurun_out/prof_hogrp{v}/bench.log"):
    if line.startswith("{"):
        print("RP", v, "frames/s", json.loads(line)["value"])
PY
done
