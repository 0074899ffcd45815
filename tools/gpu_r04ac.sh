#!/bin/bash
# HOG strip kernel with wave-scope LDS ordering instead of __syncthreads: HOG tests + kernel time
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "hog or HOG" > gpurun_out/r04ac_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04ac_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_kernels.sh hogws --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20 --warmup 3 > gpurun_out/hogws.txt 2>&1 || exit $?
python3 - <<'PY'
import csv, json
for r in csv.DictReader(open("gpurun_out/prof_hogws/hogws_kernel_stats.csv")):
    print(r["Name"][:50], float(r["AverageNs"]) / 1000)
for line in open("gpurun_out/prof_hogws/bench.log"):
    if line.startswith("{"):
        print("frames/s", json.loads(line)["value"])
PY
