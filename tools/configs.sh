#!/bin/bash
# Bench lines for every BASELINE.json config on one GPU (C4/C5's multi-GPU runs are the
# driver's); each run under its own time limit, stop on a hard failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -n 5 gpurun_out/cfg_$name.log; exit $rc; fi
  python3 - "$name" gpurun_out/cfg_$name.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"] or {}
        print(f"{sys.argv[1]:>14}: {d['value']:9.1f} frames/s  k_match {r.get('avg_launch_us')} us/launch  "
              f"median {r.get('median_post_avg_us')} us  batch {d['config'].get('frames_per_step')}")
PY
}
run c1_640x480_d64_w9 --height 480 --width 640 --num-disp 64 --win 9
run c2_640x480_d64_w9_harris --height 480 --width 640 --num-disp 64 --win 9 --harris
run c3_1080p_d128_w11 --win 11
run metric_1080p_d128_w9
run metric_batch1 --batch 1
run c5_4k_d256_w15 --height 2160 --width 3840 --num-disp 256 --win 15 --frames 2 --batch 2 --steps 50
run c5_4k_d256_w15_hog --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20
run ssd_1080p_d128_w9 --cost ssd
run ssd_1080p_d128_w11 --cost ssd --win 11
run ssd_1080p_d128_w15 --cost ssd --win 15
run sgbm_1080p_d320_w7 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 40
run sgbm_1080p_d320_w7_3calls --cost sgbm --num-disp 320 --win 7 --batch 1 --streams 3 --steps 40
timeout -k 10 300 python tools/host_rate.py > gpurun_out/host_rate.log 2>&1; tail -n 1 gpurun_out/host_rate.log
timeout -k 10 300 python tools/host_rate.py 480 640 64 9 >> gpurun_out/host_rate.log 2>&1; tail -n 1 gpurun_out/host_rate.log
