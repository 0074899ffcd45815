#!/bin/bash
# Round 4: every BASELINE config on one GPU + C2 one stream + SGBM at the reference defaults.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/configs.sh || exit $?
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -n 5 gpurun_out/cfg_$name.log; exit $rc; fi
  python3 - "$name" gpurun_out/cfg_$name.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"] or {}
        aux = (d.get("aux_kernels") or {}).get("k_harris") or {}
        print(f"{sys.argv[1]:>14}: {d['value']:9.1f} frames/s  k_match {r.get('avg_launch_us')} us/launch  "
              f"median {r.get('median_post_avg_us')} us  harris {aux.get('avg_launch_us')} us")
PY
}
run c2_1stream --height 480 --width 640 --num-disp 64 --win 9 --harris --streams 1
run sgbm_d320_w7_b1 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 100 --warmup 10
run sgbm_d320_w7_b8 --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 20 --warmup 3
run sgbm_d128_w9_b1 --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 100 --warmup 10
