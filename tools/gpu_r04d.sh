#!/bin/bash
# Round 4: GPU tests, every config, C2 one stream, HOG histogram A/B, SGBM at the reference defaults.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04d_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04d_pytest.log; [ $rc -ne 0 ] && exit $rc
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
        print(f"{sys.argv[1]:>16}: {d['value']:9.1f} frames/s  k_match {r.get('avg_launch_us')} us/launch  "
              f"median {r.get('median_post_avg_us')} us  harris {aux.get('avg_launch_us', aux.get('fused', '-'))[:20]}  verified {d['verified']}")
PY
}
run c1 --height 480 --width 640 --num-disp 64 --win 9
run c2 --height 480 --width 640 --num-disp 64 --win 9 --harris
run c2_1stream --height 480 --width 640 --num-disp 64 --win 9 --harris --streams 1
run c3 --win 11
run metric
run metric_b1 --batch 1
run c5 --height 2160 --width 3840 --num-disp 256 --win 15 --frames 2 --batch 2 --steps 50
for v in 0 1 2; do
  SV_HOG_VF=$v run c5_hog_vf$v --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20
done
SV_HOG_VF=1 run c5_hog_vf1b --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20
SV_HOG_VF=0 run c5_hog_vf0b --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20
run sgbm_d320_w7_b1 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 100 --warmup 10
run sgbm_d320_w7_b8 --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 20 --warmup 3
run sgbm_d128_w9_b1 --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 100 --warmup 10
