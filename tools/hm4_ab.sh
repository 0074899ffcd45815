#!/bin/bash
# GPU box: the Harris blocks of the C2 median launch, 248- vs 60-column waves: GPU tests of
# both forms, then the C2 bench alternating the two (SV_HARRIS_MED4).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for v in 1 0; do
  SV_HARRIS_MED4=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "harris or Harris" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/hm4_pytest.log 2>&1
  rc=$?; echo "med4=$v: $(tail -n 1 gpurun_out/hm4_pytest.log)"; [ $rc -ne 0 ] && exit $rc
done
C2="--height 480 --width 640 --num-disp 64 --win 9 --harris"
for rep in 1 2 3; do for v in 0 1; do
  SV_HARRIS_MED4=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-aux --no-host-path --no-live-pmc $C2 > gpurun_out/hm4_b.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/hm4_b.log; exit 1; }
  python3 - $v gpurun_out/hm4_b.log <<'PY'
import json,sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d=json.loads(line); r=d["roofline"]
        print(f"med4={sys.argv[1]}: {d['value']:9.1f} frames/s  k_match {r['avg_launch_us']} us  median+harris {r.get('median_post_avg_us')} us  verified {d['verified']}")
PY
done; done
