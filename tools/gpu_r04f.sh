#!/bin/bash
# GPU tests (HOG strip = vertical-first), metric streams / batch sweep, host path profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04f_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04f_pytest.log; [ $rc -ne 0 ] && exit $rc
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
        print(f"{sys.argv[1]:>16}: {d['value']:9.1f} frames/s  k_match {r.get('avg_launch_us')} us  median {r.get('median_post_avg_us')} us  verified {d['verified']}")
PY
}
for rep in 1 2; do
run m_s1 --streams 1
run m_s2 --streams 2
run m_s3 --streams 3
run m_b24 --batch 24 --frames 24
run m_b32 --batch 32 --frames 32
run m_s2b8 --streams 2 --batch 8 --frames 16
done
run c5_hog --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20
SV_HOST_PROFILE=1 timeout -k 10 300 python tools/host_rate.py > gpurun_out/r04f_host.log 2>&1; tail -n 12 gpurun_out/r04f_host.log
