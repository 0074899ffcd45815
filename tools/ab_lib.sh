#!/bin/bash
# A/B libraries and bench args: bash tools/ab_lib.sh "<SV_LIB_PATH or ->|<bench args>" ...
# GPU tests of the in-tree library first (skip with SKIP_TESTS=1); every step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -n 3 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
REPS=${REPS:-2}
for r in $(seq $REPS); do
i=0
for v in "$@"; do
  i=$((i+1))
  lib=${v%%|*}; args=${v#*|}
  if [ "$lib" = "-" ]; then unset SV_LIB_PATH; else export SV_LIB_PATH="$PWD/$lib"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-aux $args > gpurun_out/ab_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -n 5 gpurun_out/ab_$i.log; exit $rc; fi
  python3 - "$v" gpurun_out/ab_$i.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"] or {}
        print(f"{sys.argv[1]:>40}: {d['value']:10.1f} frames/s  k_match {r.get('avg_launch_us')} us  median {r.get('median_post_avg_us')} us")
PY
done
done
