#!/bin/bash
# A/B the bench under environment variants: bash tools/ab_bench.sh "A=1" "A=2" ...
# (each variant: space-separated VAR=value list; "-" = no extra env).  GPU tests first.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -n 3 gpurun_out/ab_pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -n 5 gpurun_out/ab_$i.log; exit $rc; fi
  python3 - "$v" gpurun_out/ab_$i.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"] or {}
        print(f"{sys.argv[1]:>24}: {d['value']:10.1f} frames/s  k_match {r.get('avg_launch_us')} us  median {r.get('median_post_avg_us')} us")
PY
done
