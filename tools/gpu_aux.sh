#!/bin/bash
# GPU box: reduction kernels around the path — their tests, then the bench's aux_kernels
# entries with the wave-aggregated histogram adds on and off.  Usage: bash tools/gpu_aux.sh <tag>
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-aux}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_fusion 300 python -u -m pytest tests/test_fusion.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for a in 2 1 0; do
  step "aux_agg$a" 200 env SV_STATS_AGG=$a python bench.py --steps 20 --warmup 5 --no-live-pmc --no-host-path --no-cpu-baseline
  grep '^{' "$OUT/aux_agg$a.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['aux_kernels'].items():
    if isinstance(v, dict): print('agg$a', k, v['avg_launch_us'], v['frac'])"
done
exit 0
