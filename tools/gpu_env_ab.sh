#!/bin/bash
# GPU box: A/B of an env switch at the metric config (live PMC on), alternating <VAR>=1 / 0
# twice, after the GPU suite (run with the default).  Usage: bash tools/gpu_env_ab.sh <tag> <VAR>
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-envab}"
VAR=${2:?VAR}
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/$name.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r.get('pmc') or {}
print(d['value'], r.get('avg_launch_us'), d.get('verified'), (r.get('valu') or {}).get('insts_per_wave_cell'), p.get('FETCH_SIZE'), p.get('WRITE_SIZE'), p.get('SQ_LDS_BANK_CONFLICT'))" 2>/dev/null || tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
B="--no-host-path --no-cpu-baseline --no-aux --steps 200 --warmup 20"
for rep in 1 2; do
  for v in 1 0; do
    step "metric_${v}_$rep" 240 env $VAR=$v python bench.py $B
  done
done
for v in 1 0; do
  step "c5_$v" 200 env $VAR=$v python bench.py --no-host-path --no-cpu-baseline --no-aux --no-live-pmc --height 2160 --width 3840 --num-disp 256 --win 15 --frames 2 --batch 2 --steps 50
done
exit 0
