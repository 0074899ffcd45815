#!/bin/bash
# GPU box: the ring kernel with / without the deferred second-pair reduction (SV_RING_DEFER):
# the GPU suite first (default = deferred), then A/B bench runs alternating the two, at the
# metric config, C3 (win 11, r 5: never deferred), D=192 and C5 (r 7).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-ringab}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r.get('avg_launch_us'), d.get('verified'), (r.get('valu') or {}).get('insts_per_wave_cell'))" 2>/dev/null || tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
B="--no-host-path --no-cpu-baseline --no-aux --steps 200 --warmup 20"
for rep in 1 2; do
  for d in 1 0; do
    step "metric_d${d}_$rep" 200 env SV_RING_DEFER=$d python bench.py $B
  done
done
for d in 1 0; do
  step "d192_d$d" 200 env SV_RING_DEFER=$d python bench.py $B --num-disp 192 --no-live-pmc
  step "c5_d$d" 200 env SV_RING_DEFER=$d python bench.py --no-host-path --no-cpu-baseline --no-aux --no-live-pmc --height 2160 --width 3840 --num-disp 256 --win 15 --frames 2 --batch 2 --steps 50
  step "c1_d$d" 200 env SV_RING_DEFER=$d python bench.py --no-host-path --no-cpu-baseline --no-aux --no-live-pmc --height 480 --width 640 --num-disp 64 --win 9
done
exit 0
