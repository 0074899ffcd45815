#!/bin/bash
# GPU box: SGBM A/B of an env switch: GPU tests, then D=128 w9 and the reference defaults
# D=320 w7, one frame per call and 8-frame batches, with <VAR>=1 and <VAR>=0.
# Usage: bash tools/gpu_sgbm_ab.sh <tag> <VAR>
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-sgab}"
VAR=${2:-SV_SGBM_H32}
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'].get('avg_launch_us'), d.get('verified'))" 2>/dev/null || tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
F="--cost sgbm --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 20 --warmup 3"
step test_sgbm 300 env $VAR=1 python -u -m pytest tests/test_sgbm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for p in 1 0; do
  step "d128_b1_$p" 200 env $VAR=$p python bench.py $F --batch 1 --frames 8
  step "d320_b1_$p" 200 env $VAR=$p python bench.py $F --batch 1 --frames 8 --num-disp 320 --win 7
  step "d320_b4_$p" 200 env $VAR=$p python bench.py $F --batch 4 --frames 8 --num-disp 320 --win 7
done
exit 0
