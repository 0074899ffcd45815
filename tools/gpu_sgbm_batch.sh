#!/bin/bash
# GPU box: SGBM frame batches, fused R->L/WTA (SV_SGBM_FUSED=1) vs the unfused pipeline
# (=0, vertical path + WTA fused for D > 128), D=320 w7 and D=128 w9.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-sgbatch}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'].get('avg_launch_us'))" 2>/dev/null || tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
F="--cost sgbm --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 10 --warmup 2"
for f in 1 0; do
  step "d320_b8_f$f" 200 env SV_SGBM_FUSED=$f python bench.py $F --batch 8 --frames 8 --num-disp 320 --win 7
  step "d320_b16_f$f" 300 env SV_SGBM_FUSED=$f python bench.py $F --batch 16 --frames 16 --num-disp 320 --win 7
  step "d128_b8_f$f" 200 env SV_SGBM_FUSED=$f python bench.py $F --batch 8 --frames 8
done
exit 0
