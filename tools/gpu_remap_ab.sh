#!/bin/bash
# GPU box: k_remap with / without the XCD-aware row order (SV_XCD_MAP): rectify tests, the
# bench's aux k_remap entry and the camera pipeline (--rectify), alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-remapab}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/$name.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); a=d.get('aux_kernels') or {}; k=a.get('k_remap_bgr2gray') or {}
print(d['value'], d['roofline'].get('avg_launch_us'), d.get('verified'), k.get('avg_launch_us'), k.get('frac'))" 2>/dev/null || tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_rect 300 python -u -m pytest tests/test_rectify.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for rep in 1 2; do
  for v in 1 0; do
    step "aux_${v}_$rep" 240 env SV_XCD_MAP=$v python bench.py --no-host-path --no-cpu-baseline --no-live-pmc --steps 50 --warmup 5
    step "rect_${v}_$rep" 240 env SV_XCD_MAP=$v python bench.py --no-host-path --no-cpu-baseline --no-live-pmc --no-aux --rectify --batch 8 --frames 8 --steps 50 --warmup 5
  done
done
exit 0
