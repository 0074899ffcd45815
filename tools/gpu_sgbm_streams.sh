#!/bin/bash
# GPU box: SGBM one frame per call with 1/2/3 contexts alternating (frames in flight).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-sgstreams}"
mkdir -p "$OUT"; cd "$R" || exit 2
F="--cost sgbm --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 20 --warmup 3 --batch 1 --frames 8"
for cfg in "d320 --num-disp 320 --win 7" "d128 --num-disp 128 --win 9"; do
  set -- $cfg; name=$1; shift
  for st in 1 2 3; do
    timeout -k 10 200 python bench.py $F --streams $st "$@" > "$OUT/${name}_s$st.log" 2>&1 || { tail -5 "$OUT/${name}_s$st.log"; exit 1; }
    grep "^{" "$OUT/${name}_s$st.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name streams $st', d['value'], d['verified'])"
  done
done
exit 0
