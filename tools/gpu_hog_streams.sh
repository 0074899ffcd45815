#!/bin/bash
# GPU box: C5 HOG (3840x2160 D256 w15, 2-frame batches) with 1, 2 and 3 contexts/streams
# alternating steps (one step's histograms beside the previous step's match).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-hogs}"
mkdir -p "$OUT"; cd "$R" || exit 2
for st in 1 2 3; do
  timeout -k 10 200 python bench.py --no-host-path --no-cpu-baseline --no-aux --no-live-pmc --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 4 --batch 2 --steps 20 --streams $st > "$OUT/hog_s$st.log" 2>&1 || { tail -5 "$OUT/hog_s$st.log"; exit 1; }
  grep "^{" "$OUT/hog_s$st.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $st', d['value'], d['verified'], d['roofline'].get('avg_launch_us'))"
done
exit 0
