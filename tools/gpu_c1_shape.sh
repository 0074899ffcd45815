#!/bin/bash
# GPU box: C1 (640x480 D64 w9) with 1/2/3 context streams and 16/32/64-frame batches.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-c1shape}"
mkdir -p "$OUT"; cd "$R" || exit 2
B="--no-host-path --no-cpu-baseline --no-live-pmc --no-aux --height 480 --width 640 --num-disp 64 --win 9"
run() {
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > "$OUT/$name.log" 2>&1 || { tail -5 "$OUT/$name.log"; exit 1; }
  grep "^{" "$OUT/$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['verified'], d['roofline']['avg_launch_us'], d['roofline'].get('median_post_avg_us'))"
}
run s1 --streams 1
run s2 --streams 2
run s3 --streams 3
run b32 --batch 32 --frames 32
run b64 --batch 64 --frames 64
exit 0
