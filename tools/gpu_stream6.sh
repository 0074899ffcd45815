#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-stream}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--no-host-path --no-cpu-baseline --no-aux --steps 200 --warmup 20 --no-live-pmc"
step ring 120 env SV_STREAM=0 python bench.py $B
step prio0 120 env SV_STREAM_DYN=0 SV_STREAM_DBG=16 python bench.py $B
step prio20 120 env SV_STREAM_DYN=20 SV_STREAM_SEG=4 SV_STREAM_DBG=16 python bench.py $B
step plain 120 env SV_STREAM_DYN=20 SV_STREAM_SEG=4 python bench.py $B
rm -f "$OUT/trace.bin"
step trace 120 env SV_STREAM_DYN=0 SV_STREAM_DBG=16 SV_STREAM_TRACE="$OUT/trace.bin" python bench.py --steps 6 --warmup 3 --warmup-seconds 0.5 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux --no-verify
python tools/stream_trace.py "$OUT/trace.bin" | head -3
rm -f "$OUT/trace.bin"
for f in ring prio0 prio20 plain; do
  grep '^{' "$OUT/$f.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$f', d['value'], r['avg_launch_us'], d['verified'])"
done
exit 0
