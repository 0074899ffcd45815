#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-stream}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--no-host-path --no-cpu-baseline --no-aux --steps 200 --warmup 20 --no-live-pmc"
step pytest_stream 300 python -u -m pytest tests/test_gpu_stream.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 1 "$OUT/pytest_stream.log"
step ring 120 env SV_STREAM=0 python bench.py $B
for cfg in "0 2" "10 2" "20 2" "20 4"; do
  set -- $cfg
  step "dyn$1_seg$2" 120 env SV_STREAM_DYN=$1 SV_STREAM_SEG=$2 python bench.py $B
done
step abl13 120 env SV_STREAM_DYN=0 SV_STREAM_DBG=13 python bench.py $B --no-verify
step abl1 120 env SV_STREAM_DYN=0 SV_STREAM_DBG=1 python bench.py $B --no-verify
rm -f "$OUT/trace.bin"
step trace 120 env SV_STREAM_DYN=0 SV_STREAM_TRACE="$OUT/trace.bin" python bench.py --steps 6 --warmup 3 --warmup-seconds 0.5 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux --no-verify
python tools/stream_trace.py "$OUT/trace.bin" | head -3
rm -f "$OUT/trace.bin"
for f in ring dyn0_seg2 dyn10_seg2 dyn20_seg2 dyn20_seg4 abl13 abl1; do
  grep '^{' "$OUT/$f.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$f', d['value'], r['avg_launch_us'], d['verified'])"
done
exit 0
