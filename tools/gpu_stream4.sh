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
step ring 120 env SV_STREAM=0 python bench.py $B
for k in 3 4 6 8 12 16 26; do
  step "bod$k" 120 env SV_STREAM_BODIES=$k python bench.py $B
done
step bod6_1 120 env SV_STREAM_BODIES=6 SV_STREAM_DBG=1 python bench.py $B --no-verify
step bod6_13 120 env SV_STREAM_BODIES=6 SV_STREAM_DBG=13 python bench.py $B --no-verify
for f in ring bod3 bod4 bod6 bod8 bod12 bod16 bod26 bod6_1 bod6_13; do
  grep '^{' "$OUT/$f.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$f', d['value'], r['avg_launch_us'], d['verified'])"
done
exit 0
