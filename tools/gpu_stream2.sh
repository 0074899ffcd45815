#!/bin/bash
# GPU box: stream kind — parity tests, then the metric bench (ring vs stream) and timing-only
# ablations of the stream kind (SV_STREAM_DBG: 1 no producer, 4 no bursts, 8 no stores).
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-stream}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--no-host-path --no-cpu-baseline --no-aux --steps 200 --warmup 20"
step pytest_stream 300 python -u -m pytest tests/test_gpu_stream.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step ring 200 env SV_STREAM=0 python bench.py $B
step stream 200 python bench.py $B
step abl1 120 env SV_STREAM_DBG=1 python bench.py $B --no-verify --no-live-pmc
step abl4 120 env SV_STREAM_DBG=4 python bench.py $B --no-verify --no-live-pmc
step abl8 120 env SV_STREAM_DBG=8 python bench.py $B --no-verify --no-live-pmc
step abl13 120 env SV_STREAM_DBG=13 python bench.py $B --no-verify --no-live-pmc
for f in ring stream abl1 abl4 abl8 abl13; do
  grep '^{' "$OUT/$f.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; v=r['valu']
print('$f', d['value'], r['avg_launch_us'], d['verified'], v.get('insts_per_wave_cell'), v.get('frac'), r['pmc'].get('SQ_INSTS_LDS'), r['pmc'].get('SQ_LDS_BANK_CONFLICT'))"
done
exit 0
