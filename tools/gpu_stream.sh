#!/bin/bash
# GPU box: stream-kind check — its parity tests, then the metric bench with and without it.
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-stream}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--no-host-path --no-cpu-baseline --no-aux"
step pytest_stream 300 python -u -m pytest tests/test_gpu_stream.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_stream 200 env SV_STREAM=1 python bench.py --steps 200 --warmup 20 $B
step bench_ring 200 env SV_STREAM=0 python bench.py --steps 200 --warmup 20 $B
step d192_stream 120 env SV_STREAM=1 python bench.py --steps 100 --warmup 10 --num-disp 192 $B --no-live-pmc
step d192_ring 120 env SV_STREAM=0 python bench.py --steps 100 --warmup 10 --num-disp 192 $B --no-live-pmc
for f in bench_stream bench_ring d192_stream d192_ring; do
  grep '^{' "$OUT/$f.log" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; v=r['valu']
print('$f', d['value'], r['avg_launch_us'], d['verified'], v.get('insts_per_wave_cell'), v.get('frac'), r['pmc'].get('SQ_WAVES'), r['pmc'].get('SQ_INSTS_LDS'), r['pmc'].get('SQ_LDS_BANK_CONFLICT'))"
done
exit 0
