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
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--no-live-pmc --no-host-path --no-cpu-baseline --no-aux"
step pytest_stream 300 python -u -m pytest tests/test_gpu_stream.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_stream 120 python bench.py --steps 200 --warmup 20 $B
step bench_ring 120 env SV_STREAM=0 python bench.py --steps 200 --warmup 20 $B
step bench_stream2 120 python bench.py --steps 200 --warmup 20 $B
step c3_stream 120 python bench.py --steps 100 --warmup 10 --win 11 $B
step d192_stream 120 python bench.py --steps 100 --warmup 10 --num-disp 192 $B
step d192_ring 120 env SV_STREAM=0 python bench.py --steps 100 --warmup 10 --num-disp 192 $B
for f in bench_stream bench_ring bench_stream2 c3_stream d192_stream d192_ring; do
  grep '^{' "$OUT/$f.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['avg_launch_us'], d['verified'])"
done
exit 0
