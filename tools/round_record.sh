#!/bin/bash
# GPU box: the round's record — GPU tests, smoke, default bench (live PMC, host path, CPU
# baseline), rocprofv3 kernel stats of the default bench.  Every GPU step time-limited;
# stops after a fault/abort/timeout.  Usage: bash tools/round_record.sh <tag>
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-rXX}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python bench.py
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
bash tools/prof_kernels.sh "$TAG" --steps 100 > "$OUT/prof.log" 2>&1
echo "== prof rc=$?"; tail -n 6 "$OUT/prof.log" | cut -c1-200
f=$(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
exit 0
