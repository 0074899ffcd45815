#!/bin/bash
# GPU box: SGBM-3WAY mode — GPU tests, then bench at one frame per call and in frame batches,
# plus rocprofv3 kernel stats of the batched run.  Usage: bash tools/sgbm_ab.sh <tag> [batch]
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sg}
B=${2:-8}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 2
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
FLAGS="--cost sgbm --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 20 --warmup 3"
step test_sgbm 300 python -u -m pytest tests/test_sgbm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_b1 200 python bench.py $FLAGS --batch 1 --frames 8
step bench_b$B 200 python bench.py $FLAGS --batch $B --frames $B
for BB in ${EXTRA_BATCHES:-}; do step bench_b$BB 300 python bench.py $FLAGS --batch $BB --frames $BB; done
step prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o sg -- python3 bench.py $FLAGS --batch $B --frames $B --steps 5 --warmup 1
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && cut -d, -f1-4 "$OUT/kernel_stats.csv" | cut -c1-160 | head -16
exit 0
