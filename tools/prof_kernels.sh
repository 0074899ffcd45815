#!/bin/bash
# rocprofv3 kernel trace + stats of one bench configuration.
# Usage (GPU box): bash tools/prof_kernels.sh <tag> [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o "$TAG" -- python3 "$R/bench.py" --no-cpu-baseline --no-aux --no-live-pmc --no-host-path "$@" > "$OUT/bench.log" 2>&1
rc=$?
echo "== prof $TAG rc=$rc"; tail -n 1 "$OUT/bench.log" | cut -c1-400
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -25
exit $rc
