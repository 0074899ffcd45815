#!/bin/bash
# GPU box: per-row measurements, default bench, rocprofv3 kernel trace of the default bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG=${TAG:-r01g}
timeout -k 10 400 python tools/bench_rows.py --out gpurun_out/rows_$TAG.jsonl > gpurun_out/rows_$TAG.log 2>&1 || { echo "rows failed"; tail -20 gpurun_out/rows_$TAG.log; exit 1; }
echo "== rows ok"
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo "== bench ok"; cut -c1-300 gpurun_out/bench_$TAG.json
bash tools/prof_kernels.sh $TAG --steps 100 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
echo "== prof ok"
