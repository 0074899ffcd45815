#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-trace}"
mkdir -p "$OUT"; cd "$R" || exit 2
rm -f "$OUT/trace.bin"
timeout -k 10 120 env SV_STREAM=1 SV_STREAM_TRACE="$OUT/trace.bin" python bench.py --steps 6 --warmup 3 --warmup-seconds 0.5 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux --no-verify > "$OUT/bench_trace.log" 2>&1 || exit $?
python tools/stream_trace.py "$OUT/trace.bin"
timeout -k 10 120 env SV_STREAM=1 SV_STREAM_TRACE="$OUT/trace13.bin" SV_STREAM_DBG=13 python bench.py --steps 6 --warmup 3 --warmup-seconds 0.5 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux --no-verify > "$OUT/bench_trace13.log" 2>&1 || exit $?
python tools/stream_trace.py "$OUT/trace13.bin"
