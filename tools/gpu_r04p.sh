#!/bin/bash
# SGBM batches: vertical path + WTA with one wave per SIMD and 6 steps ahead (SV_SGBM_DEEP=2)
# vs the 2-wave, 2-step form (=1, the default for batches)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_SGBM_DEEP=1" "SV_SGBM_DEEP=2" "SV_SGBM_DEEP=1" "SV_SGBM_DEEP=2" || exit $?
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 4 --frames 4 --steps 20 --warmup 2"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_SGBM_DEEP=1" "SV_SGBM_DEEP=2"
