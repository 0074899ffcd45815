#!/bin/bash
# SGBM single-frame path kernels: deeper prefetch (SV_SGBM_DEEP=1: vertical+WTA one wave per
# SIMD, horizontal two waves with ~1.5-2x the steps ahead) vs the 2-wave defaults (=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sgbm.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04o_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04o_pytest.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 60 --warmup 5"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_SGBM_DEEP=0" "SV_SGBM_DEEP=1" "SV_SGBM_DEEP=0" "SV_SGBM_DEEP=1" || exit $?
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 60 --warmup 5"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_SGBM_DEEP=0" "SV_SGBM_DEEP=1" || exit $?
SV_SGBM_DEEP=1 bash tools/prof_kernels.sh sgdeep2 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 30 --warmup 3
