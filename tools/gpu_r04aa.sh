#!/bin/bash
# SGBM D=128 w9 one frame per call: vertical path + WTA fused with the deep prefetch (SV_SGBM_VWTA=2)
# vs the concurrent vertical || horizontal form (default at D <= 128); SGBM tests with VWTA=2 first
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
SV_SGBM_VWTA=2 timeout -k 10 400 python -u -m pytest tests/test_sgbm.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04aa_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04aa_pytest.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 60 --warmup 5"
SKIP_TESTS=1 bash tools/ab_bench.sh "-" "SV_SGBM_VWTA=2" "-" "SV_SGBM_VWTA=2" || exit $?
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 64 --win 9 --height 480 --width 640 --batch 1 --steps 100 --warmup 5"
SKIP_TESTS=1 bash tools/ab_bench.sh "-" "SV_SGBM_VWTA=2"
