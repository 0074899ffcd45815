#!/bin/bash
# SSD on the ring kind (win 5..9, D <= 256): parity tests (every SSD case of the parity suite),
# then 1080p D=128 SSD w9 / w7 against the one-row SSD kind (SV_RING=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_ssd_ring.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04y_pytest.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost ssd"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_RING=0" "-" "SV_RING=0" "-" || exit $?
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --cost ssd --win 7 --height 480 --width 640 --num-disp 64"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_RING=0" "-"
