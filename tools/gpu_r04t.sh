#!/bin/bash
# Split ring kind (SAD, 256 < D <= 512): parity tests, then D=320 w7 1080p against the
# four-row kind (SV_RING=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_ring.py tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04t_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04t_pytest.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--no-live-pmc --no-host-path --no-aux --num-disp 320 --win 7"
SKIP_TESTS=1 bash tools/ab_bench.sh "SV_RING=0" "-" "SV_RING=0" "-" || exit $?
bash tools/prof_kernels.sh split320 --num-disp 320 --win 7 --steps 50 --warmup 3
