#!/bin/bash
# Median horizontal-pair networks (MQ_W 128) and HOG LDS-atomic vertical sums: full GPU suite,
# then A/B: headline (old median: abl/libsvhip_med0.so) and C5 HOG (LV0: abl/libsvhip_lv0.so vs
# LV1 with the old median: abl/libsvhip_med0.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04k_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04k_pytest.log; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_med0.so|--no-live-pmc --no-host-path" "-|--no-live-pmc --no-host-path" || exit $?
B="--no-live-pmc --no-host-path --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_lv0.so|$B" "abl/libsvhip_med0.so|$B" || exit $?
bash tools/prof_kernels.sh medh --steps 30 --warmup 3
