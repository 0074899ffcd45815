#!/bin/bash
# Median: wide tile with column-per-thread loads; A/B vs the old median, and the HOG
# histogram kernel time with LV0 / LV1 (rocprofv3)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "median or m16 or harris or depth_map or scaled" > gpurun_out/r04l_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04l_pytest.log; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 REPS=3 bash tools/ab_lib.sh "abl/libsvhip_med0.so|--no-live-pmc --no-host-path" "-|--no-live-pmc --no-host-path" || exit $?
B="--height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20 --warmup 3"
SV_LIB_PATH=$PWD/abl/libsvhip_lv0.so bash tools/prof_kernels.sh hoglv0 $B || exit $?
bash tools/prof_kernels.sh hoglv1 $B
