#!/bin/bash
# r 5 ring without the left-pack prefetch: no spills, v_sad_u32 for every group width (HEAD)
# vs abl/libsvhip_r5a.so (prefetch, 4 spilled VGPRs at 32 lanes, sub/add at 16 / 64 lanes)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_split_ring.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04w_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04w_pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-live-pmc --no-host-path"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_r5a.so|$B --win 11" "-|$B --win 11" "abl/libsvhip_r5a.so|$B --win 11 --height 480 --width 640 --num-disp 64" "-|$B --win 11 --height 480 --width 640 --num-disp 64" "abl/libsvhip_r5a.so|$B --win 11 --num-disp 192" "-|$B --win 11 --num-disp 192"
