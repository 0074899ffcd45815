#!/bin/bash
# Whole-disparity post table (lut_shift 4) for integer-cost depth-map batches: GPU suite, then
# A/B against HEAD~ (abl/libsvhip_lut0.so) at the metric config and at the reference default D=320 w7
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/r04af_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04af_pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-live-pmc --no-host-path"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_lut0.so|$B" "-|$B" "abl/libsvhip_lut0.so|$B --num-disp 320 --win 7" "-|$B --num-disp 320 --win 7"
