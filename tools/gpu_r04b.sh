#!/bin/bash
# Round 4: record of HEAD (tests, smoke, default bench, rocprofv3 stats) + r<=4 vs r<=5
# v_sad_u32 ring A/B at win 11 (C3).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/round_record.sh r04b || exit $?
B="--no-live-pmc --no-host-path"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_r4.so|$B --win 11" "-|$B --win 11" "abl/libsvhip_r4.so|$B --win 11 --height 480 --width 640 --num-disp 64" "-|$B --win 11 --height 480 --width 640 --num-disp 64"
