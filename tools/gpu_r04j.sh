#!/bin/bash
# SGBM cost chunk A/B (r 3: CL 16 vs 24) + SGBM tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
timeout -k 10 300 python -u -m pytest tests/test_sgbm.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04j_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04j_pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-live-pmc --no-host-path --cost sgbm --num-disp 320 --win 7"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_cl16.so|$B --batch 1 --steps 60 --warmup 5" "-|$B --batch 1 --steps 60 --warmup 5" "abl/libsvhip_cl16.so|$B --batch 8 --frames 8 --steps 10 --warmup 2" "-|$B --batch 8 --frames 8 --steps 10 --warmup 2"
