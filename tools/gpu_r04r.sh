#!/bin/bash
# SGBM cost kernel: window sums by v_sad_u32 (sg1: 2 waves/SIMD) and 3 waves/SIMD at r 3 (HEAD)
# vs the pk_sub/pk_add form (sg0); SGBM tests first
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sgbm.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04r_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04r_pytest.log; [ $rc -ne 0 ] && exit $rc
B1="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 60 --warmup 5"
B8="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2"
B9="--no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 60 --warmup 5"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_sg0.so|$B1" "abl/libsvhip_sg1.so|$B1" "-|$B1" "abl/libsvhip_sg0.so|$B8" "-|$B8" "abl/libsvhip_sg0.so|$B9" "-|$B9" || exit $?
bash tools/prof_kernels.sh sgcost3 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 30 --warmup 3
