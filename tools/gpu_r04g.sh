#!/bin/bash
# SGBM kernel breakdown (rocprofv3) at the reference defaults and D=128; HOG band-only test.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
timeout -k 10 200 python -u -m pytest tests/test_multi_gpu_dev.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "hog_band_only" > gpurun_out/r04g_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04g_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_kernels.sh sg320b1 --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 30 --warmup 5 || exit $?
bash tools/prof_kernels.sh sg320b8 --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 6 --warmup 2 || exit $?
bash tools/prof_kernels.sh sg128b1 --cost sgbm --num-disp 128 --win 9 --batch 1 --steps 30 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python tools/pmc_ab.py --kernel k_median_i16 - > gpurun_out/r04g_median_pmc.txt 2>&1; tail -n 20 gpurun_out/r04g_median_pmc.txt
