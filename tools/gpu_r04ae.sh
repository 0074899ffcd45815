#!/bin/bash
# u8 disparity-index gather: the new entry point's test, the launched 2-rank bench (both gather
# formats) and the one-process rehearsal, then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multi_gpu_dev.py -m gpu -q -x -p no:cacheprovider --timeout 250 --timeout-method thread -k "d8 or two_ranks or rehearsal" > gpurun_out/r04ae_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04ae_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/r04ae_full.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04ae_full.log; exit $rc
