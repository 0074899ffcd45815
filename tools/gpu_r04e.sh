#!/bin/bash
# HOG histogram kernels under rocprofv3 (SV_HOG_VF 0/1/2) + C2 kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
for v in 0 1 2; do
  SV_HOG_VF=$v bash tools/prof_kernels.sh hogvf$v --height 2160 --width 3840 --num-disp 256 --win 15 --cost hog --frames 2 --batch 2 --steps 20 --warmup 3 || exit $?
done
bash tools/prof_kernels.sh c2 --height 480 --width 640 --num-disp 64 --win 9 --harris --steps 100 || exit $?
bash tools/prof_kernels.sh c2s1 --height 480 --width 640 --num-disp 64 --win 9 --harris --streams 1 --steps 100 || exit $?
