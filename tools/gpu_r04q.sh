#!/bin/bash
# Full GPU suite; A/B of the packed (r 6..7) ring update as one v_sad_u32 (abl/libsvhip_pk0.so =
# pk_sub + pk_add) at C5 and win 13; then every BASELINE config + SGBM defaults on one GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04q_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04q_pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-live-pmc --no-host-path --height 2160 --width 3840 --num-disp 256 --win 15 --frames 2 --batch 2 --steps 50"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_pk0.so|$B" "-|$B" "abl/libsvhip_pk0.so|--no-live-pmc --no-host-path --win 13" "-|--no-live-pmc --no-host-path --win 13" || exit $?
bash tools/configs.sh > gpurun_out/r04q_configs.txt 2>&1; rc=$?; cat gpurun_out/r04q_configs.txt | grep -v "^{" | cut -c1-250; [ $rc -ne 0 ] && exit $rc
for v in "sgbm_d320_w7_b1|--cost sgbm --num-disp 320 --win 7 --batch 1 --steps 60 --warmup 5" "sgbm_d320_w7_b8|--cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2" "sgbm_d128_w9_b1|--cost sgbm --num-disp 128 --win 9 --batch 1 --steps 60 --warmup 5"; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux $a > gpurun_out/cfg_$n.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('$n', json.loads(l)['value']) for l in open('gpurun_out/cfg_$n.log') if l.startswith('{')]"
done
