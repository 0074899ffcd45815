#!/bin/bash
# final round-4 config table: every BASELINE config + the drop-in default D=320 + SSD + SGBM defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
bash tools/configs.sh > gpurun_out/r04ag_configs.txt 2>&1; rc=$?; grep -v "^{" gpurun_out/r04ag_configs.txt | cut -c1-220; [ $rc -ne 0 ] && exit $rc
for v in "sad_d320_w7|--num-disp 320 --win 7" "ssd_d128_w9|--cost ssd" "sgbm_d320_w7_b1|--cost sgbm --num-disp 320 --win 7 --batch 1 --steps 60 --warmup 5" "sgbm_d320_w7_b8|--cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2" "sgbm_d128_w9_b1|--cost sgbm --num-disp 128 --win 9 --batch 1 --steps 60 --warmup 5"; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux $a > gpurun_out/cfg_$n.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('$n', json.loads(l)['value'], 'frames/s') for l in open('gpurun_out/cfg_$n.log') if l.startswith('{')]"
done
