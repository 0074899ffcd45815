#!/bin/bash
# The drop-in defaults (NUM_DISP 320, WINDOW_SIZE 7, SAD: the four-row kind, D > 256) against
# the ring kind at D = 256 / 64 on 1080p
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for v in "d320w7|--num-disp 320 --win 7" "d256w7|--num-disp 256 --win 7" "d64w7|--num-disp 64 --win 7" "d320w7b1|--num-disp 320 --win 7 --batch 1"; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux $a > gpurun_out/cfg_$n.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('$n', json.loads(l)['value'], json.loads(l)['roofline']['avg_launch_us']) for l in open('gpurun_out/cfg_$n.log') if l.startswith('{')]"
done
