#!/bin/bash
# SGBM reference defaults with calls in flight (3 contexts alternating steps) after the round-4 changes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for v in "s1|--streams 1" "s3|--streams 3" "s2|--streams 2"; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 1 --steps 60 --warmup 5 $a > gpurun_out/cfg_sg_$n.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('sgbm d320 w7 b1 $n', json.loads(l)['value']) for l in open('gpurun_out/cfg_sg_$n.log') if l.startswith('{')]"
done
