#!/bin/bash
# SGBM D=320 w7 8-frame batches, repeated (variance check)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2 > gpurun_out/cfg_sgb8_$rep.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('rep $rep', json.loads(l)['value'], json.loads(l)['roofline']['avg_launch_us']) for l in open('gpurun_out/cfg_sgb8_$rep.log') if l.startswith('{')]"
done
bash tools/prof_kernels.sh sgb8 --cost sgbm --num-disp 320 --win 7 --batch 8 --frames 8 --steps 10 --warmup 2
