#!/bin/bash
# 8 logical GPUs on one device (one process): frames (int16 gather) and C5 row tiling, final round-4 code
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 8 --rehearse --steps 20 --warmup 3 --no-cpu-baseline --no-live-pmc --no-host-path --no-aux > gpurun_out/reh8_frames.log 2>&1 || exit $?
grep '^{' gpurun_out/reh8_frames.log | tail -1 > gpurun_out/reh8_frames.json
timeout -k 10 300 python bench.py --gpus 8 --rehearse --mode rowtile --height 2160 --width 3840 --num-disp 256 --win 15 --steps 20 --warmup 3 --no-cpu-baseline --no-live-pmc --no-host-path --no-aux > gpurun_out/reh8_rowtile.log 2>&1 || exit $?
grep '^{' gpurun_out/reh8_rowtile.log | tail -1 > gpurun_out/reh8_rowtile.json
for f in reh8_frames reh8_rowtile; do python3 -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d.get('verified'), d['distributed'].get('gather_bytes_per_step'))"; done
