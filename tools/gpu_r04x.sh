#!/bin/bash
# SSD cost at the metric config and C3 (documentation: the SSD kind is one row per wave)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for v in "ssd_w9|--cost ssd" "ssd_w11|--cost ssd --win 11" "sad_w9|" ; do
  n=${v%%|*}; a=${v#*|}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-pmc --no-host-path --no-aux $a > gpurun_out/cfg_$n.log 2>&1 || exit $?
  python3 -c "import json,sys; [print('$n', json.loads(l)['value'], json.loads(l)['roofline']['avg_launch_us']) for l in open('gpurun_out/cfg_$n.log') if l.startswith('{')]"
done
