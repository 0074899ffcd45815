#!/bin/bash
# GPU box: SGBM-3WAY at the reference's defaults (1080p D=320 win 7), one frame per call,
# under each pipeline form the library can launch (env switches read by sv_sgbm.hip), so the
# per-call record names what every decomposition measures on the same box.
# Usage: bash tools/sgbm_forms_ab.sh [reps]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
REPS=${1:-2}
FLAGS="--cost sgbm --num-disp 320 --win 7 --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 40 --warmup 5 --batch 1 --frames 8"
run() {  # run <label> <env...>
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py $FLAGS > gpurun_out/sgf.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -n 5 gpurun_out/sgf.log; exit $rc; fi
  python3 - "$label" gpurun_out/sgf.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line)
        print(f"{sys.argv[1]:>44}: {d['value']:8.1f} frames/s per call  ({d['ms_per_step']:.3f} ms)", flush=True)
PY
}
for r in $(seq "$REPS"); do
  run "default (hpath both dirs -> vpath+WTA, deep)" SV_NOOP=1
  run "concurrent hpath || vpath, then WTA" SV_SGBM_VWTA=0
  run "L->R || vpath, then fused R->L+WTA" SV_SGBM_FUSED=1
  run "vpath+WTA 2-wave form (not deep)" SV_SGBM_DEEP=0
  run "16-lane horizontal lines" SV_SGBM_H32=0
done
