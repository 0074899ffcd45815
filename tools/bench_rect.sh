#!/bin/bash
# GPU box: default bench (with aux-kernel rooflines), camera-pipeline bench, rocprofv3 trace
# of the camera pipeline.  Every GPU step has its own limit; stop after any hard failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 2
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$R/gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench_default 300 python bench.py --steps 100 --no-cpu-baseline
step bench_rectify 300 python bench.py --rectify --steps 100 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_rectify 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rect" -o rect -- python3 "$R/bench.py" --rectify --steps 50 --no-cpu-baseline --no-aux
find "$R/gpurun_out/prof_rect" -name "*stats*"
