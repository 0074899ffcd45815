#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench.  Every GPU step has its own time limit;
# after a fault/abort/timeout (exit status other than 0/1) nothing else runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYTEST_ARGS=${PYTEST_ARGS:-"-q"}
step pytest_gpu 600 python -m pytest tests -m gpu $PYTEST_ARGS -p no:cacheprovider
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py ${BENCH_ARGS:-}
