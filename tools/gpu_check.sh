#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench.  Every GPU step has its own time limit;
# after a fault/abort/timeout (exit status other than 0/1) nothing else runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-25} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYTEST_ARGS=${PYTEST_ARGS:-"-q"}
step pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest tests -m gpu $PYTEST_ARGS -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
if [ -n "$HOST_RATE" ]; then step host_rate 300 python tools/host_rate.py; fi
step bench 500 python bench.py ${BENCH_ARGS:-}
