#!/bin/bash
# GPU box, round 3 first check: new multi-GPU / verification tests, the whole GPU suite,
# then the bench at the driver's settings and at the long default (warm-up effect).
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03a}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_new 400 python -u -m pytest tests/test_multi_gpu_dev.py tests/test_gpu_parity.py -k "scatter or bench or huge or rows_multi or gathers" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_driver 300 python bench.py --steps 20 --warmup 5
grep '^{' "$OUT/bench_driver.log" | tail -1 > "$OUT/bench_driver.json"
step bench_long 200 python bench.py --steps 200 --warmup 20 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux
step bench_short_again 200 python bench.py --steps 20 --warmup 5 --no-live-pmc --no-host-path --no-cpu-baseline --no-aux
exit 0
