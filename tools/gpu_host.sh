#!/bin/bash
# GPU box: host-buffer path — its parity tests, the host rate tool (stage timings) for 1, 2
# and 4 row bands, the bench's host_path leg.  Usage: bash tools/gpu_host.sh <tag>
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-host}"
mkdir -p "$OUT"; cd "$R" || exit 2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_host 300 python -u -m pytest tests/test_gpu_parity.py -k "host_path or registered or bgr or scaled or dropin or c5_depth" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for b in 1 2 4; do
  step "host_rate_b$b" 200 env SV_HOST_BANDS=$b SV_HOST_PROFILE=1 python tools/host_rate.py
done
exit 0
