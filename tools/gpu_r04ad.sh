#!/bin/bash
# host path after removing the banded A/B: host-path parity tests + the host rate
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "host or registered or create_depth or dropin or pipeline" > gpurun_out/r04ad_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04ad_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/host_rate.py > gpurun_out/host_rate_r04ad.log 2>&1 || exit $?
tail -1 gpurun_out/host_rate_r04ad.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:v for k,v in d.items() if 'pipeline' in k or k=='create_depth_map'})"
