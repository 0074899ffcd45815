#!/bin/bash
# host path A/B: runtime pageable H2D (default) vs own pinned staging copied by the calling thread
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
for v in 0 2 0 2; do
  SV_HOST_STAGE=$v timeout -k 10 200 python tools/host_rate.py > gpurun_out/r04h_host_$v.log 2>&1 || exit $?
  echo "SV_HOST_STAGE=$v"; python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/r04h_host_$v.log') if x.startswith('{')][-1])
print({k: v for k, v in d.items() if k.startswith(('create', 'engine', 'pipeline'))})"
done
