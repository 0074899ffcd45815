#!/bin/bash
# GPU box: host-buffer path, pinned staging copy (default) vs the runtime's pageable H2D
# (SV_HOST_STAGE=0), alternating; parity tests of the path first.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-host2}"
mkdir -p "$OUT"; cd "$R" || exit 2
SV_HOST_STAGE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "host_path or registered or bgr or scaled or dropin" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for v in 1 0; do
    SV_HOST_STAGE=$v SV_HOST_PROFILE=1 timeout -k 10 200 python tools/host_rate.py > "$OUT/rate_${v}_$rep.log" 2>&1 || { tail -5 "$OUT/rate_${v}_$rep.log"; exit 1; }
    echo "stage=$v rep=$rep $(tail -1 "$OUT/rate_${v}_$rep.log" | cut -c1-330)"
  done
done
exit 0
