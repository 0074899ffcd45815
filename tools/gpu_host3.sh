#!/bin/bash
# GPU box: host-buffer path with the runtime's pageable H2D, 1 / 2 / 4 row bands (SV_HOST_BANDS).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-host4}"
mkdir -p "$OUT"; cd "$R" || exit 2
for rep in 1 2; do
  for b in 1 2 4; do
    SV_HOST_BANDS=$b timeout -k 10 200 python tools/host_rate.py > "$OUT/rate_b${b}_$rep.log" 2>&1 || { tail -5 "$OUT/rate_b${b}_$rep.log"; exit 1; }
    tail -1 "$OUT/rate_b${b}_$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bands $b rep $rep', d['create_depth_map'], d['engine.depth_map_color reused outputs'], d['pipeline depth 4'])"
  done
done
exit 0
