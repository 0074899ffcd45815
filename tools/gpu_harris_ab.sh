#!/bin/bash
# GPU box: Harris kernels — tests, then C2 (640x480 D64 w9 + Harris) and 1080p + Harris with
# the DPP kernel and the LDS-tile kernel (SV_HARRIS=lds).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-harris}"
mkdir -p "$OUT"; cd "$R" || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k harris -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for m in dpp dpp1 lds; do
  hb=8
  for cfg in "c2 --height 480 --width 640 --num-disp 64 --win 9" "hd --height 1080 --width 1920 --num-disp 128 --win 9"; do
    set -- $cfg; name=$1; shift
    SV_HARRIS=$m SV_HARRIS_HB=$hb timeout -k 10 200 python bench.py --no-host-path --no-cpu-baseline --no-live-pmc --harris "$@" > "$OUT/${name}_$m.log" 2>&1 || { tail -5 "$OUT/${name}_$m.log"; exit 1; }
    grep "^{" "$OUT/${name}_$m.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['aux_kernels']['k_harris']; print('$name $m', d['value'], d['verified'], k['avg_launch_us'], k['frac'])"
  done
done
exit 0
