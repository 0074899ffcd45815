#!/bin/bash
# GPU box: rocprofv3 kernel stats of the SGBM pipeline (one frame per call), D=320 w7 and D=128 w9.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-sgprof}"
mkdir -p "$OUT"; cd "$R" || exit 2
export TMPDIR=/tmp
F="--cost sgbm --no-cpu-baseline --no-aux --no-live-pmc --no-host-path --steps 10 --warmup 2 --batch ${SGB:-1} --frames ${SGB:-4}"
for cfg in "d320 --num-disp 320 --win 7" "d128 --num-disp 128 --win 9"; do
  set -- $cfg; name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o sg -- python3 bench.py $F "$@" > "$OUT/$name.log" 2>&1 || { echo "prof $name failed"; exit 1; }
  f=$(find "$OUT/prof_$name" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/${name}_kernel_stats.csv"; echo "== $name"; cut -d, -f1-4 "$OUT/${name}_kernel_stats.csv" | sed 's/sv::(anonymous namespace):://g' | cut -c1-120 | head -14
done
exit 0
