#!/bin/bash
# rocprofv3 passes over bench.py (kernel trace + stats, then separate PMC passes).
# Usage on the GPU box: bash tools/profile.sh [tag] [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}; shift
ARGS="--no-cpu-baseline --no-live-pmc --no-host-path --no-aux --steps ${PSTEPS:-200} --warmup 20 $*"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <seconds> <rocprofv3 args...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 "$R/bench.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
if [ ! -f "$R/gpurun_out/counters.txt" ]; then timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1; fi
run trace 300 --kernel-trace --stats
run fetch 300 --pmc FETCH_SIZE
run write 300 --pmc WRITE_SIZE
run sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU
find "$OUT" -name "*.csv" | head -50
