#!/bin/bash
# N>1 rehearsal on a 1-GPU box: ranks share GPU 0, so the process group falls back to the
# file store + host staging (RCCL needs distinct devices).  Same launcher as the driver.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port ${PORT:-29511} bench.py --gpus 2 --steps 100 \
      --warmup 10 --no-cpu-baseline --no-host-path --no-live-pmc --no-aux "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{' "gpurun_out/$name.log" || tail -n 20 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run n2_frames
PORT=29512 run n2_rowtile --mode rowtile
PORT=29513 run n2_frames_gather --gather
