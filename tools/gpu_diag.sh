#!/bin/bash
# GPU box: focused diagnosis — the batched-select tests and the 2-rank launcher bench (frames).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-diag}"
mkdir -p "$OUT"; cd "$R" || exit 2
timeout -k 10 200 python -u -m pytest tests/test_fusion.py -k select_batch -v -p no:cacheprovider --timeout 60 --timeout-method thread > "$OUT/select.log" 2>&1
echo "select rc=$?"
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --height 96 --width 400 --num-disp 64 --frames 2 --batch 2 --mode frames --no-live-pmc --no-aux --no-host-path --no-cpu-baseline --hang-timeout 60 > "$OUT/bench2.log" 2>&1
echo "bench2 rc=$?"
exit 0
