#!/bin/bash
# Round 4: k_match A/B (v_sad_u32 window update vs the sub/add form) + one-process N-GPU
# rehearsals (N logical GPUs on this box's device: frames m16 / full, rowtile C5).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r04a
B="--no-live-pmc --no-host-path"
SKIP_TESTS=1 REPS=2 bash tools/ab_lib.sh "abl/libsvhip_base.so|$B" "-|$B" \
  "abl/libsvhip_base.so|$B --height 480 --width 640 --num-disp 64" "-|$B --height 480 --width 640 --num-disp 64" \
  "abl/libsvhip_base.so|$B --num-disp 192" "-|$B --num-disp 192" || exit $?
run() {   # name, args
  timeout -k 10 240 python bench.py --no-live-pmc --no-host-path --no-cpu-baseline --no-aux --hang-timeout 200 "${@:2}" \
    > gpurun_out/r04a/$1.json 2> gpurun_out/r04a/$1.err
  rc=$?; echo "$1 rc=$rc"; tail -c 600 gpurun_out/r04a/$1.json; echo
  return $rc
}
run reh8_frames_m16 --gpus 8 --rehearse --steps 40 --warmup 5 && \
run reh8_frames_full --gpus 8 --rehearse --steps 40 --warmup 5 --root-outputs full && \
run reh8_rowtile_c5 --gpus 8 --rehearse --mode rowtile --height 2160 --width 3840 --num-disp 256 --win 15 --steps 100 --warmup 10 && \
run c5_1gpu --height 2160 --width 3840 --num-disp 256 --win 15 --batch 2 --frames 2 --steps 100 --warmup 10
