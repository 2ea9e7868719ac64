#!/bin/bash
# PMC records of every config's render kernel(s) on the current build
# (scripts/gpu_pmc.sh per config) -> gpurun_out/<TAG>/<cfg>/pmc_<cfg>.json,
# plus the cold first-call breakdown (scripts/cold_breakdown.py).
#   TAG=x CFGS="c2 c3 c4 c5" COLD=1 TIMELINE=1 bash scripts/gpu_pmc_all.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-pmcall}
export TAG
RL=scripts/render_loop.py
for c in ${CFGS:-c2 c3 c4 c5}; do
  echo "== pmc $c"
  case $c in
    c2) CFG=c2 KERNEL=k_render_tiles SIZE="1920 1080" LAST=2 FRAME_END= \
          CMD="$RL --scene 14-01-acceleration-tree__scene1 --frames 2 --opt calibrate=1" bash scripts/gpu_pmc.sh || exit 1 ;;
    c2s) CFG=c2s KERNEL="k_render_tiles|k_shadow_vis|k_shadow_compose" SIZE="1920 1080" LAST=2 FRAME_END=k_shadow_compose \
          CMD="$RL --scene 14-01-acceleration-tree__scene1 --frames 3 --opt calibrate=1 --set shadows=1" bash scripts/gpu_pmc.sh || exit 1 ;;
    c3) CFG=c3 KERNEL=k_wf_ SIZE="1920 1080" LAST=2 FRAME_END=k_wf_pixels \
          CMD="$RL --scene 11-01-refractive__scene8 --depth 8 --frames 3 --opt calibrate=1" bash scripts/gpu_pmc.sh || exit 1 ;;
    c4) CFG=c4 KERNEL=k_render_gi SIZE="3840 2160" LAST=2 FRAME_END= \
          CMD="$RL --scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 2" bash scripts/gpu_pmc.sh || exit 1 ;;
    c5) CFG=c5 KERNEL=k_render_tiles SIZE="3840 2160" LAST=2 FRAME_END= \
          CMD="$RL --synthetic 1000000 --width 3840 --height 2160 --frames 2 --opt calibrate=1" bash scripts/gpu_pmc.sh || exit 1 ;;
  esac
done
if [ -n "${TIMELINE:-}" ]; then
  mkdir -p gpurun_out/$TAG/timeline
  timeout -k 10 200 python3 scripts/wave_timeline.py --out gpurun_out/$TAG/timeline/timeline_c2.json \
    > gpurun_out/$TAG/timeline/tl.log 2>&1 || { echo "timeline failed"; tail -5 gpurun_out/$TAG/timeline/tl.log; exit 1; }
  timeout -k 10 200 python3 scripts/shard_times.py --config c2 --reps 20 --out gpurun_out/$TAG/timeline/shards_c2.json \
    > gpurun_out/$TAG/timeline/sh.log 2>&1 || { echo "shards failed"; tail -5 gpurun_out/$TAG/timeline/sh.log; exit 1; }
  tail -2 gpurun_out/$TAG/timeline/tl.log | cut -c1-1500
fi
if [ -n "${COLD:-}" ]; then
  mkdir -p gpurun_out/$TAG/cold
  timeout -k 10 300 python3 scripts/cold_breakdown.py --config c2 --out gpurun_out/$TAG/cold/cold_c2.json \
    > gpurun_out/$TAG/cold/cold_c2.log 2>&1 || { echo "cold failed"; tail -5 gpurun_out/$TAG/cold/cold_c2.log; exit 1; }
  cat gpurun_out/$TAG/cold/cold_c2.log
fi
exit 0
