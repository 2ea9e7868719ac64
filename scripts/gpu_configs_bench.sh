#!/bin/bash
# Kernel timings of every config (gpu_configs.sh) + bench.py --config c3|c4|c5 lines, one session.
#   TAG=r01u bash scripts/gpu_configs_bench.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r01u}
TAG=$TAG bash scripts/gpu_configs.sh || exit $?
for c in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 > gpurun_out/$TAG/bench_$c.json 2>gpurun_out/$TAG/bench_$c.err || exit $?
  tail -1 gpurun_out/$TAG/bench_$c.json
done
if [ -n "${GI_AB:-}" ]; then
  timeout -k 10 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4 --ab "$GI_AB" > gpurun_out/$TAG/gi_ab.log 2>&1 || exit $?
  cat gpurun_out/$TAG/gi_ab.log
fi
