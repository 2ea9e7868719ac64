#!/bin/bash
# C3 secondary-level A/B (kernel ms + work/wave counts per variant), e.g.
#   AB="CRT_WF_OCT=7,0" TAG=r01l bash scripts/gpu_c3_diag.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-c3diag}
mkdir -p "$OUT"
i=0
IFS='|' read -ra ABS <<< "${AB:-CRT_WF_RPW=64,16}"
for ab in "${ABS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth ${DEPTH:-8} --frames ${FRAMES:-6} --counts --ab "$ab" > "$OUT/ab$i.log" 2>&1 || exit $?
  cat "$OUT/ab$i.log"
done
