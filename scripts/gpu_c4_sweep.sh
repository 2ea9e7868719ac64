#!/bin/bash
# C4 (GI) cost structure: kernel ms vs max depth, per secondary walk.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-c4_sweep}
mkdir -p "$OUT"
for d in ${DEPTHS:-0 1 2 3}; do
  timeout -k 10 120 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width ${W:-1080} --height ${H:-1080} \
     --frames 2 --depth $d --ab "CRT_SECONDARY=${WALKS:-4,0}" > "$OUT/depth$d.json" 2>&1 || { echo "depth $d failed"; cat "$OUT/depth$d.json"; exit 1; }
  cat "$OUT/depth$d.json"
done
