#!/bin/bash
# C4 (15-01/scene2, GI) probe: kernel time and work counts of the GI refill
# kernel with the reference-order (4) and pruned (10) cooperative walks.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-c4probe}
mkdir -p "$OUT"
timeout -k 10 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 \
  --frames 3 --counts --opt secondary=4,10 > "$OUT/c4_1080.json" 2>&1
rc=$?; tail -3 "$OUT/c4_1080.json"; exit $rc
