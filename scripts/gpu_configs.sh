#!/bin/bash
# Kernel time of every BASELINE config on one GPU (render_loop.py, C-ABI, no torch):
# C2 14-01/s1 1080p, C3 11-01/s8 1080p depth 8, C4 15-01/s2 GI at 1080^2 and 4K,
# C5 synthetic 1M triangles at 4K, plus the bitmap-textured 12-01/s4 at 1080p.
#   TAG=r01f bash scripts/gpu_configs.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-configs}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python3 scripts/render_loop.py "$@" > "$OUT/$name.json" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.json"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
run c2 --scene 14-01-acceleration-tree__scene1 --frames 20 --counts
run c3 --scene 11-01-refractive__scene8 --depth 8 --frames 10 --counts
run c4_1080 --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 3 --counts
run c4_4k --scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 2
run c5_4k --synthetic 1000000 --width 3840 --height 2160 --frames 3 --counts
run tex_1080 --scene 12-01-textures__scene4 --frames 10
exit 0
