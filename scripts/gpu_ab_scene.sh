#!/bin/bash
# Same-box A/B of builds abtest/<b> on one render_loop workload (SCN), interleaved.
#   BUILDS="g1 g5 g6" SCN="--scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 2" bash scripts/gpu_ab_scene.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abscene}
mkdir -p "$OUT"
for r in 1 2; do
  for b in $BUILDS; do
    timeout -k 10 200 env CRT_PKG=abtest/$b python3 scripts/render_loop.py $SCN > "$OUT/${b}_$r.json" 2>&1 || exit $?
    echo "$b $(tail -1 $OUT/${b}_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["kernel"]["default"]["median_ms"],3))')"
  done
done
exit 0
