#!/bin/bash
# GI (C4 1080^2) with the pruned cooperative walk (secondary 10) in the refill
# kernel at wave caps 3/4/5 (builds abtest/h3,h4,h5) against walk 4 (h4 default).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-gi10}
mkdir -p "$OUT"
SCN="--scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4"
for r in 1 2; do
  timeout -k 10 200 env CRT_PKG=abtest/h4 python3 scripts/render_loop.py $SCN > "$OUT/w4_$r.json" 2>&1 || exit $?
  echo "walk4 $(tail -1 $OUT/w4_$r.json)"
  for b in h3 h4 h5; do
    timeout -k 10 200 env CRT_PKG=abtest/$b CRT_SECONDARY=10 python3 scripts/render_loop.py $SCN > "$OUT/${b}_$r.json" 2>&1 || exit $?
    echo "walk10 $b $(tail -1 $OUT/${b}_$r.json)"
  done
done
