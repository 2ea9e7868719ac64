#!/bin/bash
# Same-box A/B of abtest/<build> variants on C2 (and optionally C5), interleaved
# rounds, each run under its own time limit; plus wave counts of the base build.
#   BUILDS="base nosink" ROUNDS=3 TAG=x bash scripts/gpu_ab_r02.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abr02}
mkdir -p "$OUT"
SCN=${SCN:---frames 30}
for r in $(seq 1 ${ROUNDS:-3}); do
  for b in $BUILDS; do
    timeout -k 10 200 env CRT_PKG=abtest/$b python3 scripts/render_loop.py $SCN > "$OUT/${b}_$r.json" 2>&1 || { echo "$b failed"; tail -5 "$OUT/${b}_$r.json"; exit 1; }
    echo "r$r $(python3 scripts/ab_summary.py $OUT/${b}_$r.json)"
  done
done
if [ -n "${COUNTS:-}" ]; then
  for b in $BUILDS; do
    timeout -k 10 200 env CRT_PKG=abtest/$b python3 scripts/render_loop.py $SCN --frames 3 --counts > "$OUT/${b}_counts.json" 2>&1 || exit 1
    tail -1 "$OUT/${b}_counts.json"
  done
fi
exit 0
