#!/bin/bash
# Same-box A/B of two builds of the library: abtest/old (a previous commit's
# lib/ + crt_amd/) against the working tree, interleaved runs of render_loop.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abb}
mkdir -p "$OUT"
SCN=${SCN:---frames 40}
for r in 1 2; do
  timeout -k 10 200 env CRT_PKG=abtest/old python3 scripts/render_loop.py $SCN > "$OUT/old_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/old_$r.log"
  timeout -k 10 200 python3 scripts/render_loop.py $SCN > "$OUT/new_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/new_$r.log"
done
