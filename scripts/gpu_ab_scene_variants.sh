#!/bin/bash
# Same-box A/B of variant builds (abtest/<name>, scripts/make_variant.sh) on one
# scene: kernel time per variant, two alternating rounds (render_loop.py).
#   TAG=x ARGS="--scene ... --width ... --frames 4" bash scripts/gpu_ab_scene_variants.sh base <name> ...
# "base" = the in-tree build.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abs}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then run ${v}_$round 240 python3 scripts/render_loop.py $ARGS
    else CRT_PKG=abtest/$v run ${v}_$round 240 python3 scripts/render_loop.py $ARGS; fi
  done
done
exit 0
