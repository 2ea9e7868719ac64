#!/bin/bash
# Quick loop: GPU parity tests + C2 A/B of the camera walks + bench line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,ab,bench}
[[ $STEPS == *tests* ]] && run pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
[[ $STEPS == *ab* ]] && run ab_c2 300 python3 scripts/render_loop.py --frames 40 --ab "${AB:-CRT_CAMERA_FAST=0,1}"
[[ $STEPS == *abc3* ]] && run ab_c3 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 10 --ab "${AB3:-CRT_CAMERA_FAST=0,1}"
[[ $STEPS == *abc5* ]] && run ab_c5 300 python3 scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 5 --ab "${AB5:-CRT_CAMERA_FAST=0,1}"
[[ $STEPS == *tilecost* ]] && run tilecost 300 python3 scripts/tile_cost_profile.py
[[ $STEPS == *bench* ]] && run bench 300 python bench.py --no-cpu-baseline
exit 0
