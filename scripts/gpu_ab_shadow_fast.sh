#!/bin/bash
# Shadow-ray frames: parity of a variant build (abtest/$1) and C2 shadow-frame
# times of the in-tree build vs the variant, two alternating rounds.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abfs}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
CRT_PKG=abtest/$1 run tests 300 python -u -m pytest tests/test_png_pins.py -m gpu -x -q --timeout 200 --timeout-method thread
for round in 1 2; do
  run base_$round 240 python scripts/render_loop.py --frames 20 --opt shadows=1
  CRT_PKG=abtest/$1 run var_$round 240 python scripts/render_loop.py --frames 20 --opt shadows=1
done
