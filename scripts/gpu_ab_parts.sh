#!/bin/bash
# Tile parts: parity tests, then per-shard render times with tile_parts 1
# (default) and 0, and the N=1 frame (unchanged plan) for reference.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-parts}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
run tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_png_pins.py -m gpu -k "tile_parts or compact or c2_full or window or png or shadow" -x -q --timeout 200 --timeout-method thread
run shards_p1 240 python scripts/shard_times.py --counts 1,2,4,8
run shards_p0 240 python scripts/shard_times.py --counts 1,2,4,8 --opt tile_parts=0
run shards_p1b 240 python scripts/shard_times.py --counts 1,2,4,8
