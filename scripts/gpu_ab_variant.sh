#!/bin/bash
# Same-box A/B of the in-tree build against variant builds (abtest/<name>,
# scripts/make_variant.sh): C2 kernel time (render_loop.py, 40 frames, two
# alternating rounds) and the sharded frame's per-shard floor (shard_times.py).
#   TAG=x bash scripts/gpu_ab_variant.sh <name> [<name> ...]
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abv}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-400)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for round in 1 2; do
  run base_$round 240 python scripts/render_loop.py --frames 40
  for v in "$@"; do CRT_PKG=abtest/$v run ${v}_$round 240 python scripts/render_loop.py --frames 40; done
done
run shards_base 240 python scripts/shard_times.py --counts 1,8
for v in "$@"; do CRT_PKG=abtest/$v run shards_$v 240 python scripts/shard_times.py --counts 1,8; done
