#!/bin/bash
# A/B of the per-lane-walk tiles (option lane_tiles) on C2, C3 level 0 and the
# wave timeline; each GPU step under its own time limit, stop on the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-lane}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
run ab_c2 300 python scripts/render_loop.py --frames 30 --opt lane_tiles=0,1 --counts
run ab_c2b 300 python scripts/render_loop.py --frames 30 --opt lane_tiles=1,0
run tl_lane 300 python scripts/wave_timeline.py --lane-tiles 1 --out "$OUT/timeline_lane.json"
