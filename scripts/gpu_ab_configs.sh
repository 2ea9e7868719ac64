#!/bin/bash
# Same-box A/B of the in-tree build against variant builds (abtest/<name>) on
# C2 (1920x1080), C3 (depth 8) and C4 (1080x1080): render_loop kernel times,
# two alternating rounds.  TAG=x bash scripts/gpu_ab_configs.sh <name> [...]
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abc}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
RL="python3 scripts/render_loop.py"
for round in 1 2; do
  for v in base "$@"; do
    pk=chaos-ray-tracing-course-2025_amd; [ $v != base ] && pk=abtest/$v
    CRT_PKG=$pk run ${v}_c2_$round 240 $RL --frames 30
    CRT_PKG=$pk run ${v}_c3_$round 240 $RL --scene 11-01-refractive__scene8 --depth 8 --frames 10
    CRT_PKG=$pk run ${v}_c4_$round 240 $RL --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 3
  done
done
