#!/bin/bash
# Pruned-walk session: GPU parity tests, then A/B of reference-order (7) vs
# pruned (8) walks on C2 / C3 / C4 / C5 (images must be bit-identical).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-prune}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -6 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,c2,c3,c3s,c4,c4s,c5,waves}
[[ $STEPS == *tests* ]] && run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
[[ $STEPS == *c2* ]] && run ab_c2 300 python3 scripts/render_loop.py --frames 30 --counts --ab CRT_TRAVERSAL=7,8
[[ $STEPS == *c3* ]] && run ab_c3 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 10 --counts --ab CRT_TRAVERSAL=7,8
[[ $STEPS == *c3s* ]] && CRT_TRAVERSAL=8 run ab_c3_sec 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 10 --ab CRT_SECONDARY=5,9,10,11
[[ $STEPS == *c4* ]] && run ab_c4 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 3 --counts --ab CRT_TRAVERSAL=7,8
[[ $STEPS == *c4s* ]] && CRT_TRAVERSAL=8 run ab_c4_sec 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 2 --ab CRT_SECONDARY=4,9,10,11
[[ $STEPS == *waves* ]] && run waves_c2 300 python3 scripts/wave_profile.py 14-01-acceleration-tree__scene1 7,8
[[ $STEPS == *c5* ]] && run ab_c5 400 python3 scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 5 --counts --ab CRT_TRAVERSAL=7,8
exit 0
