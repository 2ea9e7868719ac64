#!/bin/bash
# Same-box A/B on C3 (11-01/scene8 1920x1080 depth 8): in-tree build vs the
# variant builds given as arguments, three alternating rounds; then their C3
# parity tests.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/abc3
mkdir -p "$OUT"
C3="scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 8"
for round in 1 2 3; do
  timeout -k 10 240 python $C3 > $OUT/base_$round.log 2>&1 || exit 1
  tail -1 $OUT/base_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']['default']; print('base', $round, round(d['median_ms'],4), round(d['min_ms'],4))"
  for v in "$@"; do
    CRT_PKG=abtest/$v timeout -k 10 240 python $C3 > $OUT/${v}_$round.log 2>&1 || exit 1
    tail -1 $OUT/${v}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']['default']; print('$v', $round, round(d['median_ms'],4), round(d['min_ms'],4))"
  done
done
for v in "$@"; do
  CRT_PKG=abtest/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -k "c3 or wavefront or render_matches or deep" -x -q --timeout 200 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { tail -20 $OUT/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $OUT/tests_$v.log)"
done
