#!/bin/bash
# Same-box A/B, three alternating rounds of 80 C2 frames: in-tree build vs the
# variant builds given as arguments (abtest/<name>), then their parity tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/absched3
for round in 1 2 3; do
  timeout -k 10 240 python scripts/render_loop.py --frames 80 > gpurun_out/absched3/base_$round.log 2>&1 || exit 1
  tail -1 gpurun_out/absched3/base_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']['default']; print('base', $round, round(d['median_ms'],5), round(d['min_ms'],5))"
  for v in "$@"; do
    CRT_PKG=abtest/$v timeout -k 10 240 python scripts/render_loop.py --frames 80 > gpurun_out/absched3/${v}_$round.log 2>&1 || exit 1
    tail -1 gpurun_out/absched3/${v}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']['default']; print('$v', $round, round(d['median_ms'],5), round(d['min_ms'],5))"
  done
done
for v in "$@"; do
  CRT_PKG=abtest/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_png_pins.py -m gpu -k "c2_full or window or png or shadow" -x -q --timeout 200 --timeout-method thread > gpurun_out/absched3/tests_$v.log 2>&1 || { tail -20 gpurun_out/absched3/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/absched3/tests_$v.log)"
done
