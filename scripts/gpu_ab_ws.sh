#!/bin/bash
# A/B of the two-stream launch (option window_stream) and of the window-only
# kernel's waves per SIMD (variant builds abtest/ws6, ws7; default 8).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ws}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
run ab_ws 300 python scripts/render_loop.py --frames 40 --opt window_stream=0,1
run ab_ws_r 300 python scripts/render_loop.py --frames 40 --opt window_stream=1,0
CRT_PKG=abtest/ws6 run ab_ws6 300 python scripts/render_loop.py --frames 40 --opt window_stream=1,0
CRT_PKG=abtest/ws7 run ab_ws7 300 python scripts/render_loop.py --frames 40 --opt window_stream=1,0
run tests 300 python -u -m pytest tests/test_gpu_parity.py -k c2_full -x -q --timeout 200 --timeout-method thread
run bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
