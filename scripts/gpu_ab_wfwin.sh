#!/bin/bash
# A/B of the wavefront levels' secondary walk on C3 (10 = pruned cooperative,
# 14 / 15 = window walks), the parity tests of the window walks, and C3 bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-wfwin}
mkdir -p "$OUT"
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
run tests 300 python -u -m pytest tests/test_gpu_parity.py -k window_walks -x -q --timeout 200 --timeout-method thread
run ab_c3 300 python scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 6 --opt secondary=10,14,15
run ab_c3r 300 python scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 6 --opt secondary=15,14,10
