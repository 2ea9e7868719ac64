#!/bin/bash
# GPU tests, then C3 A/B of the child-queue order (CRT_WF_GROUP) at 32 and 64 rays/wave.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-c3group}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rpw in 32 64; do
  timeout -k 10 200 env CRT_WF_RPW=$rpw python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 8 --counts --ab CRT_WF_GROUP=0,1 > "$OUT/rpw$rpw.log" 2>&1 || exit $?
  cat "$OUT/rpw$rpw.log"
done
