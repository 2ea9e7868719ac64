#!/bin/bash
# GI pixel refill: GPU parity tests, then C4 (15-01/scene2) A/B refill off/on
# and refill grid sizes; images are compared bit for bit across variants.
#   TAG=r01q bash scripts/gpu_gi_refill.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-gi_refill}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
SC="--scene 15-01-conclusion__scene2 --width ${W:-1080} --height ${H:-1080} --frames ${FRAMES:-5}"
timeout -k 10 300 python3 scripts/render_loop.py $SC --ab CRT_GI_REFILL=0,1 > "$OUT/ab_refill.log" 2>&1 || exit $?
cat "$OUT/ab_refill.log"
timeout -k 10 300 python3 scripts/render_loop.py $SC --ab "CRT_REFILL_WAVES=${RW:-2048,5120,8192,1000000}" > "$OUT/ab_waves.log" 2>&1 || exit $?
cat "$OUT/ab_waves.log"
