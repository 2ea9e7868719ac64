#!/bin/bash
# C3 (11-01/scene8, depth 8) kernel timeline: rocprofv3 kernel trace of a few
# frames, for the per-level durations and the gaps between level launches.
#   TAG=r01j bash scripts/gpu_c3_trace.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-c3trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 4 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 "$OUT/trace.log"; exit $rc
