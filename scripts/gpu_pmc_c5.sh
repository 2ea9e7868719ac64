#!/bin/bash
# C5 (synthetic 1M triangles, 3840x2160): HBM bytes of the render kernel from
# PMC (FETCH_SIZE / WRITE_SIZE, separate passes) + kernel trace for its duration.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc_c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
C5="scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $C5 > "$OUT/trace.log" 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $C5 > "$OUT/fetch.log" 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $C5 > "$OUT/write.log" 2>&1 || { echo write failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/l2" -o run --output-format csv -- python3 $C5 > "$OUT/l2.log" 2>&1 || echo "l2 pass failed"
grep -h "k_render_tiles" "$OUT"/trace/*kernel_stats.csv
exit 0
