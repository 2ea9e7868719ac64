#!/bin/bash
# Round 6: C2 with shadow rays — the shadow tests, then inline against
# deferred shadow rays (option shadow_defer) with and without the light bins,
# and a kernel trace of the default.   TAG=x bash scripts/gpu_r06_shadow.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sd}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 "$OUT/$name.log" | cut -c1-400)"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
run tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_png_pins.py -k "shadow or light"
run lb1 200 python scripts/render_loop.py --frames 40 --set shadows=1 --set light_bins=1 --opt shadow_defer=1,0
run lb0 200 python scripts/render_loop.py --frames 40 --set shadows=1 --set light_bins=0 --opt shadow_defer=1,0
run trace 200 rocprofv3 --kernel-trace --stats -d "$OUT/tr" -o run --output-format csv -- python3 scripts/render_loop.py --frames 20 --set shadows=1
python3 scripts/kstats.py "$(find "$OUT/tr" -name "*kernel_stats.csv" | head -1)" | head -8
exit 0
