#!/bin/bash
# C2 kernel ms over tile-plan calibration knobs (env per run, one process each).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-calib_ab}
mkdir -p "$OUT"
for cfg in "CRT_CALIB_K=4" "CRT_CALIB_K=4 CRT_CALIB_DIRECT=1" "CRT_CALIB_K=3 CRT_CALIB_DIRECT=1" "CRT_CALIB_K=2 CRT_CALIB_DIRECT=1" "CRT_CALIB_K=1.5 CRT_CALIB_DIRECT=1" "CRT_CALIB_K=6" "CRT_CALIB_K=8"; do
  name=$(echo $cfg | tr ' =' '_-')
  timeout -k 10 120 env $cfg python3 scripts/render_loop.py --frames 30 --counts > "$OUT/$name.json" 2>&1 || exit $?
  echo "$cfg $(tail -1 $OUT/$name.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["kernel"]["default"]; print(round(d["median_ms"],4), d["wave"])')"
done
exit 0
