#!/bin/bash
# Measured-cost tile plan session: parity tests, then A/B of the calibration
# knobs on C2 / C5 (images must stay bit-identical), and C2 wave timelines.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,c2,c5,waves}
[[ $STEPS == *tests* ]] && run pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
if [[ $STEPS == *c2* ]]; then
  CRT_TRAVERSAL=8 run c2_cal8 300 python3 scripts/render_loop.py --frames 30 --ab CRT_CALIBRATE=0,1
  CRT_TRAVERSAL=7 run c2_cal7 300 python3 scripts/render_loop.py --frames 30 --ab CRT_CALIBRATE=0,1
  run c2_k 300 python3 scripts/render_loop.py --frames 30 --ab "CRT_CALIB_K=0.25,0.5,1,2,4"
  run c2_min 300 python3 scripts/render_loop.py --frames 30 --ab "CRT_CALIB_MIN=1,2,4"
fi
[[ $STEPS == *c5* ]] && run c5_cal 400 python3 scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 5 --ab "CRT_CALIB_K=1,2,4,8"
[[ $STEPS == *c3* ]] && run c3_cal 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 10 --ab CRT_CALIBRATE=0,1
[[ $STEPS == *waves* ]] && run waves_c2 300 python3 scripts/wave_profile.py 14-01-acceleration-tree__scene1 7,8
exit 0
