#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export CRT_TRAVERSAL=5
run pytest_gpu 600 python -m pytest tests -m gpu -q -rf -x
run ab_split 300 python3 scripts/render_loop.py --frames 20 --ab "CRT_SPLIT=0,0.2;0.5,0.1;0.3,0.05;0.2,0.02;0.1"
run waves 300 python3 scripts/wave_profile.py 14-01-acceleration-tree__scene1 5
unset CRT_TRAVERSAL
run ab_trav 300 python3 scripts/render_loop.py --frames 20 --ab CRT_TRAVERSAL=3,5
exit 0
