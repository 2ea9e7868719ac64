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
export CRT_TRAVERSAL=6
run pytest_gpu 600 python -m pytest tests -m gpu -q -rf -x
run ab_split6 300 python3 scripts/render_loop.py --frames 20 --ab "CRT_SPLIT=0;0.2,0.5;0.05"
run waves6 300 python3 scripts/wave_profile.py 14-01-acceleration-tree__scene1 6
unset CRT_TRAVERSAL
run ab_trav 300 python3 scripts/render_loop.py --frames 20 --ab CRT_TRAVERSAL=3,5,6
run ab_c3 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 4 --ab CRT_TRAVERSAL=3,5,6
exit 0
