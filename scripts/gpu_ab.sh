#!/bin/bash
# A/B session: parity tests under a chosen variant, then in-process A/B timings.
#   AB="CRT_TRAVERSAL=3,4" TESTENV="CRT_TRAVERSAL=4" bash scripts/gpu_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "${TESTENV:-}" ]; then export ${TESTENV}; fi
run pytest_gpu 600 python -m pytest tests -m gpu -q -rf -x
if [ -n "${TESTENV:-}" ]; then unset ${TESTENV%%=*}; fi
run ab_c2 300 python3 scripts/render_loop.py --frames 20 --ab "$AB"
run ab_c3 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 6 --ab "$AB"
run ab_c4 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 2 --ab "$AB"
exit 0
