#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace.  Every GPU step
# has its own time limit; a fault / abort / timeout stops the session.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,bench,prof}
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 50 --warmup 5
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline
exit 0
