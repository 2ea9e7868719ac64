#!/bin/bash
# Round-5 GPU session: each GPU step under its own limit; a failing step ends
# the session.  STEPS (comma list) of:
#   tests   pytest -m gpu (PYTEST_K: a -k selection, e.g. "pipelined or bins")
#   smoke   __graft_entry__.smoke()
#   bench   the driver's command: python bench.py --gpus 1 --steps 20 --warmup 5
#   bench2  BENCH_ARGS: one more bench.py line
#   cmd     CMD: any command (its own limit CMD_T, default 300 s)
#   TAG=x STEPS=tests,bench bash scripts/gpu_r05.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
[[ $STEPS == *tests* ]] && run pytest_gpu ${TESTS_T:-900} python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "${PYTEST_K:-}"
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench,* || $STEPS == *bench ]] && run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
[[ $STEPS == *bench2* ]] && run bench2 600 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *cmd* ]] && run cmd ${CMD_T:-300} bash -c "${CMD:-true}"
exit 0
