#!/bin/bash
# Round-6 final evidence on one build, one GPU session (each GPU step under its
# own limit; a failing step ends the session):
#   tests   pytest -m gpu + smoke
#   pmc     PMC records of every config's render kernel(s) (scripts/gpu_pmc_all.sh),
#           copied to profiles/r06/pmc_<cfg>.json on the box so the bench lines
#           below read them (bench.py load_pmc checks the build id)
#   bench   the driver's command (python bench.py --gpus 1 --steps 20 --warmup 5)
#           and the C3, C4, C5 lines
#   trace   rocprofv3 kernel trace + stats of the driver's command
#   TAG=r06/final STEPS=tests,pmc,bench,trace bash scripts/gpu_r06_final.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r06/final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,pmc,bench,trace}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
[[ $STEPS == *tests* ]] && run pytest_gpu 1200 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
[[ $STEPS == *tests* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [[ $STEPS == *pmc* ]]; then
  CFGS="c2 c2s c3 c4 c5" TAG=$TAG/pmc bash scripts/gpu_pmc_all.sh > "$OUT/pmc_all.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/pmc_all.log"; exit 1; }
  mkdir -p profiles/r06 && for c in c2 c2s c3 c4 c5; do cp "gpurun_out/$TAG/pmc/$c/pmc_$c.json" "profiles/r06/pmc_$c.json" || exit 1; done
  grep -h "\"build_id\"" profiles/r06/pmc_c*.json | cut -c1-120 | head -5
fi
# bench: every line; bench_driver / bench_c3 / bench_c4 / bench_c5: one each
[[ $STEPS == *bench* && ( $STEPS != *bench_* || $STEPS == *bench_driver* ) ]] && run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
[[ $STEPS == *bench* && ( $STEPS != *bench_* || $STEPS == *bench_c3* ) ]] && run bench_c3 600 python bench.py --config c3 --steps 100 --warmup 10
[[ $STEPS == *bench* && ( $STEPS != *bench_* || $STEPS == *bench_c4* ) ]] && run bench_c4 1100 python bench.py --config c4 --steps 8 --warmup 2
[[ $STEPS == *bench* && ( $STEPS != *bench_* || $STEPS == *bench_c5* ) ]] && run bench_c5 900 python bench.py --config c5 --steps 10 --warmup 2
[[ $STEPS == *trace* ]] && run trace_driver 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_driver" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e
exit 0
