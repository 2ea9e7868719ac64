#!/bin/bash
# Round-4 final evidence on one build, one GPU session (each GPU step under its
# own limit; a failing step ends the session):
#   1. pytest -m gpu + smoke
#   2. PMC records of every config's render kernel(s) (scripts/gpu_pmc_all.sh),
#      copied to profiles/r04/pmc_<cfg>.json on the box so the bench lines below
#      read them (bench.py load_pmc checks the build id)
#   3. bench.py lines: C2 (default), C3, C4, C5; rocprofv3 kernel trace of the C2 bench
#   4. shard times of every config
#   5. one-GPU gloo rehearsals of the N=2 tiles path with --check
#   TAG=final STEPS=tests,pmc,bench,trace,shards,rehearse bash scripts/gpu_r04_final.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,pmc,bench,trace,shards}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
[[ $STEPS == *tests* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [[ $STEPS == *pmc* ]]; then
  TAG=$TAG/pmc bash scripts/gpu_pmc_all.sh > "$OUT/pmc_all.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/pmc_all.log"; exit 1; }
  for c in c2 c3 c4 c5; do cp "gpurun_out/$TAG/pmc/$c/pmc_$c.json" "profiles/r04/pmc_$c.json" || exit 1; done
  grep -h '"build_id"' profiles/r04/pmc_c*.json | head -4
fi
if [[ $STEPS == *bench* ]]; then
  run bench_c2 600 python bench.py
  run bench_c3 600 python bench.py --config c3 --steps 20 --warmup 3
  run bench_c4 900 python bench.py --config c4 --steps 8 --warmup 2
  run bench_c5 600 python bench.py --config c5 --steps 10 --warmup 2
fi
[[ $STEPS == *trace* ]] && run trace_bench_c2 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_bench_c2" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e
if [[ $STEPS == *shards* ]]; then
  for c in c2 c3 c4 c5; do
    r=20; [ $c = c4 ] && r=3; [ $c = c5 ] && r=5
    run shards_$c 400 python3 scripts/shard_times.py --config $c --reps $r --out "$OUT/shards_$c.json"
  done
fi
if [[ $STEPS == *rehearse* ]]; then
  run rehearse_c2_gloo2 400 python bench.py --gpus 2 --backend gloo --check --steps 20 --warmup 3
  run rehearse_c4_gloo2 600 python bench.py --config c4 --gpus 2 --backend gloo --check --steps 3 --warmup 1 --no-secondary
fi
exit 0
