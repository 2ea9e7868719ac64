#!/bin/bash
# Round-3 GPU session steps (each GPU step under its own time limit; a fault /
# abort / timeout ends the session):
#   TAG=x STEPS=tests,c4ab,c3ab,c4k bash scripts/gpu_r03.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/pmc"
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
STEPS=${STEPS:-tests}
PYTEST_ARGS=${PYTEST_ARGS:-tests}
RL="python3 scripts/render_loop.py"
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -u -m pytest $PYTEST_ARGS -m gpu -v -rf --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
[[ $STEPS == *c4ab* ]] && run c4ab 300 $RL --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4 --counts --opt secondary=${C4AB:-4,14}
[[ $STEPS == *c3ab* ]] && run c3ab 300 $RL --scene 11-01-refractive__scene8 --depth 8 --frames 8 --counts --opt secondary=${C3AB:-10,14}
[[ $STEPS == *c4k* ]] && run c4k 300 $RL --scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 3
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 20 --warmup 5
if [[ $STEPS == *shards* ]]; then
  for c in c2 c3 c4 c5; do
    r=20; [ $c = c4 ] && r=3; [ $c = c5 ] && r=5
    run shards_$c 300 python3 scripts/shard_times.py --config $c --reps $r --out "$OUT/shards_$c.json"
  done
fi
if [[ $STEPS == *rehearse* ]]; then
  run rehearse_c4_gloo2 600 python bench.py --config c4 --gpus 2 --backend gloo --check --steps 3 --warmup 1 --no-secondary
  run rehearse_c2_gloo2 300 python bench.py --gpus 2 --backend gloo --check --steps 20 --warmup 3
fi
exit 0
