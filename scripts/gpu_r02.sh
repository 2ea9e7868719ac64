#!/bin/bash
# Round-2 GPU session: tests, smoke, bench (N=1), N=2 tiles rehearsal on the one
# GPU (gloo, f32 and u8 payloads, --check), rocprofv3 kernel trace of the bench
# command, per-wave timeline, shadow-ray bench, PMC passes of the C2 render kernel -> profiles/r02/pmc_c2.json.
# Each GPU step has its own time limit; a fault / abort / timeout ends the session.
#   TAG=x STEPS=tests,smoke,bench,timeline,shadow,rehearse,prof,pmc bash scripts/gpu_r02.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r02}
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
STEPS=${STEPS:-tests,smoke,bench,timeline,shadow,rehearse,prof,pmc}
PYTEST_ARGS=${PYTEST_ARGS:-tests}
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -u -m pytest $PYTEST_ARGS -m gpu -v -rf --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 20 --warmup 5
if [[ $STEPS == *rehearse* ]]; then
  run rehearse2_f32 300 python bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --check
  run rehearse2_u8 300 python bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --check --payload u8 --no-secondary
fi
[[ $STEPS == *timeline* ]] && run timeline 300 python scripts/wave_timeline.py --out "$OUT/timeline_c2.json"
[[ $STEPS == *shadow* ]] && run bench_shadows 600 python bench.py --shadows --steps 20 --warmup 5
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e
if [[ $STEPS == *pmc* ]]; then
  CMD="python3 scripts/render_loop.py --frames 3"
  run pmc_inst 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d "$OUT/pmc/inst" -o run --output-format csv -- $CMD
  run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/pmc/sq" -o run --output-format csv -- $CMD
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc/fetch" -o run --output-format csv -- $CMD
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc/write" -o run --output-format csv -- $CMD
  run pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc/tcc" -o run --output-format csv -- $CMD
  run pmc_record 120 python3 scripts/pmc_record.py --config c2 --size 1920 1080 --dir "$OUT/pmc" --out "$OUT/pmc_c2.json" --last 3 --command "$CMD"
fi
exit 0
