#!/bin/bash
# Round-2 config session: bench.py lines for C3 / C4 / C5 and PMC passes of
# the C3 wavefront levels (k_wf_level) and the C4 GI refill kernel
# (k_render_refill) -> gpurun_out/<tag>/.  Each GPU step has its own limit;
# a fault, abort or timeout ends the session.
#   TAG=x STEPS=bench,pmc3,pmc4 bash scripts/gpu_r02_configs.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r02cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-bench,pmc3,pmc4}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
if [[ $STEPS == *bench* ]]; then
  for c in c3 c4 c5; do run bench_$c 500 python bench.py --config $c --steps ${BSTEPS:-10} --warmup 2; done
fi
pmc() {   # name, kernel, command...
  local name=$1 kern=$2; shift 2
  run ${name}_inst 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d "$OUT/$name/inst" -o run --output-format csv -- "$@"
  run ${name}_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/$name/sq" -o run --output-format csv -- "$@"
  run ${name}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$name/fetch" -o run --output-format csv -- "$@"
  run ${name}_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$name/write" -o run --output-format csv -- "$@"
  run ${name}_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/$name/tcc" -o run --output-format csv -- "$@"
  run ${name}_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name/trace" -o run --output-format csv -- "$@"
}
C3="scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 3"
C4="scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 2"
if [[ $STEPS == *pmc3* ]]; then
  pmc pmc_c3 k_wf_level python3 $C3
  run pmc_c3_record 120 python3 scripts/pmc_record.py --config c3 --size 1920 1080 --kernel "k_wf_level<10, false" --dir "$OUT/pmc_c3" --out "$OUT/pmc_c3.json" --command "python3 $C3"
fi
if [[ $STEPS == *pmc4* ]]; then
  pmc pmc_c4 k_render_refill python3 $C4
  run pmc_c4_record 120 python3 scripts/pmc_record.py --config c4 --size 1080 1080 --kernel k_render_refill --dir "$OUT/pmc_c4" --out "$OUT/pmc_c4.json" --command "python3 $C4"
fi
exit 0
