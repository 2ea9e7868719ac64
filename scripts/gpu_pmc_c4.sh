#!/bin/bash
# PMC passes over one C4 frame (15-01/scene2 GI, 1080x1080): issue, waits,
# instruction mix, lane utilisation (SQ_THREAD_CYCLES_VALU), L2 hit rate.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc_c4}
mkdir -p "$OUT"
export TMPDIR=/tmp
SC="scripts/render_loop.py --scene ${SCENE:-15-01-conclusion__scene2} --width ${W:-1080} --height ${H:-1080} --frames 1 ${EXTRA:-}"
run() {
  local name=$1; shift
  echo "== $name"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 $SC > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA
run inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR
run l2 TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
