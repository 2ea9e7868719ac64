#!/bin/bash
# Quick PMC pass on the C2 render kernel (issue/stall split and instruction mix).
#   TAG=x bash scripts/gpu_pmc.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d "$OUT/sq" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
run pmc_inst 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_SALU -d "$OUT/inst" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
run pmc_lvl 300 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/lvl" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
exit 0
