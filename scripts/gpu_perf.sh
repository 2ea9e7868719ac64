#!/bin/bash
# Perf session: A/B of kernel variants + PMC passes on the C2 render kernel.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
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
run pytest_gpu 600 python -m pytest tests -m gpu -q -rf
run ab_trav 300 python3 scripts/render_loop.py --frames 20 --ab CRT_TRAVERSAL=1,2,3
run ab_order 300 python3 scripts/render_loop.py --frames 20 --ab CRT_TILE_ORDER=0,1
run ab_trav_c3 300 python3 scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 10 --ab CRT_TRAVERSAL=1,2,3
run ab_trav_c4 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 3 --ab CRT_TRAVERSAL=1,2,3
run counters 120 rocprofv3 -L
for T in 2 3; do
export CRT_TRAVERSAL=$T
run pmc_sq_$T 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc/sq_$T -o run --output-format csv -- python3 scripts/render_loop.py --frames 2
done
unset CRT_TRAVERSAL
run pmc_inst 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH -d gpurun_out/pmc/inst -o run --output-format csv -- python3 scripts/render_loop.py --frames 2
run pmc_mem 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc/mem -o run --output-format csv -- python3 scripts/render_loop.py --frames 2
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run --output-format csv -- python3 scripts/render_loop.py --frames 2
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run --output-format csv -- python3 scripts/render_loop.py --frames 2
exit 0
