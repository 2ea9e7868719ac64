#!/bin/bash
# Kernel trace + PMC passes (one counter group per pass, MI355X_MICROARCH.md)
# of one config's render kernel -> gpurun_out/<TAG>/pmc_<CFG>.json (bench.py
# reads profiles/r05/pmc_<CFG>.json when its build id equals the library's).
#   TAG=x CFG=c4 KERNEL=k_render_refill SIZE="3840 2160" LAST=2 CMD="scripts/render_loop.py ..." bash scripts/gpu_pmc.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc}/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # name, limit, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
}
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $CMD
step inst 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d "$OUT/pmc/inst" -o run --output-format csv -- python3 $CMD
step sq 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/pmc/sq" -o run --output-format csv -- python3 $CMD
step fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc/fetch" -o run --output-format csv -- python3 $CMD
step write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc/write" -o run --output-format csv -- python3 $CMD
step tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc/tcc" -o run --output-format csv -- python3 $CMD
step record 120 python3 scripts/pmc_record.py --config $CFG --size $SIZE --kernel $KERNEL --dir "$OUT/pmc" --out "$OUT/pmc_$CFG.json" --last ${LAST:-2} ${FRAME_END:+--frame-end $FRAME_END} --command "python3 $CMD"
tail -1 "$OUT/record.log" | cut -c1-900
grep -h "$KERNEL" "$OUT"/trace/*kernel_stats.csv | head -3
exit 0
