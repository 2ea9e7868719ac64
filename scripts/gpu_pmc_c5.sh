#!/bin/bash
# C5 (synthetic 1M triangles, 3840x2160): kernel trace + PMC passes of the
# render kernel (one counter group per pass) -> profiles-ready pmc_c5.json
# (bench.py --config c5 reads profiles/r02/pmc_c5.json when its build id matches).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc_c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
C5="scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 2"
step() {   # name, limit, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
}
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $C5
step inst 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d "$OUT/pmc/inst" -o run --output-format csv -- python3 $C5
step sq 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/pmc/sq" -o run --output-format csv -- python3 $C5
step fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc/fetch" -o run --output-format csv -- python3 $C5
step write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc/write" -o run --output-format csv -- python3 $C5
step tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc/tcc" -o run --output-format csv -- python3 $C5
step record 120 python3 scripts/pmc_record.py --config c5 --size 3840 2160 --dir "$OUT/pmc" --out "$OUT/pmc_c5.json" --last 2 --command "python3 $C5"
tail -1 "$OUT/record.log" | cut -c1-600
grep -h "k_render_tiles" "$OUT"/trace/*kernel_stats.csv | head -3
exit 0
