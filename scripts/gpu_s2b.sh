#!/bin/bash
# Session-2 GPU steps (STEPS=tests,gi,cold,clitrace,bins,bench,shards,timeline), each under its own limit.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s2b}; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
[[ ${STEPS:-tests} == *tests* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
[[ ${STEPS:-tests} == *gi* ]] && run c4_1080_bitmap 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4 --opt gi_bitmap=0,1
[[ ${STEPS:-tests} == *gi* ]] && run c4_4k_bitmap 300 python3 scripts/render_loop.py --scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 3 --opt gi_bitmap=0,1
[[ ${STEPS:-tests} == *cold* ]] && run cold_c2 300 python3 scripts/cold_breakdown.py --config c2 --out $OUT/cold_c2.json --keep $OUT/scene
[[ ${STEPS:-tests} == *clitrace* ]] && run cli_trace 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $OUT/clitrace -o run --output-format csv -- chaos-ray-tracing-course-2025_amd/bin/crt_renderer $OUT/scene/scene.crtscene $OUT/scene/out.ppm --gpus 1
[[ ${STEPS:-tests} == *cold* ]] && run cold_parts 200 python3 scripts/cold_parts.py
[[ ${STEPS:-tests} == *bins* ]] && run c2_bins 300 python3 scripts/render_loop.py --frames 40 --opt bins=0,1 --counts
[[ ${STEPS:-tests} == *bench* ]] && run bench_c2 600 python3 bench.py --steps 50 --warmup 5
[[ ${STEPS:-tests} == *shards* ]] && run shards_c2 300 python3 scripts/shard_times.py --config c2 --reps 20 --out $OUT/shards_c2.json
[[ ${STEPS:-tests} == *timeline* ]] && run timeline_c2 300 python3 scripts/wave_timeline.py --out $OUT/timeline_c2.json
exit 0
