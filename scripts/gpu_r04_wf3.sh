# wavefront buffer sets: main (12/12, 16 GiB budget) vs s8t8, C3 bench lines
set -e
export TMPDIR=/tmp
for v in main s8t8 main s8t8; do
  if [ $v = main ]; then P=$PWD/chaos-ray-tracing-course-2025_amd; else P=$PWD/abtest/$v; fi
  CRT_PKG=$P timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r04_wf3_$v.json 2>/dev/null
  echo "$v $(python3 -c "import json; d=json.loads(open('gpurun_out/r04_wf3_$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
done
