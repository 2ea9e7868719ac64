# binning stream priority: main (default) vs abtest/lo (lowest), abtest/hi (highest), C2 bench lines
set -e
export TMPDIR=/tmp
for v in main lo hi main lo hi; do
  if [ $v = main ]; then P=$PWD/chaos-ray-tracing-course-2025_amd; else P=$PWD/abtest/$v; fi
  CRT_PKG=$P timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > gpurun_out/r04_c2sets_$v.json 2>/dev/null
  echo "$v $(python3 -c "import json; d=json.loads(open('gpurun_out/r04_c2sets_$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('frame_ms_one_at_a_time'))")"
done
