# C5 A/B: main vs abtest/<variants> (bench lines, 4K 1 M triangles)
set -e
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = main ]; then P=$PWD/chaos-ray-tracing-course-2025_amd; else P=$PWD/abtest/$v; fi
  CRT_PKG=$P timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/c5ab_$v.json 2>/dev/null
  echo "$v $(python3 -c "import json; print(json.loads(open('gpurun_out/c5ab_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
