# hardware queues per process (GPU_MAX_HW_QUEUES: 4 = the box's default) vs C3 / C2 frames back to back
set -e
export TMPDIR=/tmp
for q in 4 8 16 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/hwq_c3_$q.json 2>/dev/null
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > gpurun_out/hwq_c2_$q.json 2>/dev/null
  echo "q=$q c3 $(python3 -c "import json; print(json.loads(open('gpurun_out/hwq_c3_$q.json').read().strip().splitlines()[-1])['ms_per_step'])") c2 $(python3 -c "import json; print(json.loads(open('gpurun_out/hwq_c2_$q.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
