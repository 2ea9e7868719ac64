#!/bin/bash
# C2 bench: per-render HIP events every k-th step (1 = every render) — cost of the timing events
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-bench_ev}
mkdir -p "$OUT"
for r in 1 2; do
  for k in 1 5 1000; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 10 --event-every $k > "$OUT/ev${k}_$r.json" 2> "$OUT/ev${k}_$r.err" || exit $?
    echo "every $k: $(python3 -c "import json;d=json.loads(open('$OUT/ev${k}_$r.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['kernel_ms'], d['value'])")"
  done
done
