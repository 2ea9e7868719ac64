#!/bin/bash
# Per-shard render times of the sharded C2 frame (scripts/shard_times.py) for
# plan options given as arguments ("" = defaults), plus an in-process A/B of
# calib_min.  Each GPU step under its own time limit; stop on the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/shards
timeout -k 10 240 python scripts/render_loop.py --frames 40 --opt calib_min=2,1 > gpurun_out/shards/ab_min.log 2>&1 || { tail -5 gpurun_out/shards/ab_min.log; exit 1; }
tail -1 gpurun_out/shards/ab_min.log
for o in "$@"; do
  tag=$(echo "$o" | tr -c 'a-z0-9' '_')
  timeout -k 10 240 python scripts/shard_times.py $o --out gpurun_out/shards/s$tag.json > gpurun_out/shards/s$tag.log 2>&1 || { echo "fail $o"; tail -5 gpurun_out/shards/s$tag.log; exit 1; }
  tail -1 gpurun_out/shards/s$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['opts'], d['plan'], {n: (round(v['max_ms'],4), v['speedup_vs_n1']) for n, v in d['shards'].items()})"
done
