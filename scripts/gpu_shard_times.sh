set -u
mkdir -p gpurun_out/shards
for o in "" "--opt calib_min=1" "--opt calib_k_milli=1500" "--opt calib_k_milli=1000 --opt calib_min=1"; do
  tag=$(echo "$o" | tr -c 'a-z0-9' '_')
  timeout -k 10 240 python scripts/shard_times.py $o --out gpurun_out/shards/s$tag.json > gpurun_out/shards/s$tag.log 2>&1 || { echo "fail $o"; tail -5 gpurun_out/shards/s$tag.log; exit 1; }
  tail -1 gpurun_out/shards/s$tag.log | cut -c1-900
done
