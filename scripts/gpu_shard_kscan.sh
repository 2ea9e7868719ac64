set -u
mkdir -p gpurun_out/kscan
for k in 2000 2500 3000 4000 6000; do
  timeout -k 10 200 python scripts/shard_times.py --counts 1,8 --opt calib_k_milli=$k > gpurun_out/kscan/k$k.log 2>&1 || { echo fail $k; exit 1; }
  tail -1 gpurun_out/kscan/k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['plan'], {n:(round(v['max_ms'],4)) for n,v in d['shards'].items()})"
done
