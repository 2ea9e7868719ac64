set -u
mkdir -p gpurun_out/absched2
for round in 1 2 3; do
  timeout -k 10 240 python scripts/render_loop.py --frames 80 > gpurun_out/absched2/base_$round.log 2>&1 || exit 1
  CRT_PKG=abtest/silp timeout -k 10 240 python scripts/render_loop.py --frames 80 > gpurun_out/absched2/silp_$round.log 2>&1 || exit 1
  for v in base silp; do tail -1 gpurun_out/absched2/${v}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']['default']; print('$v', $round, round(d['median_ms'],5), round(d['min_ms'],5))"; done
done
