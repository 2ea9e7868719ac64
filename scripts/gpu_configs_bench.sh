set -u
TAG=r01u bash scripts/gpu_configs.sh || exit $?
for c in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 > gpurun_out/r01u/bench_$c.json 2>gpurun_out/r01u/bench_$c.err || exit $?
  tail -1 gpurun_out/r01u/bench_$c.json
done
