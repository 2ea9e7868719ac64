# wavefront frames pipeline (C3): wavefront + GPU suite, C3 render loop and bench
set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "c3" > gpurun_out/r04_wf1.log 2>&1
tail -1 gpurun_out/r04_wf1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu13.log 2>&1
tail -1 gpurun_out/r04_gpu13.log
timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_bench_c3pipe.json 2> gpurun_out/r04_bench_c3pipe.err
python3 -c "import json; d=json.loads(open('gpurun_out/r04_bench_c3pipe.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['config'].get('e2e_ms'), d['config'].get('cold_cli'))"
