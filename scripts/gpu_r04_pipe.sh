# frames pipeline of the camera bins: check build, bins tests, GPU suite, C2 profile and bench
set -e
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u scripts/bins_check_run.py > gpurun_out/r04_chk10.log 2>&1
tail -1 gpurun_out/r04_chk10.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_bins.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_bins12.log 2>&1
tail -1 gpurun_out/r04_bins12.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu12.log 2>&1
tail -1 gpurun_out/r04_gpu12.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r04_bench_pipe.json 2> gpurun_out/r04_bench_pipe.err
python3 -c "import json; d=json.loads(open('gpurun_out/r04_bench_pipe.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['config'].get('e2e_ms'), d['config'].get('cold_cli'), d['config'].get('camera_bins'))"
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_prof13 -o run -- python3 $R/scripts/render_loop.py --frames 30 > $R/gpurun_out/r04_p13.log 2>&1
cd $R && grep kernel gpurun_out/r04_p13.log | cut -c1-300
