set -e
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u scripts/bins_check_run.py > gpurun_out/r04_chk9.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_gpu9.log 2>&1
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_prof12 -o run -- python3 $R/scripts/render_loop.py --frames 30 > $R/gpurun_out/r04_p12.log 2>&1
cd $R && tail -1 gpurun_out/r04_chk9.log && tail -1 gpurun_out/r04_gpu9.log && python3 scripts/kstats.py gpurun_out/r04_prof12/run_kernel_stats.csv | head -5 && grep kernel gpurun_out/r04_p12.log
