# kernel trace of the C2 bench (frames back to back): the render kernel's duration and the gaps between renders
set -e
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c2trace -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > $R/gpurun_out/c2trace.log 2>&1
cd $R && python3 scripts/kernel_gaps.py gpurun_out/c2trace/run_kernel_trace.csv --match '0, 15, 15, false' --skip 20 --count 200
