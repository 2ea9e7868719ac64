# kernel trace of the C3 bench (frames back to back): how many wavefront levels run side by side
set -e
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c3trace -o run -- python3 $R/bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $R/gpurun_out/c3trace.log 2>&1
cd $R && f=$(ls gpurun_out/c3trace/*kernel_trace.csv gpurun_out/c3trace/*/*kernel_trace.csv 2>/dev/null | head -1) && python3 scripts/kernel_overlap.py $f --match k_wf_level --last 160 && python3 scripts/kernel_overlap.py $f --match k_wf_ --last 400
