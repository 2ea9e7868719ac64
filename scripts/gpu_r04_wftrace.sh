set -e
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04_wftrace -o run -- python3 $R/bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r04_wftrace.log 2>&1
cd $R && ls gpurun_out/r04_wftrace
grep -h '^{"metric"' gpurun_out/r04_wftrace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config'].get('e2e_ms'), d['config'].get('cold_cli'))"
