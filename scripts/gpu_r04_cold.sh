set -e
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04_c3_cold.json 2> gpurun_out/r04_c3_cold.err
timeout -k 10 600 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04_c4_cold.json 2> gpurun_out/r04_c4_cold.err
