set -e
ARGS="--scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 4" bash scripts/gpu_ab_render.sh main gimpair0 main gimpair0 > gpurun_out/r04_gim_ab.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gi or c4 or png or conclusion" > gpurun_out/r04_gim_test.log 2>&1
cat gpurun_out/r04_gim_ab.log; tail -1 gpurun_out/r04_gim_test.log
