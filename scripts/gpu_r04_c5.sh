# C5 (1M-triangle synthetic mesh at 4K): camera bins (no BVH) vs the pruned kd packet walk; the C5 tests
set -e
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 10 --opt bins=1,0 > gpurun_out/r04_c5_ab.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or bins" > gpurun_out/r04_c5_test.log 2>&1
tail -1 gpurun_out/r04_c5_ab.log; tail -1 gpurun_out/r04_c5_test.log
