set -u
mkdir -p gpurun_out/abkm2
CRT_PKG=abtest/km2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_png_pins.py -m gpu -k "c2_full or window or pngs or png or shadow or render_matches" -x -q --timeout 200 --timeout-method thread > gpurun_out/abkm2/tests.log 2>&1 || { tail -20 gpurun_out/abkm2/tests.log; exit 1; }
tail -2 gpurun_out/abkm2/tests.log
TAG=abkm2 bash scripts/gpu_ab_variant.sh km2
