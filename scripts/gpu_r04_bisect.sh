# proof treelets (KTopo2) on / off on C4, C3, C2 (same box), then the GPU suite
set -e
export TMPDIR=/tmp
ARGS="--scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 3" bash scripts/gpu_ab_render.sh v_98658a9 main topo1 > gpurun_out/r04_ab3_c4.log 2>&1
ARGS="--scene 11-01-refractive__scene8 --depth 8 --frames 10" bash scripts/gpu_ab_render.sh v_98658a9 main topo1 main topo1 > gpurun_out/r04_ab3_c3.log 2>&1
ARGS="--frames 30" bash scripts/gpu_ab_render.sh v_98658a9 main topo1 main topo1 > gpurun_out/r04_ab3_c2.log 2>&1
for f in c4 c3 c2; do echo "== $f"; grep -o '^== .*\|median_ms": [0-9.]*' gpurun_out/r04_ab3_$f.log | tr '\n' ' '; echo; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu11.log 2>&1
tail -1 gpurun_out/r04_gpu11.log
