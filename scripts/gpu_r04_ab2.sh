# round-4 A/B: proof treelets (topo1 = one KTopo a level), GI pair steps, walk_bvh pair steps, round 3's build
set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu10.log 2>&1
tail -1 gpurun_out/r04_gpu10.log
ARGS="--scene 15-01-conclusion__scene2 --width 3840 --height 2160 --frames 4" bash scripts/gpu_ab_render.sh main r3 gimpair0 topo1 main r3 > gpurun_out/r04_ab_c4.log 2>&1
ARGS="--scene 11-01-refractive__scene8 --depth 8 --frames 10" bash scripts/gpu_ab_render.sh main topo1 bvhpair r3 main topo1 bvhpair > gpurun_out/r04_ab_c3.log 2>&1
ARGS="--frames 30" bash scripts/gpu_ab_render.sh main topo1 main topo1 > gpurun_out/r04_ab_c2.log 2>&1
for f in c4 c3 c2; do echo "== $f"; grep -o '"== .*\|median_ms": [0-9.]*' gpurun_out/r04_ab_$f.log | tr '\n' ' '; echo; done
