set -u
export TAG=r01n
BUILDS="old new" SCN="--scene 11-01-refractive__scene8 --depth 8 --frames 8" bash scripts/gpu_ab_scene.sh || exit $?
TAG=r01n4 BUILDS="old new" SCN="--scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 2" bash scripts/gpu_ab_scene.sh || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01n/pytest.log 2>&1; echo pytest rc=$?; tail -2 gpurun_out/r01n/pytest.log
