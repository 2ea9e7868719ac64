#!/bin/bash
# Same-box A/B of abtest/old vs abtest/new on C4 (1080^2), C3, C2, then the GPU tests.
set -u
cd "$(dirname "$0")/.."
T=${TAG:-aball}
TAG=${T}_c4 BUILDS="old new" SCN="--scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4" bash scripts/gpu_ab_scene.sh || exit $?
TAG=${T}_c3 BUILDS="old new" SCN="--scene 11-01-refractive__scene8 --depth 8 --frames 10" bash scripts/gpu_ab_scene.sh || exit $?
TAG=${T}_c2 BUILDS="old new" SCN="--frames 60" bash scripts/gpu_ab_scene.sh || exit $?
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$T/pytest.log; exit $rc
