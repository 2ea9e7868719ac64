#!/bin/bash
# Same-box A/B of abtest/old vs abtest/new on C4 (15-01/scene2 GI, 1080^2), then the GPU tests.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-abc4} BUILDS="old new" SCN="--scene 15-01-conclusion__scene2 --width 1080 --height 1080 --frames 4" bash scripts/gpu_ab_scene.sh || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-abc4}/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG:-abc4}/pytest.log; exit $rc
