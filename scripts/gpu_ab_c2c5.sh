#!/bin/bash
# Same-box A/B of abtest/old vs abtest/new on C2 (14-01/scene1 1080p) and C5 (1 M triangles, 4K), then GPU tests.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-abc2}
TAG=$TAG BUILDS="old new" SCN="--frames 60" bash scripts/gpu_ab_scene.sh || exit $?
TAG=${TAG}_c5 BUILDS="old new" SCN="--synthetic 1000000 --width 3840 --height 2160 --frames 4" bash scripts/gpu_ab_scene.sh || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$TAG/pytest.log; exit $rc
