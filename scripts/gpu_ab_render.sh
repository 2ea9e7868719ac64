# A/B of builds on one render_loop command: ARGS="<render_loop args>" bash scripts/gpu_ab_render.sh main <variant> ...
set -e
export TMPDIR=/tmp
R=$PWD
for v in "$@"; do
  if [ "$v" = main ]; then P=$R/chaos-ray-tracing-course-2025_amd; else P=$R/abtest/$v; fi
  echo "== $v"
  CRT_PKG=$P timeout -k 10 300 python3 scripts/render_loop.py $ARGS 2>&1 | tail -1 | cut -c1-400
done
