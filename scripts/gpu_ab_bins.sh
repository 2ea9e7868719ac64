# A/B of camera-bins builds: rocprof kernel stats of render_loop (C2) per build in abtest/<name>
set -e
export TMPDIR=/tmp
R=$PWD
for v in "$@"; do
  if [ "$v" = main ]; then P=$R/chaos-ray-tracing-course-2025_amd; else P=$R/abtest/$v; fi
  cd /tmp && CRT_PKG=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$v -o run -- python3 $R/scripts/render_loop.py --frames 30 > $R/gpurun_out/ab_$v.log 2>&1
  cd $R && echo "== $v" && python3 scripts/kstats.py gpurun_out/ab_$v/run_kernel_stats.csv | head -4
done
