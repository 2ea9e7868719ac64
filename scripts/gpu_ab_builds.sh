#!/bin/bash
# Same-box A/B of several builds (abtest/<name>/{lib,crt_amd}) on C2 and C5,
# interleaved rounds; BUILDS="w1 w4 w5 w6", BASE_ENV = env of the baseline run.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abbuilds}
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 120 env CRT_PKG=abtest/${BASE:-w1} python3 scripts/render_loop.py --frames 30 --opt window=0 > "$OUT/base_c2_$r.json" 2>&1 || exit $?
  echo "base c2 $(tail -1 $OUT/base_c2_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["default"]["median_ms"])')"
  for b in ${BUILDS:-w1 w4 w5 w6}; do
    timeout -k 10 120 env CRT_PKG=abtest/$b python3 scripts/render_loop.py --frames 30 > "$OUT/${b}_c2_$r.json" 2>&1 || exit $?
    echo "$b c2 $(tail -1 $OUT/${b}_c2_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["default"]["median_ms"])')"
  done
done
for b in ${BUILDS:-w1 w4 w5 w6}; do
  timeout -k 10 120 env CRT_PKG=abtest/$b python3 scripts/render_loop.py --synthetic 1000000 --width 3840 --height 2160 --frames 3 > "$OUT/${b}_c5.json" 2>&1 || exit $?
  echo "$b c5 $(tail -1 $OUT/${b}_c5.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["default"]["median_ms"])')"
done
exit 0
