#!/bin/bash
# Build a variant of the library for same-box A/B runs: the package is copied to
# /tmp/crt_variant/<name>, built there with extra make variables, and its lib/ +
# crt_amd/ land in abtest/<name>/ (render_loop.py: CRT_PKG=abtest/<name>).
#   bash scripts/make_variant.sh <name> [MAKEVAR=value ...]
#   e.g. bash scripts/make_variant.sh nosink RENDER_FLAGS="-mllvm -disable-machine-sink"
#   REV=<git rev> builds that commit's sources instead of the working tree.
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
W=/tmp/crt_variant/$NAME
rm -rf "$W" && mkdir -p "$W"
SRC=.
if [ -n "${REV:-}" ]; then
  SRC=$W/src && mkdir -p "$SRC" && git archive "$REV" include chaos-ray-tracing-course-2025_amd | tar -x -C "$SRC"
fi
mkdir -p "$W/include" && cp "$SRC/include/crt_hip.h" "$W/include/"
mkdir -p "$W/pkg" && cp -r "$SRC"/chaos-ray-tracing-course-2025_amd/{Makefile,csrc,crt_amd} "$W/pkg/"
make -s -j8 -C "$W/pkg" lib ARCH=gfx950 "$@"
mkdir -p abtest/$NAME
rm -rf abtest/$NAME/lib abtest/$NAME/crt_amd
cp -r "$W/pkg/lib" "$W/pkg/crt_amd" abtest/$NAME/
echo "abtest/$NAME: $(ls abtest/$NAME/lib)"
