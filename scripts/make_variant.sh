#!/bin/bash
# Build a variant of the library for same-box A/B runs: the package is copied to
# /tmp/crt_variant/<name>, built there with extra make variables, and its lib/ +
# crt_amd/ land in abtest/<name>/ (render_loop.py: CRT_PKG=abtest/<name>).
#   bash scripts/make_variant.sh <name> [MAKEVAR=value ...]
#   e.g. bash scripts/make_variant.sh nosink RENDER_FLAGS="-mllvm -disable-machine-sink"
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
W=/tmp/crt_variant/$NAME
rm -rf "$W" && mkdir -p "$W"
mkdir -p "$W/include" && cp include/crt_hip.h "$W/include/"
mkdir -p "$W/pkg" && cp -r chaos-ray-tracing-course-2025_amd/Makefile chaos-ray-tracing-course-2025_amd/csrc chaos-ray-tracing-course-2025_amd/crt_amd "$W/pkg/"
make -s -j8 -C "$W/pkg" lib ARCH=gfx950 "$@"
mkdir -p abtest/$NAME
rm -rf abtest/$NAME/lib abtest/$NAME/crt_amd
cp -r "$W/pkg/lib" "$W/pkg/crt_amd" abtest/$NAME/
echo "abtest/$NAME: $(ls abtest/$NAME/lib)"
