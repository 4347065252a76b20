#!/bin/bash
# Build an experiment library from a copy of raytrace_amd/csrc with some files replaced.
# usage: tools/build_variant.sh NAME [DEFS] [file=replacement ...]
#   e.g. tools/build_variant.sh old "" rt_trace.h=/tmp/old/rt_trace.h
set -e
NAME=$1; DEFS=$2; shift 2 || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
mkdir -p "$W/raytrace_amd/csrc" "$W/include" "$ROOT/raytrace_amd/_lib/exp"
cp "$ROOT"/raytrace_amd/csrc/* "$W/raytrace_amd/csrc/"
cp "$ROOT"/include/* "$W/include/"
for r in "$@"; do cp "${r#*=}" "$W/raytrace_amd/csrc/${r%%=*}"; done
cd "$W/raytrace_amd/csrc"
make -s exp NAME="$NAME" DEFS="$DEFS"  # the Makefile's own flags
mkdir -p "$ROOT/raytrace_amd/_lib/exp"
cp "$W/raytrace_amd/_lib/exp/librt_amd_$NAME.so" "$ROOT/raytrace_amd/_lib/exp/"
rm -rf "$W"
