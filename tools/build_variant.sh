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
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics $DEFS \
  -shared -o "$ROOT/raytrace_amd/_lib/exp/librt_amd_$NAME.so" rt_api.hip rt_kernel.hip rt_bvh.cpp rt_build.cpp
rm -rf "$W"
