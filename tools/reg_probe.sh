#!/bin/bash
# Registers / spills / occupancy of ONE render-kernel instantiation (seconds instead of the whole
# library): tools/reg_probe.sh <f64|f32> <kVar> <kTex> <kMedia> <kMats> <kLeaf> [-Dmacro ...]
# e.g. tools/reg_probe.sh f64 2 0 true true 1      (pawn+fog's binary64 kernel)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$1; V=$2; T=$3; M=$4; A=$5; L=$6; shift 6
F64=$([ "$P" = f64 ] && echo 1 || echo 0); NS=$([ "$P" = f64 ] && echo rtk64 || echo rtk)
SRC=$(mktemp --suffix .hip)
printf '#define RT_F64 %s\n#define RT_KERNEL_ONLY 1\n#include "rt_render_kernel.h"\ntemplate __global__ void %s::rt_render_kernel<%s, %s, %s, %s, %s, %s>(KernelParams);\n' \
  $F64 $NS $V $T $M $A ${RP_INST:-false} $L > $SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-slp-vectorize \
  -fgpu-flush-denormals-to-zero -I${RP_SRC:-$ROOT/raytrace_amd/csrc} "$@" -c $SRC -o ${SRC%.hip}.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//; s/ *\[-Rpass.*//; p' |
  awk '/Function Name:/{n=$3} /^VGPRs:/{v=$2} /VGPRs Spill:/{vs=$3} /SGPRs Spill:/{ss=$3} /ScratchSize/{sc=$NF} /Occupancy/{o=$NF} /LDS Size/{ if (n ~ /rt_render_kernel/) print "vgpr", v, "vspill", vs, "sspill", ss, "scratch", sc, "occ", o}'
rm -f $SRC ${SRC%.hip}.o
