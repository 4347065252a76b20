#!/bin/bash
# Kernel resource table (VGPRs, spills, scratch, occupancy) of the render kernels of one source
# file, optionally side by side with another tree's: tools/resource_diff.sh rt_kernel64.hip [/tmp/base]
SRC=${1:-rt_kernel64.hip}; BASE=$2
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-slp-vectorize -fgpu-flush-denormals-to-zero"
table() {
  (cd $1/raytrace_amd/csrc && /opt/rocm/bin/hipcc $FLAGS -c $SRC -o /tmp/res_$$.o -Rpass-analysis=kernel-resource-usage 2>&1) |
    sed -n 's/.*remark: *//; s/ *\[-Rpass.*//; p' |
    awk '/Function Name:/{n=$3; sub(/.*rt_render_kernel/,"",n); sub(/EEEv13KernelParams.*/,"",n)}
         /^VGPRs:/{v=$2} /VGPRs Spill:/{vs=$3} /SGPRs Spill:/{ss=$3} /ScratchSize/{sc=$NF}
         /Occupancy/{o=$NF} /LDS Size/{ if (n ~ /^I/) printf "%-22s vgpr %3s vspill %3s sspill %3s scratch %4s occ %s\n", n, v, vs, ss, sc, o}'
}
if [ -n "$BASE" ]; then paste <(table $BASE) <(table /root/repo | cut -c23-) ; else table /root/repo; fi
