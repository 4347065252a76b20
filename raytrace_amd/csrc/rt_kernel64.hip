// rt_kernel64.hip — the binary64 instantiation of the render megakernel and its resolve
// (rt_render_kernel.h with RT_F64 = 1, namespace rtk64): the reference's arithmetic (`V3 Double`,
// Core.hs:29-31) and the C ABI's default precision.  Same scheduling, Philox stream and
// fixed-point accumulation (two words per channel) as the FP32 instantiation in rt_kernel.hip.
#define RT_F64 1
#include "rt_render_kernel.h"
