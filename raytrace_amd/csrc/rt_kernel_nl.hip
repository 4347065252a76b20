// rt_kernel_nl.hip — the FP32 render-kernel instantiations built without MachineLICM (compiled
// with -mllvm -disable-machine-licm, Makefile NOLICM): the classes RT_NOLICM_OF selects
// (rt_render_kernel.h), whose loop-invariant constants the pass would hoist into VGPRs for the
// whole persistent lane loop.  rt_kernel.hip holds the rest and the launchers.
#define RT_F64 0
#define RT_TU_NOLICM 1
#include "rt_render_kernel.h"
