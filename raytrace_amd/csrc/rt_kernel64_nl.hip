// rt_kernel64_nl.hip — the binary64 render-kernel instantiations built without MachineLICM
// (compiled with -mllvm -disable-machine-licm, Makefile NOLICM): the classes RT_NOLICM_OF selects
// (rt_render_kernel.h).  rt_kernel64.hip holds the rest and the launchers.
#define RT_F64 1
#define RT_TU_NOLICM 1
#include "rt_render_kernel.h"
