// rt_kernel.hip — MI355X (gfx950, CDNA4) kernels: the persistent path-tracing megakernel and
// the fixed-point resolve in FP32 (the opt-in fast path; rt_kernel64.hip builds the binary64
// default from the same rt_render_kernel.h), and the 8-bit output epilogue.  The per-lane logic
// lives in rt_trace.h.
//
// rt_render_kernel: a grid of exactly the resident workgroups (occupancy query), instantiated per
// scene class (texture level, media, materials, leaf class, instancing; see render_kernel_of).
// Workgroups: one wave (64 lanes) for the flat kernels; 768 or 1024 lanes for the BVH classes at
// 3 / 6 or 4 / 8 waves per SIMD, 256 otherwise (rt_render_kernel.h RT_BLOCK_OF; 512-lane twins for
// deep BVHs).  Waves start with a static pool of item ids and refill it with one returning
// atomicAdd on one of four queue heads (ballot the lanes that need work; ids are handed out in
// lane order); ids are
// pixel-major, so a pool covers a few pixels (coherent primary rays) and its items' int64
// fixed-point sums are added up per pixel in the wave's LDS slot before one 64-bit atomic per
// word goes to HBM (commutative: bit-exact for any schedule; rt_render_kernel.h WaveWork).  Each
// lane keeps its BVH traversal stack in LDS, laid out [depth][lane]: the 64 lanes of a wave touch
// 64 consecutive dwords (conflict-free).  The stack depth is the scene's BVH depth (dynamic LDS),
// so shallow scenes are not occupancy-limited by LDS.
// No MFMA: the work is branchy scalar floating point, not a contraction.
#define RT_F64 0
#include "rt_render_kernel.h"

// Output epilogue of writeImage / writeImageSqrt (Ray.hs:248-260): 8-bit codes
// min(255, floor(256 * transfer(clamp01 x))), transfer = sRGB or sqrt, as the number of code
// thresholds <= x (rt_encode8_table.h: per code, the smallest binary64 with that code under the
// exactly evaluated transfer) — a binary search in an LDS copy of the 256-entry table, no
// transcendental, so the device codes equal the host encoder's (raytrace_amd.ray.encode8, same
// table) bit for bit on every input.  NaN encodes as 0.  Memory-bound: 4 values per lane.
struct Enc8Table {
  double thr[256];
};
template <bool kF64>
__global__ __launch_bounds__(256) void rt_encode8_kernel(const void* __restrict__ in_, uint8_t* __restrict__ out,
                                                         int64_t n, Enc8Table T) {
  __shared__ double thr[256];
  thr[threadIdx.x] = T.thr[threadIdx.x];
  __syncthreads();
  const float* inf = (const float*)in_;
  const double* ind = (const double*)in_;
  int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  for (; i < n; i += (int64_t)gridDim.x * 256 * 4) {
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double x = (i + k < n) ? (kF64 ? ind[i + k] : (double)inf[i + k]) : 0.0;
      int code = 0;  // largest k with thr[k] <= x (thr[0] = 0; NaN and x < thr[1] -> 0)
#pragma unroll
      for (int step = 128; step >= 1; step >>= 1) code = thr[code + step] <= x ? code + step : code;
      packed |= (uint32_t)code << (8 * k);
    }
    if (i + 4 <= n && ((reinterpret_cast<uintptr_t>(out + i) & 3) == 0)) {
      *reinterpret_cast<uint32_t*>(out + i) = packed;
    } else {
      for (int k = 0; k < 4 && i + k < n; ++k) out[i + k] = (uint8_t)(packed >> (8 * k));
    }
  }
}

int rt_launch_encode8(const void* in, int in_f64, uint8_t* out, int64_t n, const double* thr, int encoding,
                      void* stream) {
  (void)encoding;  // the table is the encoding
  if (n <= 0) return 0;
  int64_t blocks = (n / 4 + 255) / 256 + 1;
  if (blocks > 4096) blocks = 4096;
  Enc8Table T;
  for (int k = 0; k < 256; ++k) T.thr[k] = thr[k];
  if (in_f64)
    hipLaunchKernelGGL(rt_encode8_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, out, n,
                       T);
  else
    hipLaunchKernelGGL(rt_encode8_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, out, n,
                       T);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
