// rt_kernel.hip — MI355X (gfx950, CDNA4) kernels: the path-tracing megakernel and the 8-bit
// output epilogue.  The per-lane logic lives in rt_trace.h.
//
// Launch shape: 256-lane workgroups (4 waves), one lane per tile pixel, consecutive lanes on
// consecutive pixels of a row (coherent primary rays, coalesced output).  Each lane keeps a
// BVH traversal stack of RT_STACK_DEPTH entries in LDS, laid out [depth][lane] so the 64
// lanes of a wave touch 64 consecutive dwords (conflict-free).  No MFMA: the work is branchy
// scalar FP32, not a contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_trace.h"

__global__ __launch_bounds__(RT_BLOCK) void rt_render_kernel(KernelParams P) {
  __shared__ int stack_mem[RT_STACK_DEPTH * RT_BLOCK];
  const int tile_pixel = blockIdx.x * RT_BLOCK + threadIdx.x;
  if (tile_pixel >= P.tile_rows * P.cam.width) return;
  int overflow = rtk::render_pixel(P, tile_pixel, stack_mem + threadIdx.x, RT_BLOCK);
  if (overflow) atomicOr(P.status, 1);
}

// Output epilogue of writeImage / writeImageSqrt (Ray.hs:248-260): 8-bit codes
// min(255, floor(256 * transfer(clamp01 x))).  Memory-bound, 16 B in / 4 B out per lane.
__global__ __launch_bounds__(256) void rt_encode8_kernel(const float* __restrict__ in, uint8_t* __restrict__ out,
                                                         int64_t n, int encoding) {
  int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  for (; i < n; i += (int64_t)gridDim.x * 256 * 4) {
    float v[4];
    const bool full = i + 4 <= n && ((reinterpret_cast<uintptr_t>(in + i) & 15) == 0);
    if (full) {
      float4 q = *reinterpret_cast<const float4*>(in + i);
      v[0] = q.x;
      v[1] = q.y;
      v[2] = q.z;
      v[3] = q.w;
    } else {
      for (int k = 0; k < 4; ++k) v[k] = (i + k < n) ? in[i + k] : 0.0f;
    }
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float x = fminf(1.0f, fmaxf(0.0f, v[k]));
      float e;
      if (encoding == 1)
        e = sqrtf(x);
      else
        e = x <= 0.0031308f ? 12.92f * x : 1.055f * powf(x, 1.0f / 2.4f) - 0.055f;
      int code = (int)floorf(256.0f * e);
      code = code > 255 ? 255 : (code < 0 ? 0 : code);
      packed |= (uint32_t)code << (8 * k);
    }
    if (i + 4 <= n && ((reinterpret_cast<uintptr_t>(out + i) & 3) == 0)) {
      *reinterpret_cast<uint32_t*>(out + i) = packed;
    } else {
      for (int k = 0; k < 4 && i + k < n; ++k) out[i + k] = (uint8_t)(packed >> (8 * k));
    }
  }
}

int rt_launch_render(const KernelParams& p, void* stream) {
  int n = p.tile_rows * p.cam.width;
  if (n <= 0) return 0;
  dim3 grid((n + RT_BLOCK - 1) / RT_BLOCK);
  hipLaunchKernelGGL(rt_render_kernel, grid, dim3(RT_BLOCK), 0, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_encode8(const float* in, uint8_t* out, int64_t n, int encoding, void* stream) {
  if (n <= 0) return 0;
  int64_t blocks = (n / 4 + 255) / 256 + 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(rt_encode8_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, out, n,
                     encoding);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
