// valu_rates.hip — calibration of the VALU issue roofline (bench.py `roofline`): the chip-wide
// throughput of each instruction class the render kernel's PMC mix counts (SQ_INSTS_VALU_*),
// measured with every CU full of waves issuing independent chains of that instruction.
// Prints one JSON object: class -> G wave64-instructions/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#define ITERS 4096
#define CHAINS 8

template <int kOp>
__global__ __launch_bounds__(256) void bench(double* out, float* outf, unsigned long long* outi, double seed) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  double d[CHAINS];
  float f[CHAINS];
  unsigned u[CHAINS];
  unsigned long long q[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    d[c] = seed + 1e-3 * (t + c);
    f[c] = (float)d[c];
    u[c] = (unsigned)(t * 7 + c);
    q[c] = u[c];
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (kOp == 0) f[c] = __builtin_fmaf(f[c], 0.999f, 1e-3f);                       // v_fma_f32
      if constexpr (kOp == 1) d[c] = __builtin_fma(d[c], 0.999, 1e-3);                           // v_fma_f64
      if constexpr (kOp == 2) d[c] = d[c] * 0.999;                                               // v_mul_f64
      if constexpr (kOp == 3) d[c] = d[c] + 1e-3;                                                // v_add_f64
      if constexpr (kOp == 4) d[c] = __builtin_amdgcn_rcp(d[c]);                                 // v_rcp_f64
      if constexpr (kOp == 5) d[c] = __builtin_amdgcn_sqrt(d[c]) + 1.0;                          // v_sqrt_f64 (+add)
      if constexpr (kOp == 6) f[c] = __builtin_amdgcn_sinf(f[c]);                                // v_sin_f32
      if constexpr (kOp == 7) f[c] = __builtin_amdgcn_rcpf(f[c]);                                // v_rcp_f32
      if constexpr (kOp == 8) q[c] = (unsigned long long)0xD2511F53u * (unsigned)q[c] + (q[c] >> 32);  // v_mad_u64_u32
      if constexpr (kOp == 9) u[c] = (u[c] ^ 0x9E3779B9u) + 0x7F4A7C15u;                          // 2 int32
      if constexpr (kOp == 10) d[c] = __builtin_amdgcn_rsq(d[c]) + 0.5;                          // v_rsq_f64 (+add)
      if constexpr (kOp == 11) d[c] = (double)(int)d[c] + 0.25;                                  // cvt i32<->f64 (+add)
      if constexpr (kOp == 12) d[c] = __builtin_fmin(d[c], 0.5) + 1e-3;                          // v_min_f64 (+add)
    }
  }
  double s = 0;
  float sf = 0;
  unsigned long long si = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    s += d[c];
    sf += f[c];
    si += q[c] + u[c];
  }
  out[t] = s;
  outf[t] = sf;
  outi[t] = si;
}

template <int kOp>
double run(int blocks, double* d, float* f, unsigned long long* q) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(bench<kOp>, dim3(blocks), dim3(256), 0, 0, d, f, q, 0.5);  // warm
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(bench<kOp>, dim3(blocks), dim3(256), 0, 0, d, f, q, 0.5);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = (double)blocks * 4;
  return waves * ITERS * CHAINS * 5 / (ms * 1e-3) / 1e9;  // G wave-"ops"/s
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;  // 32 waves per CU: every SIMD full
  double* d;
  float* f;
  unsigned long long* q;
  hipMalloc(&d, sizeof(double) * blocks * 256);
  hipMalloc(&f, sizeof(float) * blocks * 256);
  hipMalloc(&q, sizeof(unsigned long long) * blocks * 256);
  printf("{\"cus\": %d", cus);
  printf(", \"fma_f32\": %.1f", run<0>(blocks, d, f, q));
  printf(", \"fma_f64\": %.1f", run<1>(blocks, d, f, q));
  printf(", \"mul_f64\": %.1f", run<2>(blocks, d, f, q));
  printf(", \"add_f64\": %.1f", run<3>(blocks, d, f, q));
  printf(", \"rcp_f64\": %.1f", run<4>(blocks, d, f, q));
  printf(", \"sqrt_f64_plus_add\": %.1f", run<5>(blocks, d, f, q));
  printf(", \"sin_f32\": %.1f", run<6>(blocks, d, f, q));
  printf(", \"rcp_f32\": %.1f", run<7>(blocks, d, f, q));
  printf(", \"mad_u64_u32_plus\": %.1f", run<8>(blocks, d, f, q));
  printf(", \"int32_pair\": %.1f", run<9>(blocks, d, f, q));
  printf(", \"rsq_f64_plus_add\": %.1f", run<10>(blocks, d, f, q));
  printf(", \"cvt_f64_pair\": %.1f", run<11>(blocks, d, f, q));
  printf(", \"min_f64_plus_add\": %.1f", run<12>(blocks, d, f, q));
  printf(", \"unit\": \"G wave64 loop-ops/s (one op per chain step; see source for the instructions per op)\"}\n");
  return 0;
}
