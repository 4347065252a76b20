// f64_math_check.hip — accuracy of the render kernel's binary64 device math (rt_trace.h
// rt_math64: v_rcp_f64 / v_rsq_f64 with a third-order correction, sin / cos of 2 pi u) against the IEEE /
// OCML results on the device.  Prints one JSON object: per function the largest difference in
// units in the last place and the fraction of inputs that differ at all.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#define RT_F64 1
#include "../../raytrace_amd/csrc/rt_trace.h"

__global__ void check(const double* x, const double* u, double* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double s, c;
  rt_math64::sincos_turns(u[i], &s, &c);
  out[10 * i + 0] = rt_math64::rcp(x[i]);
  out[10 * i + 1] = 1.0 / x[i];
  out[10 * i + 2] = rt_math64::rsqrt(x[i]);
  out[10 * i + 3] = 1.0 / sqrt(x[i]);
  out[10 * i + 4] = rt_math64::sqrt_nonneg(x[i]);
  out[10 * i + 5] = sqrt(x[i]);
  out[10 * i + 6] = s;
  out[10 * i + 7] = sin(6.283185307179586 * u[i]);
  out[10 * i + 8] = c;
  out[10 * i + 9] = cos(6.283185307179586 * u[i]);
}

static double ulps(double a, double b) {
  if (a == b) return 0;
  if (!std::isfinite(a) || !std::isfinite(b)) return 1e300;
  const double m = std::max(std::fabs(a), std::fabs(b));
  return std::fabs(a - b) / (std::nextafter(m, INFINITY) - m);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), u(n), out(10 * (size_t)n);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
  };
  for (int i = 0; i < n; ++i) {
    // magnitudes 1e-12 .. 1e12 (directions, t values, radii, pdfs), plus exact squares
    x[i] = std::ldexp(1.0 + (double)(rnd() >> 11) / 9007199254740992.0, (int)(rnd() % 80) - 40);
    if (i % 97 == 0) x[i] = (double)(i % 1000 + 1) * (double)(i % 1000 + 1);
    u[i] = (double)((uint32_t)rnd() >> 8) * (1.0 / 16777216.0);  // the 24-bit uniforms
  }
  x[0] = 0.0;
  double *dx, *du, *dout;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&du, n * 8);
  (void)hipMalloc(&dout, 10 * (size_t)n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(du, u.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(n / 256), dim3(256), 0, 0, dx, du, dout, n);
  (void)hipMemcpy(out.data(), dout, 10 * (size_t)n * 8, hipMemcpyDeviceToHost);
  const char* names[5] = {"rcp", "rsqrt", "sqrt", "sin_turns", "cos_turns"};
  printf("{\"n\": %d", n);
  for (int f = 0; f < 5; ++f) {
    double worst = 0;
    long diff = 0;
    for (int i = (f == 1 ? 1 : 0); i < n; ++i) {  // rsqrt: x > 0 only
      const double a = out[10 * (size_t)i + 2 * f], b = out[10 * (size_t)i + 2 * f + 1];
      double e = ulps(a, b);
      if (f >= 3) e = std::fabs(a - b) / 2.220446049250313e-16;  // absolute, in units of 2^-52
      worst = std::max(worst, e);
      diff += a != b;
    }
    printf(", \"%s\": {\"max_ulp\": %.3g, \"frac_differ\": %.4g}", names[f], worst, (double)diff / n);
  }
  printf(", \"note\": \"rcp / rsqrt / sqrt vs IEEE division and OCML sqrt; sin/cos of 2 pi u vs OCML sin/cos of "
         "fl(2 pi) u, absolute error in units of 2^-52\"}\n");
  return 0;
}
