// rt_trace.h — the per-lane path-tracing logic of the MI355X megakernel (rt_kernel.hip).
//
// Work decomposition: the frame (this shard's rows) x spp is cut into ITEMS = (tile pixel,
// chunk of consecutive samples), numbered pixel-major.  Lanes are persistent: a lane whose item
// is exhausted claims the next item from its wave's pool, refilled from one of four queue head
// words (one wave-aggregated atomic per 128 items; rt_render_kernel.h WaveWork, which also sums a
// pool's items per pixel in LDS before they reach HBM), so every lane stays busy until the queue
// drains and the tail is one chunk long.  Inside an item a lane
// regenerates paths: when a path terminates the next sample starts at once.  Per segment:
//   1. closest hit: flat sets (class loops and box groups over wave-uniform records), or the
//      surface set's large-primitive prefix then its BVH (stack in LDS, near child first,
//      leaves tested once a per-scene share of the lanes hold one), with the reference's
//      depth-first tie-break in a 64-bit key; and, for every constantMedium, its boundary
//      (Geometry.hs:298-330);
//   2. the material of the hit: a `switch` over the ten reference materials
//      (Material.hs:41-129) and the texture (Texture.hs:18-53);
//   3. HemisphereF / SphereF: direction from the redirect mixture, weight pdf1 / pdf
//      (Ray.hs:187-224).
// rayColor's recursion (Ray.hs:174-224) is carried as throughput T and radiance L
// (L = e0 + a0 (e1 + a1 (...)) = sum_k T_k e_k).  Each sample's L is added to the pixel's sum
// in 64-bit fixed point (2^-32): integer addition commutes, so the mean (Ray.hs:232) is bit-for-
// bit independent of chunking, scheduling and the multi-GPU row partition.
//
// Precision: the header is instantiated twice, for `real` = double (RT_F64 = 1, namespace
// rtk64: the reference's binary64 arithmetic, Core.hs:29-31; the default of the C ABI) and for
// `real` = float (RT_F64 = 0, namespace rtk: the opt-in FP32 fast path).  The includer defines
// RT_F64; a translation unit may include the header once per precision.  Philox4x32-10 keyed
// by the seed with counter (pixel, sample, segment, event) and 24-bit uniforms; direct
// samplers in place of the reference's rejection loops (same distributions).  The FP64
// oracle's Philox mode (oracle/rt_oracle.c) consumes the same numbers, which is what the
// per-pixel parity tests check.
//
// The header is compiled by hipcc for gfx950 (rt_kernel.hip, rt_kernel64.hip).  tests/kernel_emu compiles the
// same text for the host (RT_HOST_EMU) so the kernel's logic can be checked against the oracle
// without a GPU; that build is test tooling and is never linked into the product library.
#ifndef RT_TRACE_COMMON_H
#define RT_TRACE_COMMON_H
#include <stdint.h>

#include "../../include/rt.h"
#include "rt_internal.h"
#include "rt_sincos_table.h"

#ifdef RT_HOST_EMU
#include <cmath>
#include <cstring>
#define RT_FN static inline
#define RT_FN_SPEC inline  // explicit specialisations take no storage class
namespace rt_emu {
inline int f2i(float f) {
  int i;
  std::memcpy(&i, &f, 4);
  return i;
}
// traversal counters of the host build (nodes visited, primitives tested, segments)
extern thread_local long long counters[4];
}  // namespace rt_emu
#define RT_F2I(f) rt_emu::f2i(f)
#define RT_COUNT(i) (++rt_emu::counters[i])
#define RT_ANY(x) (x)  // the emulator runs one lane per wave
#define RT_BALLOT_COUNT(x) ((x) ? 1 : 0)
#define RT_CAS
#else
#define RT_FN __device__ __forceinline__
#define RT_FN_SPEC __device__ __forceinline__
#define RT_F2I(f) __float_as_int(f)
#define RT_COUNT(i) ((void)0)
#define RT_ANY(x) __any(x)
#define RT_BALLOT_COUNT(x) ((int)__popcll(__ballot(x)))
// Scene data is read through the constant address space: the kernel never writes it, so
// wave-uniform reads (flat sets, kernel-argument indices) become scalar loads into SGPRs and
// divergent reads stay vector loads.
#define RT_CAS __attribute__((address_space(4)))
#endif

// Debug hooks (no-ops; the emulator's debug build defines them to trace one path on the CPU)
#ifndef RT_HOOK_SEGMENT
#define RT_HOOK_SEGMENT(pix, sample, seg, R, tbest, best, hit_medium, L, T)
#endif
#ifndef RT_HOOK_SAMPLE
#define RT_HOOK_SAMPLE(pix, sample, L)
#endif
#endif  // RT_TRACE_COMMON_H

// ------------------------------------------------------------------ per-precision macros
#ifndef RT_F64
#define RT_F64 0
#endif
#undef RT_NS
#undef RL
#undef RMIN
#undef RMAX
#undef RABS
#undef RFLOOR
#undef RCOPYSIGN
#undef RATAN2
#undef RACOS
#undef RSIN
#undef RFMA
#undef RT_NAN
#undef RT_HUGE
#undef RT_R2I
#undef RT_SINCOS_TURNS
#undef RT_LOG
#undef RT_RSQRT
#undef RT_RCP
#undef RT_RCP_NZ
#undef RT_SQRT
#undef RT_NODE_F32
#if RT_F64
// binary64: IEEE division and square root, libm / OCML transcendentals (the oracle's libm calls)
#define RT_NS rtk64
#define RL(x) x
#define RMIN fmin
#define RMAX fmax
#define RABS fabs
#define RFLOOR floor
#define RCOPYSIGN copysign
#define RATAN2 atan2
#define RACOS acos
#define RSIN sin
#define RFMA fma
#define RT_NAN __builtin_nan("")
#define RT_HUGE __builtin_huge_val()
// an int stored in a binary64 record: the low word of its bit pattern (rt_build.cpp ibits)
#define RT_R2I(x) ((int)(uint32_t)__builtin_bit_cast(unsigned long long, (double)(x)))
#define RT_LOG(x) log(x)
#if defined(RT_HOST_EMU) || defined(RT_MATH64_IEEE)  // RT_MATH64_IEEE: A/B builds with the IEEE sequences
#define RT_SINCOS_TURNS(x, s, c) (*(s) = sin(6.283185307179586 * (x)), *(c) = cos(6.283185307179586 * (x)))
#define RT_RSQRT(x) (1.0 / sqrt(x))
#define RT_RCP(x) (1.0 / (x))
#define RT_RCP_NZ(x) (1.0 / (x))
#define RT_SQRT(x) sqrt(x)
#else
// Device binary64 math (rt_math64 below): the hardware reciprocal / reciprocal square root
// refined by one third-order correction step instead of the IEEE division and square-root sequences, and sin / cos
// of 2 pi u by an exact quadrant reduction and polynomials — each within ~1 ulp of the correctly
// rounded result (tools/microbench/f64_math_check.hip measures it), 2-5x fewer instructions.
#define RT_SINCOS_TURNS(x, s, c) rt_math64::sincos_turns(x, s, c)
#define RT_RSQRT(x) rt_math64::rsqrt(x)
#define RT_RCP(x) rt_math64::rcp(x)
#define RT_RCP_NZ(x) rt_math64::rcp_nz(x)
#define RT_SQRT(x) rt_math64::sqrt_nonneg(x)
#ifndef RT_MATH64_DEFINED
#define RT_MATH64_DEFINED
namespace rt_math64 {
// 1 / x: v_rcp_f64 and one third-order correction: 1/x = r0 / (1 - e) = r0 (1 + e + e^2 + ...)
// with e = 1 - x r0 ~ 2^-24, so e^3 is below the last place (bit-identical to IEEE division on
// tools/microbench/f64_math_check's 4 M inputs, one FMA fewer than two Newton steps); x = +-0 /
// +-inf keep the hardware's +-inf / +-0
__device__ __forceinline__ double rcp(double x) {
  const double r0 = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, r0, 1.0);
  const double r = __builtin_fma(r0, __builtin_fma(e, e, e), r0);
  return r == r ? r : r0;
}
// 1 / x where a +-0 / +-inf x need not give +-inf / +-0 (they give NaN): callers whose result is
// discarded for such x (a plane test's |n . d| <= 1e-8 margin, a redirect target's checked
// denominator) skip rcp's NaN guard
__device__ __forceinline__ double rcp_nz(double x) {
  const double r0 = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, r0, 1.0);
  return __builtin_fma(r0, __builtin_fma(e, e, e), r0);
}
// 1 / sqrt(x), x > 0: v_rsq_f64 and one third-order correction, 1/sqrt(x) = y (1 - e)^(-1/2) =
// y (1 + e/2 + 3 e^2 / 8 + ...) with e = 1 - x y^2 (within 2 ulp, as two Newton steps were)
__device__ __forceinline__ double rsqrt(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = __builtin_fma(-x * y, y, 1.0);
  return __builtin_fma(y, __builtin_fma(e, 0.375, 0.5) * e, y);
}
// sqrt(x), x >= 0: Goldschmidt iteration from v_rsq_f64 and a final residual correction
__device__ __forceinline__ double sqrt_nonneg(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-s, h, 0.5);
  s = __builtin_fma(s, r, s);
  h = __builtin_fma(h, r, h);
  const double d = __builtin_fma(-s, s, x);
  s = __builtin_fma(d, h, s);
  return x == 0.0 || x == __builtin_huge_val() ? x : s;
}
// sin / cos of 2 pi u for u in [0, 1) (the samplers' angles; u has 24 random bits): u = k / 128 +
// b with k = rint(128 u) and |b| <= 1/256 exact, (sin, cos)(2 pi k / 128) from a correctly rounded
// table (rt_sincos_table.h, 2 KB, L1-resident), sin / cos (2 pi b) by short Taylor polynomials
// (|2 pi b| <= 0.0246: truncation < 1e-17), combined by the angle-addition formulas
__device__ const double rt_sincos_tab[2 * RT_SINCOS_TABLE_N] = RT_SINCOS_TABLE_INIT;
// (a table-free version — quadrant reduction and fdlibm's minimax kernels, 3.25 ulp — ran Cornell
// 4.89 -> 5.42 ms: the table's two loads cost less than the longer polynomials; profiles/r5/variants)
__device__ __forceinline__ void sincos_turns(double u, double* sn, double* cs) {
  const double kq = __builtin_rint(u * (double)RT_SINCOS_TABLE_N);
  const double b = __builtin_fma(kq, -1.0 / RT_SINCOS_TABLE_N, u);
  const int k = (int)kq & (RT_SINCOS_TABLE_N - 1);
  const double sa = rt_sincos_tab[2 * k], ca = rt_sincos_tab[2 * k + 1];
  const double x = b * 6.283185307179586, x2 = x * x;
  double ps = __builtin_fma(x2, -1.0 / 5040.0, 1.0 / 120.0);
  ps = __builtin_fma(x2, ps, -1.0 / 6.0);
  const double sb = __builtin_fma(x2 * x, ps, x);
  double pc = __builtin_fma(x2, -1.0 / 720.0, 1.0 / 24.0);
  pc = __builtin_fma(x2, pc, -0.5);
  const double cb = __builtin_fma(x2, pc, 1.0);
  *sn = __builtin_fma(sa, cb, ca * sb);
  *cs = __builtin_fma(ca, cb, -(sa * sb));
}
}  // namespace rt_math64
#endif
#endif
#else
#define RT_NS rtk
#define RL(x) x##f
#define RMIN fminf
#define RMAX fmaxf
#define RABS fabsf
#define RFLOOR floorf
#define RCOPYSIGN copysignf
#define RATAN2 atan2f
#define RACOS acosf
#define RSIN sinf
#define RFMA fmaf
#define RT_NAN __builtin_nanf("")
#define RT_HUGE __builtin_huge_valf()
#define RT_R2I(x) RT_F2I(x)
#ifdef RT_HOST_EMU
#define RT_SINCOS_TURNS(x, s, c) (*(s) = sinf(6.283185307179586f * (x)), *(c) = cosf(6.283185307179586f * (x)))
#define RT_LOG(x) logf(x)
#define RT_RSQRT(x) (1.0f / sqrtf(x))
#define RT_RCP(x) (1.0f / (x))
#define RT_RCP_NZ(x) (1.0f / (x))
#define RT_SQRT(x) sqrtf(x)
#else
// sin / cos of 2 pi x for x in [0, 1): v_sin_f32 / v_cos_f32 take their argument in turns
#define RT_SINCOS_TURNS(x, s, c) (*(s) = __builtin_amdgcn_sinf(x), *(c) = __builtin_amdgcn_cosf(x))
#define RT_LOG(x) __logf(x)
#define RT_RSQRT(x) __frsqrt_rn(x)
#define RT_RCP(x) __builtin_amdgcn_rcpf(x)
#define RT_RCP_NZ(x) __builtin_amdgcn_rcpf(x)
#define RT_SQRT(x) __builtin_amdgcn_sqrtf(x)  // v_sqrt_f32 (1 ulp), no IEEE fix-up sequence
#endif
#endif

namespace RT_NS {

#if RT_F64
using real = double;
using ureal = unsigned long long;  // the bit pattern of a real
#else
using real = float;
using ureal = uint32_t;
#endif
using KernelParams = ::KernelParamsT<real>;
using DevMaterial = ::DevMaterialT<real>;
using DevTexture = ::DevTextureT<real>;
using DevMedium = ::DevMediumT<real>;
using DevBox = ::DevBoxT<real>;
using DevTarget = ::DevTargetT<real>;
using DevCamera = ::DevCameraT<real>;
using DevInstance = ::DevInstanceT<real>;



constexpr real kPi = RL(3.14159265358979323846);
constexpr real kTmin = RL(0.0001);  // Ray.hs:178
constexpr real kInf = RT_HUGE;

#ifdef RT_HOST_EMU
struct alignas(16) v4 {  // the host emulator's std::vector buffers guarantee 16 B
#else
struct alignas(4 * sizeof(real)) v4 {
#endif
  real x, y, z, w;
};
struct alignas(16) v4f {  // BVH node data (float in both precisions)
  float x, y, z, w;
};
struct alignas(16) i4 {
  int x, y, z, w;
};
struct f3 {
  real x, y, z;
};
RT_FN f3 mk3(real x, real y, real z) { return f3{x, y, z}; }
RT_FN f3 ld3(const real* p) { return f3{p[0], p[1], p[2]}; }
RT_FN f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_FN f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_FN f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
RT_FN f3 operator*(real s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
RT_FN f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_FN real dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_FN f3 normalize(f3 v) {
  real l = dot(v, v);
#if RT_F64
  // linear's normalize: v unchanged when its quadrance is nearZero or nearZero (1 - quadrance)
  if (RABS(l) <= RL(1e-12) || RABS(RL(1.0) - l) <= RL(1e-12)) return v;
#else
  if (l <= RL(1e-12)) return v;  // linear's normalize leaves (near-)zero vectors alone
#endif
  return RT_RSQRT(l) * v;
}
// Re-normalise a direction that is unit in exact arithmetic (reflect / refract of unit vectors,
// Core.hs:49-51, Material.hs:81-85).  The reference's sphere test assumes |d| = 1 (Geometry.hs:
// 64-68); in binary64 the rounding drift is ~1e-16 and harmless, but in FP32 a chain of total
// internal reflections inside a glass sphere amplifies it each bounce (the point lands off the
// surface, the normal (p - c) / r is no longer unit, reflect lengthens d) until the path
// diverges.  Re-normalising keeps the FP32 path on the exact-arithmetic result.
RT_FN f3 unit(f3 v) { return RT_RSQRT(dot(v, v)) * v; }
RT_FN f3 reflect(f3 n, f3 v) { return v - (RL(2.0) * dot(n, v)) * n; }  // Core.hs:49-51
RT_FN f3 xyz(v4 v) { return f3{v.x, v.y, v.z}; }
RT_FN v4 ld4(const real* p) { return *reinterpret_cast<const v4*>(p); }
typedef const RT_CAS real* cfp;  // pointer to read-only scene data
RT_FN cfp cf(const real* p) { return (cfp)p; }
RT_FN f3 ldc3(cfp p) { return f3{p[0], p[1], p[2]}; }
RT_FN v4 ldc4(cfp p) {
  const RT_CAS v4* q = (const RT_CAS v4*)p;
  return v4{q->x, q->y, q->z, q->w};
}
RT_FN int ldci(const int* p, int i) { return ((const RT_CAS int*)p)[i]; }
typedef const RT_CAS float* cfpf;  // BVH nodes
RT_FN v4f ldc4f(cfpf p) {
  const RT_CAS v4f* q = (const RT_CAS v4f*)p;
  return v4f{q->x, q->y, q->z, q->w};
}

// ------------------------------------------------------------------ Philox4x32-10
struct u4 {
  uint32_t x, y, z, w;
};
// a ^ b ^ c in one VALU instruction: gfx950's three-input bit operation (truth table 0x96)
#ifdef RT_HOST_EMU
#define RT_XOR3(a, b, c) ((a) ^ (b) ^ (c))
#else
#define RT_XOR3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#endif
RT_FN u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#ifndef RT_PHILOX_ROUNDS
#define RT_PHILOX_ROUNDS 10
#endif
#ifndef RT_HOST_EMU
  // the round keys are two scalar adds per round: recompute them at every call instead of
  // letting the compiler keep all twenty live (and spilled) across the lane loop
  asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int r = 0; r < RT_PHILOX_ROUNDS; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // one full 32x32->64 product per word: a single v_mad_u64_u32 instead of mul_hi + mul_lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = RT_XOR3(hi1, c1, k0), n2 = RT_XOR3(hi0, c3, k1);
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return u4{c0, c1, c2, c3};
}
// [0, 1) with 24 random bits: exact in both FP32 and the oracle's FP64
RT_FN real u01(uint32_t w) { return (real)(w >> 8) * (RL(1.0) / RL(16777216.0)); }
// (assembling m 2^-24 and a + m 2^-24 from binary64 bit patterns instead of the conversions spilled
// the binary64 Cornell kernel and ran 0.5-2 % slower: profiles/r6/flat)

// uniform direction on the unit sphere (the distribution of randomUnitVector, Core.hs:54-60)
RT_FN f3 unit_vector(uint32_t a, uint32_t b) {
  real z = RL(1.0) - RL(2.0) * u01(a);
  real r = RT_SQRT(RMAX(RL(0.0), RL(1.0) - z * z));
  real s, c;
  RT_SINCOS_TURNS(u01(b), &s, &c);
  return mk3(r * c, r * s, z);
}

// Binary64 kernels test BVH nodes in FP32 (the node boxes are floats; RT_NODE_F64 restores the
// binary64 slab test): the ray carries 1 / d and two offsets, o / d plus and minus a rounding pad,
// so the FP32 slab interval contains the exact one (prep_ray, trav_round).
#if RT_F64 && !defined(RT_NODE_F64)
#define RT_NODE_F32 1
struct f3n {
  float x, y, z;
};
#else
#define RT_NODE_F32 0
#endif
struct RayCtx {
  f3 o, d;
#if RT_NODE_F32
  f3n idir, off0, off1;  // 1 / d; o / d for the box-min planes (off0) and the box-max planes (off1)
#else
  f3 idir, oidir;
#endif
  uint32_t time_w;  // the ray's time as its Philox word: time = u01(time_w), exact (one VGPR in binary64)
  int self_gid;   // the leaf the ray leaves (skipped: FP32 robustness, rt_trace.h isect_*)
  int self_inst;  // ... and its instance (-1: a world leaf; two-level instancing, RT_VAR_INST)
};
// The leaf the ray leaves: gid equal, and (instancing) the same placement of the object.
template <bool kInst>
RT_FN bool is_self(const RayCtx& R, int gid, int cur_inst) {
  if constexpr (kInst) return gid == R.self_gid && cur_inst == R.self_inst;
  return gid == R.self_gid;
}

RT_FN real u01(uint32_t w);
RT_FN f3 motion_shift(const KernelParams& P, int m, uint32_t time_w) {
  const real time = u01(time_w);
  f3 v0 = ldc3(cf(P.motions) + 8 * m), v1 = ldc3(cf(P.motions) + 8 * m + 4);
  return (RL(1.0) - time) * v0 + time * v1;
}

RT_FN real safe_rcp(real d) { return RT_RCP(RABS(d) > RL(1e-20) ? d : RCOPYSIGN(RL(1e-20), d)); }

// reciprocal direction and origin x reciprocal for the BVH slab tests
#if RT_NODE_F32
// One axis of the FP32 node ray.  t = b (1/d) - o/d in FP32 is off the exact (b - o) / d by at
// most ~3 eps |o/d| (rounding of 1/d and o/d to float, the offset's own rounding) plus ~2 eps |t|
// (the fma, and 1/d's rounding times b/d): pad = 5 eps |o/d| moves the entry plane down and the
// exit plane up (which plane enters follows the sign of 1/d), and trav_round widens the far end
// by (1 + 2^-20) for the relative part.
#ifndef RT_RCPF
#ifdef RT_HOST_EMU
#define RT_RCPF(x) (1.0f / (x))
#else
#define RT_RCPF(x) __builtin_amdgcn_rcpf(x)
#endif
#endif
RT_FN void prep_axis(real o, real d, float& fi, float& f0, float& f1) {
#ifndef RT_NODE_RCP64
  // FP32 reciprocal of the (clamped) direction: t = (b - o) fi is then t (1 + delta), |delta| <=
  // ~3 eps (rounding of d, v_rcp_f32), inside the far end's (1 + 2^-20) margin; o fi in binary64
  // keeps the offset consistent with fi
  const float i = RT_RCPF((float)(RABS(d) > RL(1e-20) ? d : RCOPYSIGN(RL(1e-20), d)));
  const float oi = (float)(o * (real)i);
#else
  const real i = safe_rcp(d);
  const float oi = (float)(o * i);
#endif
  const float pad = 3.0e-7f * fabsf(oi);
  const float sp = i >= 0 ? pad : -pad;
  fi = (float)i;
  f0 = oi + sp;  // box-min plane: the entry when 1/d >= 0 (its t lowered)
  f1 = oi - sp;  // box-max plane
}
RT_FN void prep_ray(RayCtx& R) {
  prep_axis(R.o.x, R.d.x, R.idir.x, R.off0.x, R.off1.x);
  prep_axis(R.o.y, R.d.y, R.idir.y, R.off0.y, R.off1.y);
  prep_axis(R.o.z, R.d.z, R.idir.z, R.off0.z, R.off1.z);
}
// The two children's slab intervals of one BVH node (n0 = left x / y bounds, n1 = right x / y,
// n2 = left z, right z; min before max) against (tmin, t_closest); a child is entered when its
// near <= far.  tests/test_node_test.py checks on the host emulator that this accepts every box
// the exact slab test accepts.
RT_FN void node_slabs_f32(const RayCtx& R, const v4f& n0, const v4f& n1, const v4f& n2, float tminf, float ctf,
                          float& lnear, float& lfar, float& rnear, float& rfar) {
  const float lx0 = fmaf(n0.x, R.idir.x, -R.off0.x), lx1 = fmaf(n0.y, R.idir.x, -R.off1.x);
  const float ly0 = fmaf(n0.z, R.idir.y, -R.off0.y), ly1 = fmaf(n0.w, R.idir.y, -R.off1.y);
  const float lz0 = fmaf(n2.x, R.idir.z, -R.off0.z), lz1 = fmaf(n2.y, R.idir.z, -R.off1.z);
  const float rx0 = fmaf(n1.x, R.idir.x, -R.off0.x), rx1 = fmaf(n1.y, R.idir.x, -R.off1.x);
  const float ry0 = fmaf(n1.z, R.idir.y, -R.off0.y), ry1 = fmaf(n1.w, R.idir.y, -R.off1.y);
  const float rz0 = fmaf(n2.z, R.idir.z, -R.off0.z), rz1 = fmaf(n2.w, R.idir.z, -R.off1.z);
  lnear = fmaxf(fmaxf(fminf(lx0, lx1), fminf(ly0, ly1)), fmaxf(fminf(lz0, lz1), tminf));
  lfar = fminf(fminf(fmaxf(lx0, lx1), fmaxf(ly0, ly1)), fminf(fmaxf(lz0, lz1), ctf)) * 1.00000095f;
  rnear = fmaxf(fmaxf(fminf(rx0, rx1), fminf(ry0, ry1)), fmaxf(fminf(rz0, rz1), tminf));
  rfar = fminf(fminf(fmaxf(rx0, rx1), fmaxf(ry0, ry1)), fminf(fmaxf(rz0, rz1), ctf)) * 1.00000095f;
}
#else
RT_FN void prep_ray(RayCtx& R) {
  R.idir = mk3(safe_rcp(R.d.x), safe_rcp(R.d.y), safe_rcp(R.d.z));
  R.oidir = R.o * R.idir;
}
#endif

// Two-level instancing (rt_internal.h DevInstance): world -> object space through the inverse of
// the rigid placement (R^T (p - t); t is unchanged along the ray) and object -> world normals.
RT_FN const RT_CAS DevInstance* inst_rec(const KernelParams& P, int k) { return (const RT_CAS DevInstance*)P.instances + k; }
RT_FN f3 inst_to_object(const RT_CAS DevInstance* I, f3 v, bool point) {
  if (point) v = v - mk3(I->m[3], I->m[7], I->m[11]);
  return mk3(I->m[0] * v.x + I->m[4] * v.y + I->m[8] * v.z, I->m[1] * v.x + I->m[5] * v.y + I->m[9] * v.z,
             I->m[2] * v.x + I->m[6] * v.y + I->m[10] * v.z);
}
RT_FN f3 inst_rotate(const RT_CAS DevInstance* I, f3 v) {
  return mk3(I->m[0] * v.x + I->m[1] * v.y + I->m[2] * v.z, I->m[4] * v.x + I->m[5] * v.y + I->m[6] * v.z,
             I->m[8] * v.x + I->m[9] * v.y + I->m[10] * v.z);
}

// Closest hit so far, keyed by (t, depth-first order): smaller t wins, ties go to the earlier
// leaf (Geometry.hs:340-361).  Float kernels pack the key into 64 bits, (bits of t) << 32 |
// order: for t > 0 its integer order is that rule, so one 64-bit compare replaces the t / tie /
// validity mask logic; invalid candidates carry t = NaN (bits above +inf), the initial key is
// (+inf, 0).  Binary64 kernels compare (t, order) as a pair.
#if RT_F64
struct Closest {
  real t;
  int ord;
  int prim;
  int inst;  // the instance of the winning leaf (-1: world)
};
#else
struct Closest {
  real t;
  unsigned long long key;
  int prim;
  int inst;  // the instance of the winning leaf (-1: world)
};
#endif
// Per-lane traversal resources: the lane's stack (stack[k * stride]) and the workgroup's LDS copy
// of the first P.lds_nodes BVH nodes (breadth-first numbering puts the top levels there).
struct Trav {
  int* stack;
  int stride;
  const v4f* lds_nodes;
};
#if RT_F64
RT_FN Closest no_hit() { return Closest{kInf, 0, -1, -1}; }
#else
RT_FN Closest no_hit() { return Closest{kInf, 0x7f80000000000000ull, -1, -1}; }
RT_FN unsigned long long hit_key(real t, int ord) {
  return ((unsigned long long)(unsigned)RT_F2I(t) << 32) | (unsigned)ord;
}
#endif

// A primitive record (rt_internal.h layout, 64 B): a = (center | normal, kind+flags),
// b = (radius, r^2, uvframe, gid | q, gid), c = (-, -, -, order | wa, order), e = (wb, motion).
struct PrimRec {
  v4 a, b, c, e;
};
RT_FN PrimRec ld_rec(cfp pr) { return PrimRec{ldc4(pr), ldc4(pr + 4), ldc4(pr + 8), ldc4(pr + 12)}; }
// one record: 64 B (float) / 128 B (binary64), record-aligned in device memory (hipMalloc bases
// are 256-B aligned) so a wave-uniform record is one wide scalar load; the host emulator's
// std::vector buffers only guarantee 16 B
#ifdef RT_HOST_EMU
#define RT_REC_ALIGN 16
#else
#define RT_REC_ALIGN (16 * sizeof(real))
#endif
struct alignas(RT_REC_ALIGN) PrimRec64 {
  real f[16];
};
RT_FN PrimRec ld_rec64(const RT_CAS PrimRec64* p) {
  const RT_CAS real* r = p->f;
  return PrimRec{v4{r[0], r[1], r[2], r[3]}, v4{r[4], r[5], r[6], r[7]}, v4{r[8], r[9], r[10], r[11]},
                 v4{r[12], r[13], r[14], r[15]}};
}

// Primitive intersection (Geometry.hs:58-144), branch-free: each test yields a parameter t and
// one validity margin q (valid iff q >= 0) that also carries the interval test t > tmin as
// t - up(tmin) >= 0 (up = next real: exact for the open interval), so the closest-hit update is
// a single compare and select with no per-test lane-mask bookkeeping on the scalar unit.
#if RT_F64
RT_FN real float_up(real x) { return __builtin_bit_cast(real, __builtin_bit_cast(long long, x) + 1); }  // x > 0
#else
RT_FN real float_up(real x) { return __builtin_bit_cast(real, RT_F2I(x) + 1); }  // x > 0
#endif
// sphere (Geometry.hs:58-94); geometric discriminant for FP32 robustness.  A ray leaving this
// sphere (self) can only reach the far root 2h (the near one is t = 0).
RT_FN void isect_sphere(const PrimRec& r, f3 o, const RayCtx& R, real tmin, real tmin_up, bool self, real& t,
                        real& q) {
  f3 oc = xyz(r.a) - o;
  real h = dot(R.d, oc);
  f3 l = oc - h * R.d;
  real disc = r.b.y - dot(l, l);
  real sq = RT_SQRT(RMAX(disc, RL(0.0)));
  real r1 = h - sq, r2 = h + sq;
  real tn = r1 > tmin ? r1 : r2;
  t = self ? RL(2.0) * h : tn;
  q = RMIN(self ? RL(1.0) : disc, t - tmin_up);
}
// planeShape (Geometry.hs:117-144): parallelogram a, b in [0,1]; triangle a, b >= 0, a + b <= 1.
// kQuad: 1 parallelogram, 0 triangle, -1 either (per-lane `quad`, a select instead of a branch)
template <int kQuad>
RT_FN void isect_plane(const PrimRec& r, f3 o, const RayCtx& R, real tmin_up, bool self, real& t, real& q,
                       bool quad = false) {
  f3 n = xyz(r.a);
  real denom = dot(n, R.d);
  f3 qo = xyz(r.b) - o;
  t = dot(n, qo) * RT_RCP_NZ(denom);  // |denom| <= 1e-8 (NaN t included) fails the margin m2
  f3 prel = t * R.d - qo;
  real aa = dot(prel, xyz(r.c)), bb = dot(prel, xyz(r.e));
  real m1, m2 = RMIN(RABS(denom) - RL(1e-8), t - tmin_up);
  if constexpr (kQuad < 0) {  // quad: min(1 - a, 1 - b); triangle: 1 - a - b
    m1 = RMIN(RMIN(aa, bb), quad ? RMIN(RL(1.0) - aa, RL(1.0) - bb) : RL(1.0) - aa - bb);
  } else if constexpr (kQuad == 1) {
    m1 = RMIN(RMIN(aa, bb), RL(1.0) - aa);
    m2 = RMIN(m2, RL(1.0) - bb);
  } else {
    m1 = RMIN(RMIN(aa, bb), RL(1.0) - aa - bb);
  }
  q = self ? -RL(1.0) : RMIN(m1, m2);
}
// kKeyOnly (flat sets): only the key is tracked; t and the primitive follow from it afterwards
template <bool kKeyOnly, bool kInst = false>
RT_FN void consider(Closest& C, real t, real q, int ord, int pi, int inst = -1) {
#if RT_F64
  // flat sets: bitwise, not short-circuit — three compares and mask ANDs instead of nested exec
  // branches (Cornell -1.4 %); BVH leaves keep the branches (their kernels' SGPR spills grew)
  const bool take = kKeyOnly ? (q >= RL(0.0)) & ((t < C.t) | ((t == C.t) & (ord < C.ord)))
                             : q >= RL(0.0) && (t < C.t || (t == C.t && ord < C.ord));
  C.t = take ? t : C.t;
  C.ord = take ? ord : C.ord;
  if constexpr (!kKeyOnly) C.prim = take ? pi : C.prim;
  if constexpr (kInst) C.inst = take ? inst : C.inst;
#else
  const real tc = q >= RL(0.0) ? t : RT_NAN;
  const unsigned long long key = hit_key(tc, ord);
  const bool take = key < C.key;
  C.key = take ? key : C.key;
  if constexpr (!kKeyOnly) {
    C.t = take ? tc : C.t;
    C.prim = take ? pi : C.prim;
  }
  if constexpr (kInst) C.inst = take ? inst : C.inst;
#endif
}

// Any primitive record against the open interval (tmin, C.t).  When the record is wave-uniform
// (flat sets) it sits in SGPRs and the kind / motion tests are scalar branches.
// kInst: the leaf may belong to instance cur_inst (its key order is offset by ord_base).
template <bool kKeyOnly = false, bool kInst = false>
RT_FN void test_rec(const KernelParams& P, const PrimRec& r, int pi, const RayCtx& R, real tmin, real tmin_up,
                    Closest& C, int cur_inst = -1, int ord_base = 0) {
  RT_COUNT(1);
  const int kf = RT_R2I(r.a.w);
  f3 o = R.o;
  if (kf & RT_FLAG_MOTION) o = o - motion_shift(P, RT_R2I(r.e.w), R.time_w);
  const bool self = is_self<kInst>(R, RT_R2I(r.b.w), cur_inst);
  real t, q;
  if ((kf & RT_KIND_MASK) == 0)
    isect_sphere(r, o, R, tmin, tmin_up, self, t, q);
  else if constexpr (!kKeyOnly)  // BVH leaves: parallelograms and triangles share one path
    isect_plane<-1>(r, o, R, tmin_up, self, t, q, (kf & RT_KIND_MASK) == 1);
  else if ((kf & RT_KIND_MASK) == 1)  // flat sets (uniform kind): scalar branch
    isect_plane<1>(r, o, R, tmin_up, self, t, q);
  else
    isect_plane<0>(r, o, R, tmin_up, self, t, q);
  consider<kKeyOnly, kInst>(C, t, q, RT_R2I(r.c.w) + ord_base, pi, cur_inst);
}

// A static primitive of a known kind (flat sets are grouped by class: rt_build.cpp).
template <int kKind, bool kKeyOnly = true, bool kInst = false>
RT_FN void test_static(const PrimRec& r, const RayCtx& R, real tmin, real tmin_up, Closest& C, int pi = 0) {
  RT_COUNT(1);
  const bool self = is_self<kInst>(R, RT_R2I(r.b.w), -1);  // a world leaf
  real t, q;
  if constexpr (kKind == RT_PRIM_CLASS_SPHERE)
    isect_sphere(r, R.o, R, tmin, tmin_up, self, t, q);
  else
    isect_plane<kKind == RT_PRIM_CLASS_QUAD ? 1 : 0>(r, R.o, R, tmin_up, self, t, q);
  consider<kKeyOnly, kInst>(C, t, q, RT_R2I(r.c.w), pi, -1);
}

// A box group (rt_internal.h DevBox): slabs in the box frame give the entry and exit points of
// the ray on the box surface; each is a candidate hit on the face it lies on (if the box has
// that face), with the same validity rules as a parallelogram test (t > tmin, not the face the
// ray leaves).  Wave-uniform record (scalar loads).
RT_FN int box_field(int base, int code, int f, bool& present) {
  const int off = (int)((unsigned)code >> (5 * f)) & 31;
  present = off != RT_BOX_NO_FACE;
  return base + off;
}
// (RT_BOX_EXIT_SKIP=0: the exit face decoded for every lane, as in round 3)
#ifndef RT_BOX_EXIT_SKIP
#define RT_BOX_EXIT_SKIP 1
#endif
// a face's key order, its primitive and whether the hit on it is valid (margin q >= 0, the face
// exists, and it is not the face the ray leaves)
template <bool kInst>
RT_FN bool box_face(const RT_CAS DevBox* B, int f, real q, const RayCtx& R, int& ord, int& prim, bool with_prim) {
  bool present;
  ord = box_field(B->ord_base, B->ord_code, f, present);
  const int gid = box_field(B->gid_base, B->gid_code, f, present);
  if (with_prim) prim = box_field(B->prim_base, B->prim_code, f, present);
  return present && !is_self<kInst>(R, gid, -1) && q >= RL(0.0);
}
template <bool kKeyOnly, bool kInst = false>
RT_FN void test_box(const RT_CAS DevBox* B, const RayCtx& R, real tmin_up, Closest& C) {
  RT_COUNT(1);
  const f3 ax[3] = {f3{B->a0[0], B->a0[1], B->a0[2]}, f3{B->a1[0], B->a1[1], B->a1[2]},
                    f3{B->a2[0], B->a2[1], B->a2[2]}};
  real lo[3], hi[3];
  int flip[3];
#if RT_F64 && !defined(RT_BOX_THREE_RCP)
  // Binary64: the three slab reciprocals from ONE reciprocal of their product, 1 / d_k =
  // (d_i d_j) / (d_0 d_1 d_2) — one v_rcp_f64 and its correction instead of three (within ~4 ulp
  // of 1 / d_k).  A product that is zero, denormal or infinite (an axis parallel to the ray)
  // takes the three guarded reciprocals instead, a branch no lane normally enters.
  real dk[3], invk[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) dk[k] = dot(ax[k], R.d);
  {
    const real d01 = dk[0] * dk[1], p = d01 * dk[2];
    const real r = RT_RCP_NZ(p);
    invk[0] = r * (dk[1] * dk[2]);
    invk[1] = r * (dk[0] * dk[2]);
    invk[2] = r * d01;
    if (!(RABS(p) >= RL(1e-300) && RABS(p) <= RL(1e300))) {
#pragma unroll
      for (int k = 0; k < 3; ++k) invk[k] = RT_RCP(dk[k]);
    }
  }
#endif
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#if RT_F64 && !defined(RT_BOX_THREE_RCP)
    const real inv = invk[k];
#else
    const real inv = RT_RCP(dot(ax[k], R.d));
#endif
    // s_k = a_k . (o - c) as a_k . o - a_k . c (DevBox::sc, host binary64): one FMA chain
    const real s = RFMA(ax[k].x, R.o.x, RFMA(ax[k].y, R.o.y, RFMA(ax[k].z, R.o.z, -B->sc[k])));
    const real t0 = -s * inv, t1 = RFMA(-s, inv, inv);  // the s = 0 and s = 1 planes
    // entering through the s = 1 end: t1 - t0 = inv, so t1 < t0 iff inv < 0 (the sign bit; the
    // two differ only when rounding makes t1 == t0, a slab |s| >= 2^52 box widths away)
    flip[k] = (int)(__builtin_bit_cast(ureal, inv) >> (8 * sizeof(real) - 1));
    lo[k] = RMIN(t0, t1);
    hi[k] = RMAX(t0, t1);
  }
  const real tn = RMAX(RMAX(lo[0], lo[1]), lo[2]), tf = RMIN(RMIN(hi[0], hi[1]), hi[2]);
  const int an = lo[0] == tn ? 0 : lo[1] == tn ? 1 : 2;
  const int fn = 2 * an + (an == 0 ? flip[0] : an == 1 ? flip[1] : flip[2]);
  const real gap = tf - tn;  // >= 0: the line meets the box
  // the entry point is nearer than the exit point: the exit matters only when the entry is not
  // a valid hit (one key compare per box)
  int ord_n, ord_f = 0, prim_n = 0, prim_f = 0;
  const bool vn = box_face<kInst>(B, fn, RMIN(gap, tn - tmin_up), R, ord_n, prim_n, !kKeyOnly);
  bool vf = false;
  const real qf = RMIN(gap, tf - tmin_up);
#if RT_BOX_EXIT_SKIP
  // ... and then only when the exit itself lies beyond tmin on a met box: rays from inside the box
  // (the Cornell room) need it, rays outside an object box (hitting its entry face, missing it, or
  // leaving its surface) do not — a wave-uniform branch skips the exit face's decode for them
  if (RT_ANY(!vn && qf >= RL(0.0)))
#endif
  {
    const int af = hi[0] == tf ? 0 : hi[1] == tf ? 1 : 2;
    const int ff = 2 * af + 1 - (af == 0 ? flip[0] : af == 1 ? flip[1] : flip[2]);
    vf = box_face<kInst>(B, ff, qf, R, ord_f, prim_f, !kKeyOnly);
  }
  consider<kKeyOnly, kInst>(C, vn ? tn : tf, (vn || vf) ? RL(0.0) : -RL(1.0), vn ? ord_n : ord_f,
                            vn ? prim_n : prim_f, -1);
}

// BVH scenes: the surface set's large-primitive prefix (rt_build.cpp; P.flat_sets[0]), tested
// before the traversal so that its closest hit bounds it.  The range is a kernel argument, so
// the records are wave-uniform (scalar loads) even when only some lanes start a query here.
template <bool kInst = false>
RT_FN void prefix_hits(const KernelParams& P, cfp prims, const RayCtx& R, real tmin, Closest& C) {
  const DevFlatSet& S = P.flat_sets[0];
  if (!P.surface_prefix || (S.end == S.first && S.box_end == S.box_first)) return;
  const real tmin_up = float_up(tmin);
  for (int b = S.box_first; b < S.box_end; ++b)
    test_box<false, kInst>((const RT_CAS DevBox*)P.boxes + b, R, tmin_up, C);
  int k = S.first;
  const RT_CAS PrimRec64* rp = (const RT_CAS PrimRec64*)prims + k;
  for (; k < S.end_quad; ++k, ++rp)
    test_static<RT_PRIM_CLASS_QUAD, false, kInst>(ld_rec64(rp), R, tmin, tmin_up, C, k);
  for (; k < S.end_tri; ++k, ++rp) test_static<RT_PRIM_CLASS_TRI, false, kInst>(ld_rec64(rp), R, tmin, tmin_up, C, k);
  for (; k < S.end_sphere; ++k, ++rp)
    test_static<RT_PRIM_CLASS_SPHERE, false, kInst>(ld_rec64(rp), R, tmin, tmin_up, C, k);
}


// Closest hit over one primitive set.  kFlat: the set is a single flat leaf (RT_FLAT_MAX
// leaves at most): every lane walks the same records in the same order, so the loop is coherent
// and the records are read with scalar loads (uniform addresses).
template <bool kFlat>
RT_FN void closest(const KernelParams& P, cfp prims, int root, int set, const RayCtx& R, real tmin, Closest& C,
                   const Trav& W, int* overflow);

struct HitInfo {
  f3 p, n;
  bool front;
  real u, v;
  int gid;
};

// front side of a boundary hit (constantMedium's case split, Geometry.hs:308)
RT_FN bool prim_front(const KernelParams& P, cfp prims, int pi, const RayCtx& R, real t) {
  cfp pr = prims + 16 * (size_t)pi;
  v4 a = ldc4(pr);
  int kf = RT_R2I(a.w);
  if ((kf & RT_KIND_MASK) == 0) {
    f3 c = xyz(a);
    if (kf & RT_FLAG_MOTION) c = c + motion_shift(P, RT_R2I(pr[15]), R.time_w);
    f3 p = R.o + t * R.d;
    return dot(R.d, p - c) * (pr[4] < RL(0.0) ? -RL(1.0) : RL(1.0)) <= RL(0.0);
  }
  return dot(xyz(a), R.d) < RL(0.0);
}

// need_uv: the material reads a (u, v) texture; otherwise the texture coordinates (sphereUV's
// atan2 / acos, the triangle's uv lerp and its prim_uv loads) are skipped.
RT_FN HitInfo surface_info(const KernelParams& P, cfp prims, int pi, const RayCtx& R, real t, bool need_uv) {
  HitInfo h;
  cfp pr = prims + 16 * (size_t)pi;
  v4 a = ldc4(pr), b = ldc4(pr + 4);
  int kf = RT_R2I(a.w);
  h.p = R.o + t * R.d;
  h.gid = RT_R2I(b.w);
  if ((kf & RT_KIND_MASK) == 0) {
    f3 c = xyz(a);
    if (kf & RT_FLAG_MOTION) c = c + motion_shift(P, RT_R2I(pr[15]), R.time_w);
    f3 outward = RT_RCP(b.x) * (h.p - c);
    h.front = dot(R.d, outward) <= RL(0.0);
    h.n = h.front ? outward : -outward;
    h.u = h.v = RL(0.0);
    if (!need_uv) return h;
    int uvf = RT_R2I(b.z);
    f3 on = outward;
    if (uvf >= 0) {
      cfp fr = cf(P.uvframes) + 12 * uvf;
      on = mk3(dot(ldc3(fr), outward), dot(ldc3(fr + 4), outward), dot(ldc3(fr + 8), outward));
    }
    // sphereUV (Geometry.hs:100-104)
    h.u = RATAN2(on.x, on.z) * (RL(0.5) / kPi) + RL(0.5);
    h.v = RACOS(RMIN(RL(1.0), RMAX(-RL(1.0), -on.y))) * (RL(1.0) / kPi);
  } else {
    f3 n = xyz(a);
    real denom = dot(n, R.d);
    h.front = denom < RL(0.0);
    h.n = h.front ? n : -n;
    h.u = h.v = RL(0.0);
    if (!need_uv) return h;
    f3 o = R.o;
    if (kf & RT_FLAG_MOTION) o = o - motion_shift(P, RT_R2I(pr[15]), R.time_w);
    f3 prel = (o + t * R.d) - xyz(b);
    real aa = dot(prel, ldc3(pr + 8)), bb = dot(prel, ldc3(pr + 12));
    cfp uv = cf(P.prim_uv) + 6 * (size_t)pi;
    real w0 = RL(1.0) - aa - bb;
    h.u = w0 * uv[0] + aa * uv[2] + bb * uv[4];
    h.v = w0 * uv[1] + aa * uv[3] + bb * uv[5];
  }
  return h;
}

// Perlin noise (Noise.hs:21-45): gradients at the 8 lattice corners, smoothstep weights.
// Kept compact (corner loop not unrolled) so the rarely used noise textures do not raise the
// register allocation of the whole lane loop.
RT_FN real smooth3(real x) { return x * x * (RL(3.0) - RL(2.0) * x); }
RT_FN real perlin_noise(const RT_CAS int* perm, cfp grad, f3 p) {
  const real x0 = RFLOOR(p.x), y0 = RFLOOR(p.y), z0 = RFLOOR(p.z);
  const int ix = (int)x0, iy = (int)y0, iz = (int)z0;
  const real fx = p.x - x0, fy = p.y - y0, fz = p.z - z0;
  real sum = RL(0.0);
#pragma unroll 1
  for (int c = 0; c < 8; ++c) {
    const int i = c >> 2, j = (c >> 1) & 1, k = c & 1;
    const int g = perm[(ix + i) & 255] ^ perm[256 + ((iy + j) & 255)] ^ perm[512 + ((iz + k) & 255)];
    const real rx = fx - (real)i, ry = fy - (real)j, rz = fz - (real)k;
    const real w = smooth3(i ? fx : RL(1.0) - fx) * smooth3(j ? fy : RL(1.0) - fy) * smooth3(k ? fz : RL(1.0) - fz);
    sum += w * dot(ldc3(grad + 4 * g), mk3(rx, ry, rz));
  }
  return sum;
}
// fractalNoise (Noise.hs:48-53): layers of doubling frequency and halving weight
RT_FN real fractal_noise(const RT_CAS int* perm, cfp grad, int depth, f3 p) {
  real sum = RL(0.0), w = RL(1.0);
#pragma unroll 1
  for (int l = 0; l < depth; ++l) {
    sum += w * perlin_noise(perm, grad, p);
    w *= RL(0.5);
    p = RL(2.0) * p;
  }
  return sum;
}
// Solid noise textures.  Their register needs (lattice corners per octave, on top of the live
// path state) would raise the allocation of the whole lane loop, so they are compiled only into
// the kernel instantiations for scenes that use them (template flag kNoise, host-selected).
RT_FN f3 eval_noise_texture(const RT_CAS int* perm, cfp grad, const RT_CAS DevTexture* T, f3 p) {
  f3 c0 = f3{T->c0[0], T->c0[1], T->c0[2]};
  if (T->kind == RT_TEX_NOISE) {  // noiseTexture (Texture.hs:56-67)
    const f3 q = T->prm[0] * p + mk3(T->prm[1], T->prm[2], T->prm[3]);
    const real n = fractal_noise(perm, grad, T->nu, q) * (RL(0.5) / RL(0.8)) + RL(0.5);
    return c0 + n * (f3{T->c1[0], T->c1[1], T->c1[2]} - c0);
  }
  // marbleTexture (Texture.hs:70-78)
  const real freq = T->prm[3];
  const real arg = freq * dot(mk3(T->prm[0], T->prm[1], T->prm[2]), p);
  const real turb =
      RABS(fractal_noise(perm, grad, 7, (RL(0.25) * freq) * p + mk3(T->prm[4], T->prm[5], T->prm[6])));
  const real m = RL(0.5) + RL(0.5) * RSIN(arg + RL(10.0) * turb);
  return mk3(m, m, m);
}

// Textures (Texture.hs:18-78); (u, v) for uv textures, the hit point p for solid ones
template <bool kNoise>
RT_FN f3 eval_texture(const KernelParams& P, int tex, real u, real v, f3 p) {
  const RT_CAS DevTexture* T = (const RT_CAS DevTexture*)P.texs + tex;
  const int kind = T->kind;
  f3 c0 = f3{T->c0[0], T->c0[1], T->c0[2]};
  if (kind == RT_TEX_CONSTANT) return c0;
  if (kind == RT_TEX_CHECKER) {  // checkerTexture (Texture.hs:45-53)
    int i = (int)RFLOOR(u * (real)T->nu), j = (int)RFLOOR(v * (real)T->nv);
    return ((i + j) & 1) == 0 ? c0 : f3{T->c1[0], T->c1[1], T->c1[2]};
  }
  if (kind == RT_TEX_IMAGE) {  // imageTexture (Texture.hs:31-41): wrap, v = 0 at the bottom row
    const int w = T->nu, h = T->nv;
    int i = (int)RFLOOR(u * (real)w) % w, j = (int)RFLOOR((RL(1.0) - v) * (real)h) % h;
    i += i < 0 ? w : 0;
    j += j < 0 ? h : 0;
    return ldc3(cf(P.texels) + 4 * ((size_t)T->off + (size_t)j * w + i));
  }
  if constexpr (kNoise) return eval_noise_texture((const RT_CAS int*)P.perlin_perm, cf(P.perlin_grad), T, p);
  return c0;  // not reached: scenes with noise textures run the kNoise kernels
}

// rt_hit of a redirect target: parallelogram on (0, infinity) (Ray.hs:143-145); rinv = 1 / (n . d)
RT_FN bool target_hit(const DevTarget& T, f3 o, f3 d, real& t, real& rinv) {
  f3 n = ld3(T.n);
  real denom = dot(n, d);
  if (!(RABS(denom) > RL(1e-8))) return false;
  f3 qo = ld3(T.q) - o;
  rinv = RT_RCP_NZ(denom);
  t = dot(n, qo) * rinv;
  if (!(t > RL(0.0))) return false;
  f3 prel = t * d - qo;
  real a = dot(prel, ld3(T.wa)), b = dot(prel, ld3(T.wb));
  return a >= RL(0.0) && a <= RL(1.0) && b >= RL(0.0) && b <= RL(1.0);
}

// Per-sample radiance -> fixed point; non-finite values set the pixel's flag.  A lane sums the
// samples of its item in an Acc and commits it with integer atomics (rt_kernel.hip).
#if RT_F64
// trunc(x 2^32) and the next 32 bits of x 2^64 (RT_ACC_WORDS = 6): x 2^32 and its floor are
// exact in binary64 (a power-of-two scale), so is the fraction, and the fraction times 2^32 is
// exact too, so the two words hold x to 2^-64 — every bit of a binary64 radiance >= 2^-11.
struct Acc {
  long long hi[3];
  unsigned long long lo[3];
};
RT_FN void acc_add(Acc& A, int c, real x, bool& bad) {
  if (!(RABS(x) < RL(1.0e9))) {
    bad = true;
    return;
  }
  // (the same words from 32-bit conversions only, floor(x) 2^32 + floor(frac(x) 2^32), measured no
  // faster: Cornell 4.887 vs 4.889 ms, pawn+fog +1 %; profiles/r5/variants.  From the low words of
  // integer-valued binary64 plus 1.5 2^52, no conversions: Cornell +1.4 %, profiles/r6/flat)
  const real xs = x * RL(4294967296.0);
  const real fl = RFLOOR(xs);
  A.hi[c] += (long long)fl;
  A.lo[c] += (unsigned long long)(unsigned)((xs - fl) * RL(4294967296.0));
}
#else
// trunc(x 2^32) (RT_ACC_WORDS = 3)
struct Acc {
  long long hi[3];
};
RT_FN long long to_fixed(real x, bool& bad) {
  if (!(RABS(x) < RL(1.0e9))) {
    bad = true;
    return 0;
  }
  // x * 2^32 without FP64: for x >= 0 (radiance) the integer part and the fraction are exact
  // in FP32 (x - floor(x) is exact) and the fraction scaled by 2^32 is exact, so two 32-bit
  // conversions give exactly trunc(x * 2^32).  (Negative inputs, possible only with negative
  // user colours, are within 2^-25 relative of it.)
  const real fl = RFLOOR(x);
  const long long hi = (long long)(int)fl;
  const unsigned lo = (unsigned)((x - fl) * RL(4294967296.0));
  return (long long)((unsigned long long)hi << 32) + (long long)lo;
}
RT_FN void acc_add(Acc& A, int c, real x, bool& bad) { A.hi[c] += to_fixed(x, bad); }
#endif
RT_FN void acc_clear(Acc& A) { A = Acc{}; }
RT_FN void acc_sample(Acc& A, f3 L, bool& bad) {
  acc_add(A, 0, L.x, bad);
  acc_add(A, 1, L.y, bad);
  acc_add(A, 2, L.z, bad);
}
// The item's sums in the workgroup's LDS instead of registers (the device kernels): word k of the
// lane is w[k * stride] (word-major: a wave's 64 lanes touch consecutive 8-B words, no bank
// conflicts).  A sample adds its words with LDS atomics (ds_add_u64, no return); the words are
// read once per item, at its commit.  Frees RT_ACC_WORDS x 2 VGPRs of state that is touched once
// per sample but live across the whole lane loop.
struct AccLds {
  unsigned long long* w;
  int stride;
};
RT_FN void acc_clear(AccLds& A) {
#pragma unroll
  for (int k = 0; k < RT_ACC_WORDS(real); ++k) A.w[k * A.stride] = 0ull;
}
RT_FN void lds_add(unsigned long long* p, unsigned long long v) {
#ifdef RT_HOST_EMU
  *p += v;
#else
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
RT_FN void acc_sample(AccLds& A, f3 L, bool& bad) {
  Acc t;
  acc_clear(t);
  acc_sample(t, L, bad);
#pragma unroll
  for (int c = 0; c < 3; ++c)
    if (t.hi[c]) lds_add(A.w + c * A.stride, (unsigned long long)t.hi[c]);
#if RT_F64
#pragma unroll
  for (int c = 0; c < 3; ++c)
    if (t.lo[c]) lds_add(A.w + (3 + c) * A.stride, t.lo[c]);
#endif
}
// the sums of an accumulator (commit)
RT_FN Acc acc_words(const Acc& A) { return A; }
RT_FN Acc acc_words(const AccLds& A) {
  Acc t;
#pragma unroll
  for (int c = 0; c < 3; ++c) t.hi[c] = (long long)A.w[c * A.stride];
#if RT_F64
#pragma unroll
  for (int c = 0; c < 3; ++c) t.lo[c] = A.w[(3 + c) * A.stride];
#endif
  return t;
}

// Diagnostic build only (make exp DEFS=-DRT_PHASE_PROF, tools/phase_prof.py): per-wave shader
// clocks and lane counts by phase of lane_loop_bvh and trav_round, summed over the launch into
// rt_prof_buf.
#if defined(RT_PHASE_PROF) && !defined(RT_HOST_EMU)
enum : int { PF_FRONT, PF_TRAV, PF_SHADE, PF_ITERS, PF_ROUNDS, PF_TRACING, PF_LIVE, PF_SHADING, PF_FRONT_LANES,
             PF_NODE_STEPS, PF_NODE_LANES, PF_LEAF_STEPS, PF_LEAF_LANES, PF_NODE_CLK, PF_LEAF_CLK, PF_CAM,
             PF_CAM_LANES, PF_N };
static __device__ unsigned long long rt_prof_buf[PF_N];  // (one per translation unit: rt_render_kernel.h)
#define RT_PROF_DECL unsigned long long prof[PF_N] = {}; unsigned long long pf_t0 = clock64(), pf_t1;
#define RT_PROF_MARK(k) (pf_t1 = clock64(), prof[k] += pf_t1 - pf_t0, pf_t0 = pf_t1)
#define RT_PROF_ADD(k, x) (prof[k] += (unsigned long long)(x))
#define RT_PROF_FLUSH                                                       \
  if ((threadIdx.x & 63) == 0)                                              \
    for (int k = 0; k < PF_N; ++k) atomicAdd(&rt_prof_buf[k], prof[k]);
#define RT_PROF_PARAM , unsigned long long* prof
#define RT_PROF_ARG , prof
#define RT_PROF_NULLARG , (unsigned long long*)nullptr
#define RT_PROF_PADD(k, x) (prof ? (void)(prof[k] += (unsigned long long)(x)) : (void)0)
#define RT_PROF_CLK() clock64()
#else
#define RT_PROF_DECL
#define RT_PROF_MARK(k) ((void)0)
#define RT_PROF_ADD(k, x) ((void)0)
#define RT_PROF_FLUSH
#define RT_PROF_PARAM
#define RT_PROF_ARG
#define RT_PROF_NULLARG
#define RT_PROF_PADD(k, x) ((void)0)
#define RT_PROF_CLK() 0ull
#endif

// ---------------------------------------------------------------- BVH traversal
// Resumable per-lane BVH traversal (the body of trace_set, split so a lane can stop between
// rounds and continue in a later iteration of the lane loop with its state intact).
struct TravState {
  int node, leaf, sp;
  real tmin, tmin_up;
  Closest C;
  int inst, ord_base;  // instancing: the placement being traversed (-1: world) and its key-order offset
  f3 wo, wd;           // ... and the world ray, restored at RT_INST_EXIT
};
RT_FN void trav_begin(TravState& S, int root, real tmin) {
  S.node = root;
  S.leaf = 0;
  S.sp = 0;
  if (root < 0) {  // an empty set, or a set that is one leaf
    S.leaf = root == RT_EMPTY_ROOT ? 0 : root;
    S.node = RT_EMPTY_ROOT;
  }
  S.tmin = tmin;
  S.tmin_up = float_up(tmin);
  S.C = no_hit();
  S.inst = -1;
  S.ord_base = 0;
}
RT_FN bool trav_done(const TravState& S) { return S.node == RT_EMPTY_ROOT && S.leaf == 0; }

// FP32 kernels read global nodes at a 32-bit offset from the uniform base (bunny-Cornell -0.3 %,
// demo1 -1.5 %, pawn+fog -1.0 %); the binary64 kernels keep 64-bit addresses (demo1 +2.4 % with
// the offsets, bunny and pawn+fog -0.9 %: profiles/r3/fetch)
#ifndef RT_NODE_SADDR
#define RT_NODE_SADDR (!RT_F64)
#endif
// The word offset of a stack row.  (Experiments, profiles/r6/nondet: RT_STACK_ASM_NOP computes it
// with v_mul_lo_u32 in inline assembly followed by wait states, to test a multiply -> LDS-address
// hazard in the runtime-stride builds that rendered nondeterministically.)
#if defined(RT_STACK_ASM_NOP) && !defined(RT_HOST_EMU)
RT_FN int stack_row_asm(int row, int stride) {
  int off;
  asm volatile("v_mul_lo_u32 %0, %1, %2\n\ts_nop 7\n\ts_nop 7" : "=v"(off) : "v"(row), "s"(stride));
  return off;
}
#define RT_STACK_ROW(row, stride) stack_row_asm((row), (stride))
#else
#define RT_STACK_ROW(row, stride) ((row) * (stride))
#endif
// One while-while round: descend until this lane (and the wave) holds a leaf, then test leaves.
// kInst (two-level instancing): a child RT_INST_FLAG | k enters placement k — the lane's ray R
// is moved to object space, RT_INST_EXIT is pushed and the object's BVH is traversed; popping
// RT_INST_EXIT restores the world ray.  t is the same in both spaces (rigid), so the closest
// hit's bound carries over; a parked leaf is tested before the ray changes space.
// kLeaf: 0 generic leaf records; 1 / 2 every leaf record is a static triangle / sphere (one test,
// no class dispatch or motion; a measured 2-4 % on the bunny and demo1 scenes)
template <bool kInst = false, int kLeaf = 0, class RC>
RT_FN void trav_round(const KernelParams& P, RC& R, TravState& S, const Trav& W, int& overflow RT_PROF_PARAM) {
  unsigned long long pf_c0 = RT_PROF_CLK();
  constexpr int kDone = RT_EMPTY_ROOT;
  int* const stack = W.stack;
  const int stride = W.stride;
  auto pop = [&]() -> int {
    if (S.sp == 0) return kDone;
    --S.sp;
    return stack[RT_STACK_ROW(S.sp, stride)];
  };
  while (S.node >= 0) {
    RT_PROF_PADD(PF_NODE_STEPS, 1);
    RT_PROF_PADD(PF_NODE_LANES, RT_BALLOT_COUNT(true));
    if constexpr (kInst) {
      if (S.node >= RT_INST_FLAG) {
        if (S.leaf != 0) break;  // test the parked leaf in the space it was found in
        if (S.node == RT_INST_EXIT) {
          R.o = S.wo;
          R.d = S.wd;
          prep_ray(R);
          S.inst = -1;
          S.ord_base = 0;
          S.node = pop();
          if (S.node < 0 && S.node != kDone) {  // a world leaf was the next entry: park it
            S.leaf = S.node;
            S.node = pop();
          }
        } else {
          const int k = S.node - RT_INST_FLAG;
          const RT_CAS DevInstance* I = inst_rec(P, k);
          if (S.sp < P.stack_depth) {
            stack[RT_STACK_ROW(S.sp, stride)] = RT_INST_EXIT;
            ++S.sp;
          } else {
            overflow = 1;  // the stack is sized for world + object levels (rt_build.cpp): not reached
          }
          S.wo = R.o;
          S.wd = R.d;
          R.o = inst_to_object(I, R.o, true);
          R.d = inst_to_object(I, R.d, false);
          prep_ray(R);
          S.inst = k;
          S.ord_base = I->order;
          S.node = I->root;
          if (S.node < 0 && S.node != kDone) {  // the object is one leaf: park it, pop the exit
            S.leaf = S.node;
            S.node = pop();
          }
        }
        continue;
      }
    }
    RT_COUNT(0);
    v4f n0, n1, n2;
    int cl, cr;
    const int node = S.node;
    // (a wave-uniform source — LDS only when every stepping lane's node is staged — measured
    // slower: pawn+fog +8.5 % FP32)
    const bool from_lds = node < P.lds_nodes;
    if (from_lds) {  // top levels of the surface BVH, staged in LDS per workgroup
      const v4f* nd = W.lds_nodes + 4 * node;
      n0 = nd[0];
      n1 = nd[1];
      n2 = nd[2];
      cl = RT_F2I(nd[3].x);
      cr = RT_F2I(nd[3].y);
    } else {
#if RT_NODE_SADDR
      // a 32-bit byte offset from the uniform base (node < 2^26: rt_build.cpp refuses larger BVHs,
      // RT_MAX_NODES): the loads take the scalar-base +
      // vector-offset form, no 64-bit address arithmetic per lane
      cfpf nd = (cfpf)((const RT_CAS char*)P.nodes + ((uint32_t)node << 6));
#else
      cfpf nd = (cfpf)P.nodes + 16 * (size_t)node;
#endif
      n0 = ldc4f(nd);
      n1 = ldc4f(nd + 4);
      n2 = ldc4f(nd + 8);
      const RT_CAS i4* n3p = (const RT_CAS i4*)(nd + 12);
      cl = n3p->x;
      cr = n3p->y;
    }
#if RT_NODE_F32
    float lnear, lfar, rnear, rfar;
    node_slabs_f32(R, n0, n1, n2, (float)S.tmin, (float)S.C.t, lnear, lfar, rnear, rfar);
#else
    real lx0 = RFMA(n0.x, R.idir.x, -R.oidir.x), lx1 = RFMA(n0.y, R.idir.x, -R.oidir.x);
    real ly0 = RFMA(n0.z, R.idir.y, -R.oidir.y), ly1 = RFMA(n0.w, R.idir.y, -R.oidir.y);
    real lz0 = RFMA(n2.x, R.idir.z, -R.oidir.z), lz1 = RFMA(n2.y, R.idir.z, -R.oidir.z);
    real rx0 = RFMA(n1.x, R.idir.x, -R.oidir.x), rx1 = RFMA(n1.y, R.idir.x, -R.oidir.x);
    real ry0 = RFMA(n1.z, R.idir.y, -R.oidir.y), ry1 = RFMA(n1.w, R.idir.y, -R.oidir.y);
    real rz0 = RFMA(n2.z, R.idir.z, -R.oidir.z), rz1 = RFMA(n2.w, R.idir.z, -R.oidir.z);
    real lnear = RMAX(RMAX(RMIN(lx0, lx1), RMIN(ly0, ly1)), RMAX(RMIN(lz0, lz1), S.tmin));
    real lfar = RMIN(RMIN(RMAX(lx0, lx1), RMAX(ly0, ly1)), RMIN(RMAX(lz0, lz1), S.C.t));
    real rnear = RMAX(RMAX(RMIN(rx0, rx1), RMIN(ry0, ry1)), RMAX(RMIN(rz0, rz1), S.tmin));
    real rfar = RMIN(RMIN(RMAX(rx0, rx1), RMAX(ry0, ry1)), RMIN(RMAX(rz0, rz1), S.C.t));
#endif
    const bool hl = lnear <= lfar, hr = rnear <= rfar;
    {
      // Branch-free step: the stack slots a pop may need (sp-1, sp-2) are read and the far child
      // is written to slot sp (free; slot stack_depth is a spare row) every step, and the next
      // node / stack pointer are selects — no divergent branches around the LDS accesses.
      const bool both = hl && hr, one = hl != hr;
      const bool rfirst = rnear < lnear;
      const int nearc = both ? (rfirst ? cr : cl) : (hl ? cl : cr);
      const int farc = rfirst ? cl : cr;
      const int sp = S.sp;
      const int top1 = stack[RT_STACK_ROW(sp > 0 ? sp - 1 : 0, stride)];
      const int top2 = stack[RT_STACK_ROW(sp > 1 ? sp - 2 : 0, stride)];
      const bool room = sp < P.stack_depth;
      stack[RT_STACK_ROW(room ? sp : P.stack_depth, stride)] = farc;
      overflow |= (both && !room) ? 1 : 0;
      int next = (both || one) ? nearc : (sp > 0 ? top1 : kDone);
      int nsp = both ? (room ? sp + 1 : sp) : one ? sp : (sp > 0 ? sp - 1 : 0);
      if (next < 0 && next != kDone && S.leaf == 0) {  // park the first leaf, keep descending
        S.leaf = next;
        const bool pushed = both && room;  // its pop is the far child just written
        next = pushed ? farc : (both || one) ? (sp > 0 ? top1 : kDone) : (sp > 1 ? top2 : kDone);
        nsp = pushed ? sp : (both || one) ? (sp > 0 ? sp - 1 : 0) : (sp > 1 ? sp - 2 : 0);
      }
      S.node = next;
      S.sp = nsp;
    }
    // leave the node loop once P.leaf_exit_pct % of its lanes hold a leaf (100: all of them,
    // Aila & Laine's while-while); the rest keep their state and descend in the next round
    if (RT_BALLOT_COUNT(S.leaf != 0) * 100 >= RT_BALLOT_COUNT(true) * P.leaf_exit_pct) break;
  }
  unsigned long long pf_c1 = RT_PROF_CLK();
  RT_PROF_PADD(PF_NODE_CLK, pf_c1 - pf_c0);
  while (S.leaf < 0) {
    RT_PROF_PADD(PF_LEAF_STEPS, 1);
    RT_PROF_PADD(PF_LEAF_LANES, RT_BALLOT_COUNT(true));
    const int enc = ~S.leaf;
    const int first = enc >> RT_LEAF_SHIFT, count = (enc & ((1 << RT_LEAF_SHIFT) - 1)) + 1;
    auto test_one = [&](const PrimRec& r, int pi) {
      if constexpr (kLeaf == 1)  // every leaf a static triangle (RT_VAR_LEAF_TRI)
        test_static<RT_PRIM_CLASS_TRI, false>(r, R, S.tmin, S.tmin_up, S.C, pi);
      else if constexpr (kLeaf == 2)  // every leaf a static sphere (RT_VAR_LEAF_SPHERE)
        test_static<RT_PRIM_CLASS_SPHERE, false>(r, R, S.tmin, S.tmin_up, S.C, pi);
      else
        test_rec<false, kInst>(P, r, pi, R, S.tmin, S.tmin_up, S.C, S.inst, S.ord_base);
    };
    // (both records of a 2-record leaf loaded before either test — one memory latency per leaf
    // instead of two — spilled the binary64 bunny kernel: +3.4 %, pawn+fog FP32 +4 %, demo1 -0.7 %;
    // profiles/r5/variants)
    for (int k = 0; k < count; ++k) test_one(ld_rec(cf(P.prims) + 16 * (size_t)(first + k)), first + k);
    S.leaf = 0;
    if (S.node < 0 && S.node != kDone) {  // the node we stopped at is a leaf too: test it next
      S.leaf = S.node;
      S.node = pop();
    }
  }
  RT_PROF_PADD(PF_LEAF_CLK, RT_PROF_CLK() - pf_c1);
  (void)pf_c0;
  (void)pf_c1;
}

// A query whose set is one leaf (trav_begin parked it): its records by the generic test.
template <bool kInst, class RC>
RT_FN void test_leaf_generic(const KernelParams& P, RC& R, TravState& S) {
  while (S.leaf < 0) {
    const int enc = ~S.leaf;
    const int first = enc >> RT_LEAF_SHIFT, count = (enc & ((1 << RT_LEAF_SHIFT) - 1)) + 1;
    for (int k = 0; k < count; ++k)
      test_rec<false, kInst>(P, ld_rec(cf(P.prims) + 16 * (size_t)(first + k)), first + k, R, S.tmin, S.tmin_up, S.C,
                             S.inst, S.ord_base);
    S.leaf = 0;
  }
}

// kFlat: the set is one flat leaf (rt_internal.h DevFlatSet); every lane walks the same
// records in the same order, so the loops are coherent and the records are scalar loads.
template <>
RT_FN_SPEC void closest<true>(const KernelParams& P, cfp prims, int root, int set, const RayCtx& R, real tmin, Closest& C,
                         const Trav& W, int* overflow) {
  (void)prims;
  (void)root;
  (void)W;
  (void)overflow;
  {
    // set comes from the kernel arguments: the ranges are wave-uniform, every loop is scalar
    const DevFlatSet& S = P.flat_sets[set];
    const real tmin_up = float_up(tmin);
    for (int b = S.box_first; b < S.box_end; ++b) test_box<true>((const RT_CAS DevBox*)P.boxes + b, R, tmin_up, C);
    int k = S.first;
    const RT_CAS PrimRec64* rp = (const RT_CAS PrimRec64*)P.flat_recs + k;  // one 64-B scalar load per record
    for (; k < S.end_quad; ++k, ++rp) test_static<RT_PRIM_CLASS_QUAD>(ld_rec64(rp), R, tmin, tmin_up, C);
    for (; k < S.end_tri; ++k, ++rp) test_static<RT_PRIM_CLASS_TRI>(ld_rec64(rp), R, tmin, tmin_up, C);
    for (; k < S.end_sphere; ++k, ++rp) test_static<RT_PRIM_CLASS_SPHERE>(ld_rec64(rp), R, tmin, tmin_up, C);
    for (; k < S.end; ++k, ++rp) test_rec<true>(P, ld_rec64(rp), k, R, tmin, tmin_up, C);
#if RT_F64
    if (C.t < kInf) C.prim = C.ord;  // slot = primitive index (flat scenes store prims in slot order)
#else
    const uint32_t hi = (uint32_t)(C.key >> 32);
    if (hi < 0x7f800000u) {  // a finite t won
      C.t = __builtin_bit_cast(real, hi);
      C.prim = (int)(uint32_t)C.key;  // slot = primitive index (flat scenes store prims in slot order)
    }
#endif
  }
}

// BVH set (lockstep variant): resumable rounds run to completion.
template <>
RT_FN_SPEC void closest<false>(const KernelParams& P, cfp prims, int root, int set, const RayCtx& R, real tmin,
                          Closest& C, const Trav& W, int* overflow) {
  TravState S;
  trav_begin(S, root, tmin);
  if (set == 0) prefix_hits(P, prims, R, tmin, S.C);
  while (!trav_done(S)) trav_round(P, R, S, W, *overflow RT_PROF_NULLARG);
  C = S.C;
}

// The kernel arguments through a pointer the compiler cannot see through (RT_KARGS): a field read
// after it is a scalar load from the kernarg segment at that point, not a value hoisted out of the
// persistent lane loop and held in SGPRs for the whole kernel.  The lane loops re-derive P at
// each phase (front end, traversal round, shading; the flat loop per iteration) and the work queue
// per call (rt_render_kernel.h WaveWork::kp): the camera, material, target and queue fields are
// then live for their phase only.  SGPR spills (each restore a v_readlane, a VALU instruction, in
// the loop) 31 / 56 / 84 -> 0 / 2 / 2 in the binary64 Cornell / bunny / demo1 kernels, none left in
// a loop; demo1 binary64 -4.2 %, pawn+fog -1.8 % (profiles/r4/kargs_ab).  The kernel's one
// argument is its KernelParams, so the kernarg segment starts with it: RT_KARGS(P0) stands for the
// KERNEL'S OWN argument (never a modified copy — the kernels pass theirs, unmodified, to the lane
// loops); the host emulator returns P0 itself.
#ifndef RT_KARGS_OPAQUE
#define RT_KARGS_OPAQUE 1
#endif
#if defined(RT_HOST_EMU) || !RT_KARGS_OPAQUE
#define RT_KARGS(P0) (P0)
#else
RT_FN const KernelParams& rt_kargs() {
  const RT_CAS KernelParams* pp = (const RT_CAS KernelParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pp));
  return *(const KernelParams*)pp;
}
#define RT_KARGS(P0) rt_kargs()
#endif
// per-phase switches (1: re-read), measured per precision (profiles/r4/kargs_phase_ab): the FP32
// BVH kernels keep the traversal rounds' arguments in SGPRs (bunny-Cornell / demo1 / pawn+fog
// -0.9 / -0.9 / -1.0 % against re-reading them per round), the binary64 ones re-read them (pawn+fog
// +0.7 % without); the BVH kernels' work queue re-reads its fields in FP32 only
// (rt_render_kernel.h RT_KARGS_WORK_BVH)
#ifndef RT_KARGS_TRAV
#define RT_KARGS_TRAV RT_F64
#endif
#define RT_KARGS_IF(on, P0) ((on) ? RT_KARGS(P0) : (P0))

// ------------------------------------------------------------------ per-path pieces
// Ray.hs:157-172, 229: pixel jitter, time, defocus-disk point -> primary ray
RT_FN uint32_t fast_div(uint32_t n, const FastDiv& f) {
  if (f.d == 1u) return n;  // uniform
  const uint32_t t = (uint32_t)(((uint64_t)n * f.m) >> 32);
  return (t + ((n - t) >> 1)) >> f.s;
}
// pxgy: the pixel's gy << 16 | px (the flat kernel keeps it from open_item), or ~0u: derived from
// pix here (the register-bound BVH kernels, for which a persistent word costs more than a division)
RT_FN void camera_ray(const KernelParams& P, uint32_t pix, int sample, uint32_t pxgy, RayCtx& R) {
  int gy, px;
  if (pxgy == ~0u) {
    gy = (int)fast_div(pix, P.div_width);
    px = (int)pix - gy * P.cam.width;
  } else {
    gy = (int)(pxgy >> 16);
    px = (int)(pxgy & 0xffffu);
  }
  u4 w0 = philox(pix, (uint32_t)sample, 0u, RT_EV_CAMERA0, P.key0, P.key1);
  R.time_w = w0.z;
  f3 origin = ld3(P.cam.center);
  if (P.cam.disk_u[0] != RL(0.0) || P.cam.disk_u[1] != RL(0.0) || P.cam.disk_u[2] != RL(0.0) || P.cam.disk_v[0] != RL(0.0) ||
      P.cam.disk_v[1] != RL(0.0) || P.cam.disk_v[2] != RL(0.0)) {
    u4 w1 = philox(pix, (uint32_t)sample, 0u, RT_EV_CAMERA1, P.key0, P.key1);
    real rad = RT_SQRT(u01(w0.w)), s, c;
    RT_SINCOS_TURNS(u01(w1.x), &s, &c);
    origin = origin + (rad * c) * ld3(P.cam.disk_u) + (rad * s) * ld3(P.cam.disk_v);
  }
  f3 target = ld3(P.cam.top_left) + ((real)px + u01(w0.x)) * ld3(P.cam.pixel_u) +
              ((real)gy + u01(w0.y)) * ld3(P.cam.pixel_v);
  R.o = origin;
  R.d = normalize(target - origin);
  R.self_gid = -1;
  R.self_inst = -1;
}

// constantMedium's free-flight draw over the segment (lo, hi) (Geometry.hs:312-328); wm is the
// Philox block of event RT_EV_MEDIA + m / 4 of this segment
RT_FN void medium_draw(const KernelParams& P, int m, u4 wm, real lo, real hi, real& tbest, int& hit_medium) {
  // no FMA contraction of lo + hit_dist (the reference's two roundings, Geometry.hs:320-322): the
  // compiler's choice would otherwise depend on where the draw is inlined, and the media_late and
  // query-chain kernels must agree bit for bit
#ifndef RT_HOST_EMU
#pragma clang fp contract(off)
#endif
  uint32_t wsel = (m & 3) == 0 ? wm.x : (m & 3) == 1 ? wm.y : (m & 3) == 2 ? wm.z : wm.w;
  real rnd = RL(1.0) - u01(wsel);
  real hit_dist = P.media[m].neg_inv_density * RT_LOG(rnd);
  if (hit_dist < hi - lo) {
    real t = lo + hit_dist;
    if (t < tbest) {
      tbest = t;
      hit_medium = m;
    }
  }
}
RT_FN u4 medium_block(const KernelParams& P, int m, uint32_t pix, int sample, int seg) {
  return philox(pix, (uint32_t)sample, (uint32_t)seg, RT_EV_MEDIA + (uint32_t)(m >> 2), P.key0, P.key1);
}
RT_FN void medium_event(const KernelParams& P, int m, uint32_t pix, int sample, int seg, real lo, real hi,
                        real& tbest, int& hit_medium) {
  medium_draw(P, m, medium_block(P, m, pix, sample, seg), lo, hi, tbest, hit_medium);
}

// The HemisphereF / SphereF scatter (Ray.hs:187-224): the direction from the redirect mixture
// (target k by the cumulative probabilities, else the default sampler) and the weight
// f pdf1 / pdf with pdf = remProb pdf1 + sum_k p_k t_k^2 / |(U_k x V_k) . dir|.  Returns false
// when a HemisphereF direction is below the surface (pdf1 <= 0: the path ends, Ray.hs:198).
// kEarly: return there, newdir and Tf untouched (the full-material kernels, whose register
// allocation needs the short exit); otherwise they are written either way.
template <bool kMats, bool kEarly>
RT_FN bool mixture_scatter(const KernelParams& P, const HitInfo& h, const RayCtx& R, const u4& w, const DevMaterial& Mt,
                           bool hemi, f3 tex, f3& newdir, f3& Tf) {
  real cr = u01(w.x);
  int choice = -1;
  for (int k = 0; k < P.n_targets; ++k) {
    if (cr < P.targets[k].thresh) {
      choice = k;
      break;
    }
  }
  f3 dir;
  if (choice < 0) {
    f3 uu = unit_vector(w.y, w.z);
    dir = hemi ? normalize(h.n + uu) : uu;
  } else {
    const DevTarget& Tg = P.targets[choice];
    f3 lp = ld3(Tg.q) + u01(w.y) * ld3(Tg.u) + u01(w.z) * ld3(Tg.v);
    dir = normalize(lp - h.p);
  }
  real pdf1 = hemi ? dot(dir, h.n) * (RL(1.0) / kPi) : RL(0.25) / kPi;
  if constexpr (kEarly)
    if (hemi && pdf1 <= RL(0.0)) return false;
  real mix = RL(0.0);
  for (int k = 0; k < P.n_targets; ++k) {
    // p t^2 / |(u x v) . dir| (Ray.hs:202) with (u x v) . dir = |u x v| (n . dir): the target
    // test's reciprocal serves both
    real tt, rinv;
    if (target_hit(P.targets[k], h.p, dir, tt, rinv)) mix += P.targets[k].prob_icr * (tt * tt * RABS(rinv));
  }
  real pdf = P.rem_prob * pdf1 + mix;
  f3 f = tex;
  if constexpr (kMats) {
    if (Mt.kind == 3) {  // lommelSeeliger
      real mu0 = -dot(R.d, h.n), mu1 = dot(dir, h.n);
      f = (RL(0.25) * RT_RCP(mu0 + mu1)) * f;
    } else if (Mt.kind == 9) {  // anisotropic (Henyey-Greenstein)
      real g = Mt.param, mu = dot(R.d, dir);
      real base = RL(1.0) + g * g - RL(2.0) * g * mu;
      f = ((RL(1.0) - g * g) * RT_RCP(base * RT_SQRT(base))) * f;
    }
  }
  Tf = (pdf1 * RT_RCP(pdf)) * f;
  newdir = dir;
  return !(hemi && pdf1 <= RL(0.0));
}

// One rayColor level after the closest hit (Ray.hs:176-224): background on a miss, else the
// material of the surface / medium hit.  Updates L, T and, when the path continues, the ray
// (and seg).  Returns true when the path terminates.
// kMats: the scene has materials beyond lightSource / pitchBlack / lambertian; their code is
// compiled only into those instantiations (the Cornell box and the bunny have none: -2.4 % / -1.2 %)
template <int kTex, bool kMats, bool kInst>
RT_FN bool shade_event(const KernelParams& P, cfp prims, uint32_t pix, int sample, int seg, real tbest, int best,
                       int hit_medium, const RayCtx& R, f3& L, const f3& T, int best_inst, f3& np, f3& nd, f3& Tf,
                       int& ngid) {
  RT_HOOK_SEGMENT(pix, sample, seg, R, tbest, best, hit_medium, L, T);
  if (hit_medium < 0 && best < 0) {
    // miss: cs_background (Ray.hs:179)
    f3 bg = ld3(P.cam.bg0);
    if (P.cam.bg_kind == 1) {
      real a = RL(0.5) * (R.d.y + RL(1.0));
      bg = (RL(1.0) - a) * bg + a * ld3(P.cam.bg1);
    }
    L = L + T * bg;
#ifndef RT_HOST_EMU
    Tf = bg;  // (defined, in a register already; the path ends)
#endif
    return true;
  }
  bool terminate = false;
  // the material: one record load (DevMaterial, per primitive for surfaces)
  const RT_CAS DevMaterial* Mp = hit_medium >= 0
                                     ? (const RT_CAS DevMaterial*)P.mats + P.media[hit_medium].material
                                     : (const RT_CAS DevMaterial*)P.prim_shade + best;
  if constexpr (kInst) {  // a placement's own material (the outermost `<$`) overrides its leaves'
    if (hit_medium < 0 && best_inst >= 0) {
      const int im = inst_rec(P, best_inst)->material;
      if (im >= 0) Mp = (const RT_CAS DevMaterial*)P.mats + im;
    }
  }
  const DevMaterial Mt = DevMaterial{Mp->kind, Mp->tex, Mp->param, Mp->tex_const, {RL(0.), RL(0.), RL(0.)}, RL(0.)};
  // every material but pitchBlack and dielectric reads its texture; constant textures come with
  // the record, the others are evaluated once (one inlined copy keeps the register allocation down)
  // (kTex: 0 — every texture is constant, the texture code is not compiled in; 1 — uv / image
  // textures; 2 — noise / marble textures too)
  const bool need_tex = kTex > 0 && !Mt.tex_const && Mt.kind != RT_MAT_PITCH_BLACK && Mt.kind != RT_MAT_DIELECTRIC;
  HitInfo h;
  if (hit_medium >= 0) {
    h.p = R.o + tbest * R.d;
    h.n = -R.d;
    h.front = true;
    h.u = RL(0.);
    h.v = RL(0.);
    h.gid = -1;
  } else {
    if constexpr (kInst) {
      if (best_inst >= 0) {  // hit information in object space, point and normal back to world
        const RT_CAS DevInstance* I = inst_rec(P, best_inst);
        RayCtx Ro = R;
        Ro.o = inst_to_object(I, R.o, true);
        Ro.d = inst_to_object(I, R.d, false);
        h = surface_info(P, prims, best, Ro, tbest, need_tex);
        h.p = R.o + tbest * R.d;
        h.n = inst_rotate(I, h.n);
      } else {
        h = surface_info(P, prims, best, R, tbest, need_tex);
      }
    } else {
      h = surface_info(P, prims, best, R, tbest, need_tex);
    }
  }
  f3 tex = f3{Mp->c0[0], Mp->c0[1], Mp->c0[2]};
  if (need_tex) tex = eval_texture<kTex == 2>(P, Mt.tex, h.u, h.v, h.p);
  u4 w = philox(pix, (uint32_t)sample, (uint32_t)seg, RT_EV_SCATTER, P.key0, P.key1);
#ifdef RT_HOST_EMU
  f3 newdir = mk3(RT_NAN, RT_NAN, RT_NAN);  // poison on the CPU: read only where the path goes on
#elif defined(RT_SHADE_UNDEF)
  f3 newdir;  // (experiment builds only: left unset on the terminating paths, as in round 5)
#else
  // defined on every path (read only where the path goes on): the incoming direction on the
  // terminating ones, a value already in registers, so the join needs no copies
  f3 newdir = R.d;
  Tf = tex;
#endif
  if constexpr (!kMats) {
    // lightSource / pitchBlack / lambertian only (the Cornell box, the bunny): every hit lane runs
    // the lambertian scatter, the light and black lanes too, which then end the path (Absorb,
    // Material.hs:41-47) and never read it.  In a wave the scatter runs whenever any lane is
    // diffuse, so their lanes cost nothing extra, and the direction and weight come out defined
    // on every path without a terminating branch of their own
    if (Mt.kind == 0) L = L + T * tex;  // lightSource: emit
    terminate = !mixture_scatter<false, false>(P, h, R, w, Mt, true, tex, newdir, Tf) || Mt.kind < 2;
  } else {
    switch (Mt.kind) {
      case 0:  // lightSource: emit, Absorb
        L = L + T * tex;
        terminate = true;
        break;
      case 1:  // pitchBlack
        terminate = true;
        break;
      case 4:  // mirror
        Tf = tex;
        newdir = unit(reflect(h.n, R.d));
        break;
      case 5: {  // metal
        f3 d2 = reflect(h.n, R.d) + Mt.param * unit_vector(w.y, w.z);
        if (dot(d2, h.n) > RL(0.0)) {
          Tf = tex;
          newdir = normalize(d2);
        } else {
          terminate = true;
        }
        break;
      }
      case 6: {  // dielectric
        Tf = mk3(RL(1.), RL(1.), RL(1.));
        real ior = Mt.param;
        real ratio = h.front ? RT_RCP(ior) : ior;
        real cos_t = RMIN(RL(1.0), -dot(h.n, R.d));
        real sin_t = RT_SQRT(RMAX(RL(0.0), RL(1.0) - cos_t * cos_t));
        real r0 = (RL(1.0) - ratio) * RT_RCP(RL(1.0) + ratio);
        r0 = r0 * r0;
        real x1 = RL(1.0) - cos_t, x2 = x1 * x1;
        real reflectance = r0 + (RL(1.0) - r0) * (x2 * x2 * x1);
        if (ratio * sin_t > RL(1.0) || u01(w.x) < reflectance) {
          newdir = unit(reflect(h.n, R.d));
        } else {
          f3 perp = ratio * (R.d + cos_t * h.n);
          newdir = unit(perp - RT_SQRT(RABS(RL(1.0) - dot(perp, perp))) * h.n);
        }
        break;
      }
      case 7:  // transparent
        Tf = tex;
        newdir = R.d;
        break;
      default:  // 2 lambertian, 3 lommelSeeliger (HemisphereF); 8 isotropic, 9 anisotropic (SphereF)
        terminate = !mixture_scatter<true, true>(P, h, R, w, Mt, Mt.kind == 2 || Mt.kind == 3, tex, newdir, Tf);
        break;
    }
  }
  np = h.p;
  nd = newdir;
  ngid = h.gid;
  return terminate;
}
// One rayColor level (shade_event) and the path's next segment.  The loop-carried ray and
// throughput are written unconditionally from shade_event's outputs: where the path goes on they
// are the next segment's; where it ends they are values of no meaning (defined in the GPU builds,
// NaN-poisoned in the host emulator) that camera_ray replaces (origin, direction, self ids) with a
// fresh throughput and segment count before anything reads them.  INVARIANT of the lane loops
// (lane_loop_lockstep, lane_loop_bvh): after shade returns true nothing reads R, T or the self ids
// before camera_ray (the emulator tests fail otherwise).  Keeping the unchanged ray on the
// terminating exits instead cost the flat binary64 kernel ~40 copies per lane-loop iteration
// (round 4).
template <int kTex, bool kMats, bool kInst = false>
RT_FN bool shade(const KernelParams& P, cfp prims, uint32_t pix, int sample, int& seg, real tbest, int best,
                 int hit_medium, RayCtx& R, f3& L, f3& T, int best_inst = -1) {
#ifdef RT_HOST_EMU
  // poison on the CPU: a path that ends leaves R, T and the self ids undefined (NaN / an id no leaf
  // has) until camera_ray restarts it, so an emulator test fails if anything reads them in between
  const real nan = RT_NAN;
  f3 np = mk3(nan, nan, nan), nd = np, Tf = np;
  int ngid = RT_EMPTY_ROOT;
#elif defined(RT_SHADE_UNDEF)
  f3 np, nd, Tf;  // (experiment builds only: the round-5 code, unset on the terminating paths)
  int ngid;
#else
  // GPU builds: every output defined on every path, so no lane carries an uninitialised value
  // through the lane loop's divergent joins.  A miss keeps the incoming ray (and throughput
  // factor 1); shade_event's terminating paths set the hit point, the incoming direction and the
  // texture colour — values already in registers (constants here cost ~40 copies per iteration
  // of the flat binary64 loop, 3 % of the Cornell frame)
  f3 np = R.o, nd = R.d, Tf = mk3(RL(1.), RL(1.), RL(1.));
  int ngid = R.self_gid;
#endif
  const bool term =
      shade_event<kTex, kMats, kInst>(P, prims, pix, sample, seg, tbest, best, hit_medium, R, L, T, best_inst, np, nd, Tf, ngid);
  R.o = np;
  R.d = nd;
  T = T * Tf;
  R.self_gid = ngid;
  if constexpr (kInst) R.self_inst = hit_medium >= 0 ? -1 : best_inst;
  // rayColor (depth - 1) with depth - 1 <= 0 is zero: the path ends at the last depth (Ray.hs:176)
  const bool cont = !term && seg + 1 < P.cam.max_depth;
  ++seg;
  return !cont;
}

// Work item -> pixel / sample range.  Ids are pixel-major within each item size (rt_internal.h
// KernelParams): a pixel's chunks are consecutive ids, so a wave's pool of consecutive ids
// covers a few pixels and their sums can be aggregated in LDS before the commit atomics.
struct ItemCtx {
  // tile pixel (-1: no item yet); an item aggregated in an LDS slot carries its slot code in bits
  // 24-31 (the host aggregates only tiles below 2^24 pixels; rt_render_kernel.h WaveWork::tag)
  int tp;
  int sample, s_end;
  uint32_t pix;   // global pixel gy * width + px
  uint32_t pxgy;  // gy << 16 | px (rt_build.cpp limits images to 65535 x 65535)
};
// kTwoSizes: the item may be big (flat kernel only: the BVH kernels run one item size, rt_build.cpp
// rt_host_plan_work, so their register allocation does not carry the decode)
template <bool kTwoSizes>
RT_FN bool open_item(const KernelParams& P, int item, ItemCtx& I) {
  const int W = P.cam.width;
  // item, tile pixel and row are non-negative: exact multiply-shift division by the launch
  // constants instead of the ~20-instruction signed integer division sequences
  const bool big = kTwoSizes && item < P.big_items;
  const int id = kTwoSizes && !big ? item - P.big_items : item;
  const int n = big ? P.n_big_chunks : P.n_chunks;
  I.tp = (int)fast_div((uint32_t)id, big ? P.div_big : P.div_small);
  const int k = id - I.tp * n;
  const int tr = (int)fast_div((uint32_t)I.tp, P.div_width);
  const int px = I.tp - tr * W;
  const int tb = (int)fast_div((uint32_t)tr, P.div_block);
  const int gy = (tb * P.n_shards + P.shard) * P.row_block + (tr - tb * P.row_block);
  I.pix = (uint32_t)(gy * W + px);
  I.pxgy = (uint32_t)gy << 16 | (uint32_t)px;
  // big chunk k: samples [k big_chunk, (k + 1) big_chunk); small chunk k: from small_start + k chunk
  const int chunk = big ? P.big_chunk : P.chunk;
  I.sample = (big || !kTwoSizes ? 0 : P.small_start) + k * chunk;
  I.s_end = I.sample + chunk < P.cam.spp ? I.sample + chunk : P.cam.spp;
  if (gy >= P.cam.height || P.cam.max_depth <= 0) I.s_end = I.sample;  // padding row / black image
  return I.sample < I.s_end;
}

// Sample stealing once the queue is drained (flat lane loop; RT_TAIL_STEAL).  A lane that finds no
// item left takes the last pending sample of a lane of its wave that still holds two or more (the
// one in flight and at least one more): the victim's item ends one sample earlier, the thief
// renders that sample as an item of its own — same pixel, same sample index, so the same Philox
// draws — and commits it directly (`tp_plain`: the tile pixel without the victim's aggregation
// slot code, whose open-id count belongs to the victim's commit).  Integer sums commute: the image
// is bit-identical.  Without it the frame ends on the waves whose lanes still hold up to three
// samples each (a lane's item of the queue's tail) while their other lanes idle.  Wave-uniform
// call; one pair per loop step, scalar (readlane) moves.
#ifndef RT_TAIL_STEAL
#define RT_TAIL_STEAL 1
#endif
#ifndef RT_TAIL_STEAL_BVH  // (the same in the decoupled BVH lane loop)
#define RT_TAIL_STEAL_BVH 1
#endif
#if (RT_TAIL_STEAL || RT_TAIL_STEAL_BVH) && !defined(RT_HOST_EMU)
RT_FN bool steal_sample(bool thief, ItemCtx& I, int tp_plain) {
  unsigned long long tm = __ballot(thief);
  unsigned long long vm = __ballot(!thief && I.tp != -1 && I.s_end - I.sample >= 2);
  const int lane = (int)__lane_id();
  bool got = false;
  while (tm != 0ull && vm != 0ull) {
    const int t = __ffsll(tm) - 1, v = __ffsll(vm) - 1;
    tm &= tm - 1ull;
    vm &= vm - 1ull;
    const int s_end = __builtin_amdgcn_readlane(I.s_end, v);
    const int tp = __builtin_amdgcn_readlane(tp_plain, v);
    const uint32_t pix = (uint32_t)__builtin_amdgcn_readlane((int)I.pix, v);
    const uint32_t pxgy = (uint32_t)__builtin_amdgcn_readlane((int)I.pxgy, v);
    if (lane == t) {
      I.tp = tp;
      I.sample = s_end - 1;
      I.s_end = s_end;
      I.pix = pix;
      I.pxgy = pxgy;
      got = true;
    }
    if (lane == v) I.s_end = s_end - 1;
  }
  return got;
}
#endif

// The lockstep persistent lane loop.  `work.grab(need, slot)` is wave-collective: it
// returns a fresh item for lanes with need == true (and its aggregation slot); `work.commit(c,
// tile_pixel, acc, bad)`, also wave-collective, adds the finished items' sums of lanes with
// c == true.  One segment per iteration, all of its queries run by the whole wave together: the flat
// kernel (every lane tests the same primitives), and the lockstep BVH variant kept for
// experiments (RT_VAR_BVH_LOCKSTEP; BVH scenes, media or not, default to lane_loop_bvh).
template <bool kFlat, int kTex, bool kMedia, bool kMats, class Work, class AccT>
RT_FN int lane_loop_lockstep(const KernelParams& P0, Work& work, const Trav& TW, const real* prims_, AccT& acc) {
  const cfp prims = cf(prims_);
  int overflow = 0;
  ItemCtx I{-1, 0, 0, 0u, 0u};
  int seg = 0;
  acc_clear(acc);
  bool bad = false;
  bool alive = false;
  // T: the path throughput.  No radiance register across iterations (as lane_loop_bvh): only the
  // event that ends a path emits, so a sample's radiance is that one term, summed at once.
  f3 T = mk3(RL(1.), RL(1.), RL(1.));
  RayCtx R;
  R.o = R.d = mk3(RL(0.), RL(0.), RL(0.));
#if RT_NODE_F32
  R.idir = R.off0 = R.off1 = f3n{0.f, 0.f, 0.f};
#else
  R.idir = R.oidir = R.o;
#endif
  R.time_w = 0u;
  R.self_gid = -1;
  R.self_inst = -1;
  RT_PROF_DECL
  for (;;) {
    const KernelParams& P = RT_KARGS(P0);  // (per iteration: RT_KARGS)
    const bool need = !alive && I.sample >= I.s_end;
    RT_PROF_ADD(PF_ITERS, 1);
    RT_PROF_ADD(PF_FRONT_LANES, RT_BALLOT_COUNT(need));
    work.commit(need && I.tp != -1, I.tp, acc, bad);
    int aslot;
    const int got = work.grab(need, aslot);
#if RT_TAIL_STEAL && !defined(RT_HOST_EMU)
    bool stolen = false;
    if constexpr (kFlat) {
      const bool thief = need && got >= P.n_items;
      if (RT_ANY(thief)) stolen = steal_sample(thief, I, work.untag(I.tp));
    }
#else
    const bool stolen = false;
#endif
    if (need) {
      if (got >= P.n_items && !stolen) break;
      acc_clear(acc);
      bad = false;
      if (!stolen) {
        const bool ok = open_item<kFlat>(P, got, I);
        I.tp = work.tag(I.tp, aslot);
        if (!ok) continue;
      }
    }
    RT_PROF_MARK(PF_FRONT);
    RT_PROF_ADD(PF_CAM_LANES, RT_BALLOT_COUNT(!alive));
    if (!alive) {
      camera_ray(P, I.pix, I.sample, I.pxgy, R);
      T = mk3(RL(1.), RL(1.), RL(1.));
      seg = 0;
      alive = true;
    }
    RT_PROF_MARK(PF_CAM);
    RT_COUNT(2);
    // ---- closest hit over the surfaces and every medium (Ray.hs:178)
    if constexpr (!kFlat) prep_ray(R);  // reciprocal direction: BVH slab tests only
    Closest C = no_hit();
    closest<kFlat>(P, prims, P.surface_root, 0, R, kTmin, C, TW, &overflow);
    real tbest = C.t;
    const int best = C.prim;
    int hit_medium = -1;
    // media: compiled only into the instantiations for scenes that have them (kMedia)
    const int n_media = kMedia ? P.n_media : 0;
    for (int m = 0; m < n_media; ++m) {
      // constantMedium (Geometry.hs:306-328)
      const DevMedium& M = P.media[m];
      Closest C1 = no_hit();
      if (M.alias_surface) {  // the boundary is the surface set: its first hit is the surface hit
        C1.t = C.t;
        C1.prim = C.prim;
      } else {
        closest<kFlat>(P, prims, M.root, m + 1, R, kTmin, C1, TW, &overflow);
      }
      if (C1.prim < 0) continue;
      const real t1 = C1.t;
      real lo, hi;
      if (prim_front(P, prims, C1.prim, R, t1)) {
        if (!(t1 < tbest)) continue;
        Closest C2 = no_hit();
        closest<kFlat>(P, prims, M.root, m + 1, R, t1, C2, TW, &overflow);
        if (C2.prim < 0) continue;
        lo = t1;
        hi = C2.t;
      } else {
        lo = kTmin;
        hi = t1;
      }
      medium_event(P, m, I.pix, I.sample, seg, lo, hi, tbest, hit_medium);
    }
    RT_PROF_MARK(PF_TRAV);
    f3 L = mk3(RL(0.), RL(0.), RL(0.));
    if (shade<kTex, kMats>(P, prims, I.pix, I.sample, seg, tbest, best, hit_medium, R, L, T)) {
      // the path ended: R and T are indeterminate until camera_ray (shade's invariant)
      RT_HOOK_SAMPLE(I.pix, I.sample, L);
      acc_sample(acc, L, bad);
      alive = false;
      ++I.sample;
    }
    RT_PROF_MARK(PF_SHADE);
  }
  RT_PROF_FLUSH
  return overflow;
}

// The segment's media events after its surface query, with the lanes that shade (KernelParams::
// media_late: every medium's boundary is the surface set or a single leaf, whose records are the
// same for every lane), instead of a query chain inside the traversal loop run by the few lanes
// whose query just ended.  Same queries, same draws, same order as the chain (Geometry.hs:306-328):
// per medium its first boundary hit on (tmin, inf) and, for a ray entering it before the closest
// hit so far, the second; the images are bit-identical (RT_AMD_MEDIA_LATE=0 runs the chain).
// A kernel has one of the two compiled in (kMedia 2 / 1, rt_render_kernel.h): the chain's state
// (query index, entry distance, the surface hit kept apart) and its code cost the pawn+fog
// binary64 kernel ~40 VGPRs over the bunny's, which held it at 3 waves per SIMD.
template <bool kInst>
RT_FN void media_events_late(const KernelParams& P, cfp prims, const RayCtx& R, uint32_t pix, int sample, int seg, int best,
                             real t_surf, real& tbest, int& hit_medium) {
  for (int m = 0; m < P.n_media; ++m) {
    const DevMedium& M = P.media[m];
    // the event's interval (lo, hi), if any; one draw site (one inlined copy of Philox and log)
    bool ev = false;
    real lo = kTmin, hi = t_surf;
    if (M.alias_surface) {  // the surface hit is the boundary's first hit (DevMedium)
      ev = best >= 0 && !prim_front(P, prims, best, R, t_surf);
    } else {
      // a single leaf: its records from the kernel arguments' root, the same for every lane
      // (scalar loads, as the surface prefix's), by the generic test
      const int enc = ~M.root;
      const int first = enc >> RT_LEAF_SHIFT, end = first + (enc & ((1 << RT_LEAF_SHIFT) - 1)) + 1;
      Closest C1 = no_hit();
      for (int k = first; k < end; ++k)
        test_rec<false, kInst>(P, ld_rec64((const RT_CAS PrimRec64*)prims + k), k, R, kTmin, float_up(kTmin), C1);
      if (C1.prim >= 0) {
        const real t1 = C1.t;
        if (prim_front(P, prims, C1.prim, R, t1)) {
          if (t1 < tbest) {  // entering: the exit hit bounds the segment
            Closest C2 = no_hit();
            for (int k = first; k < end; ++k)
              test_rec<false, kInst>(P, ld_rec64((const RT_CAS PrimRec64*)prims + k), k, R, t1, float_up(t1), C2);
            ev = C2.prim >= 0;
            lo = t1;
            hi = C2.t;
          }
        } else {
          ev = true;
          hi = t1;
        }
      }
    }
    if (ev) medium_event(P, m, pix, sample, seg, lo, hi, tbest, hit_medium);
  }
}

// The persistent lane loop of the BVH kernel, with traversal decoupled from shading inside the
// wave.  Incoherent secondary rays need very different numbers of traversal rounds; if every
// lane waited for the wave's slowest traversal before shading, most lanes would idle (measured
// ~21 % lane utilisation).  Here a lane is in one of the states below; the wave runs traversal
// rounds for the TRACE lanes until at most P.trav_exit_pct % of the loop's live lanes still
// trace, then lets the others shade and start their next ray, and goes back to traversal with
// the stragglers keeping their traversal state (stack in LDS).  A segment's queries run in the
// reference's order — the surfaces, then per medium its first boundary hit and, for a ray
// entering it, the second (Geometry.hs:306-328) — each starting inside the traversal loop as
// soon as the previous one finishes.
enum : int { ST_NEED_ITEM = 0, ST_NEED_SAMPLE = 1, ST_START_SEG = 2, ST_TRACE = 3, ST_SHADE = 4 };
// kMedia: 0 no media; 1 the media queries chained in the traversal loop; 2 the media events in
// the shading phase (media_events_late)
template <int kTex, int kMedia, bool kMats, bool kInst, int kLeaf, class Work, class AccT>
RT_FN int lane_loop_bvh(const KernelParams& P0, Work& work, const Trav& TW, const real* prims_, AccT& acc) {
  const cfp prims = cf(prims_);
  const int n_media = kMedia == 1 ? P0.n_media : 0;  // the chain only in its instantiations
  int overflow = 0;
  ItemCtx I{-1, 0, 0, 0u, 0u};
  int seg = 0;
  acc_clear(acc);
  bool bad = false;
  int state = ST_NEED_ITEM;
  // T: the path throughput.  The radiance needs no register across iterations: only the event
  // that ends a path emits (lightSource absorbs, Material.hs:41-44; a miss returns the background,
  // Ray.hs:179), so a sample's radiance is that one term, formed in `shade` and summed at once.
  f3 T = mk3(RL(1.), RL(1.), RL(1.));
  RayCtx R;
  R.o = R.d = mk3(RL(0.), RL(0.), RL(0.));
#if RT_NODE_F32
  R.idir = R.off0 = R.off1 = f3n{0.f, 0.f, 0.f};
#else
  R.idir = R.oidir = R.o;
#endif
  R.time_w = 0u;
  R.self_gid = -1;
  R.self_inst = -1;
  TravState S;
  trav_begin(S, RT_EMPTY_ROOT, kTmin);
  // query sequencing within a segment (the chain, kMedia 1): q = 0 surfaces; q = 1 + 2m / 2 + 2m
  // medium m, 1st / 2nd hit.  Without the chain the surface query's S.C holds the closest hit
  // until the shading phase: no loop-carried copies (kMedia 2: the media events take a local one)
  constexpr bool kChain = kMedia == 1;
  int q = 0, best = -1, hit_medium = -1, best_inst = -1;
  real tbest = kInf, t1 = RL(0.0), t_surf = kInf;
  RT_PROF_DECL
  for (;;) {
    const KernelParams& P = RT_KARGS(P0);  // (per phase: RT_KARGS)
    // ---- front end: items, samples, segment starts (lanes not tracing)
    const bool need = state == ST_NEED_ITEM;
    RT_PROF_ADD(PF_ITERS, 1);
    RT_PROF_ADD(PF_FRONT_LANES, RT_BALLOT_COUNT(state != ST_TRACE));
    work.commit(need && I.tp != -1, I.tp, acc, bad);
    int aslot;
    const int got = work.grab(need, aslot);
#if RT_TAIL_STEAL_BVH && !defined(RT_HOST_EMU)
    bool stolen = false;
    {
      const bool thief = need && got >= P.n_items;
      if (RT_ANY(thief)) stolen = steal_sample(thief, I, work.untag(I.tp));
    }
#else
    const bool stolen = false;
#endif
    if (need) {
      if (got >= P.n_items && !stolen) break;
      acc_clear(acc);
      bad = false;
      if (stolen) {
        state = ST_NEED_SAMPLE;
      } else {
        state = open_item<false>(P, got, I) ? ST_NEED_SAMPLE : ST_NEED_ITEM;
        I.tp = work.tag(I.tp, aslot);
      }
    }
    if (state == ST_NEED_SAMPLE) {
      camera_ray(P, I.pix, I.sample, ~0u, R);
      T = mk3(RL(1.), RL(1.), RL(1.));
      seg = 0;
      state = ST_START_SEG;
    }
    if (state == ST_START_SEG) {
      RT_COUNT(2);
      prep_ray(R);
      q = 0;
      best = -1;
      best_inst = -1;
      hit_medium = -1;
      tbest = kInf;
      trav_begin(S, P.surface_root, kTmin);
      prefix_hits<kInst>(P, prims, R, kTmin, S.C);
      state = ST_TRACE;
    }
    RT_PROF_MARK(PF_FRONT);
    // ---- traversal rounds; a finished query starts the segment's next one in place
    for (;;) {
      const KernelParams& P = RT_KARGS_IF(RT_KARGS_TRAV, P0);
      const bool tr = state == ST_TRACE;
      const int n_tr = RT_BALLOT_COUNT(tr);
      if (n_tr == 0) break;
      const int n_live = RT_BALLOT_COUNT(true);
      if (n_tr < n_live && n_tr * 100 <= n_live * P.trav_exit_pct) break;
      RT_PROF_ADD(PF_ROUNDS, 1);
      RT_PROF_ADD(PF_TRACING, n_tr);
      RT_PROF_ADD(PF_LIVE, n_live);
      if (tr) {
        trav_round<kInst, kLeaf>(P, R, S, TW, overflow RT_PROF_ARG);
        while (trav_done(S)) {
          int next_m = -1;  // medium whose first query starts next
          if (!kChain || q == 0) {
            if constexpr (kChain) {
              tbest = t_surf = S.C.t;
              best = S.C.prim;
              best_inst = S.C.inst;
            }
            next_m = 0;
          } else {
            const int m = (q - 1) >> 1;
            next_m = m + 1;
            if ((q & 1) == 1) {  // first boundary hit of medium m
              if (S.C.prim >= 0) {
                t1 = S.C.t;
                if (prim_front(P, prims, S.C.prim, R, t1)) {
                  if (t1 < tbest) {  // entering: the exit hit bounds the segment
                    q = q + 1;
                    trav_begin(S, P.media[m].root, t1);
                    next_m = -1;
                  }
                } else {
                  medium_event(P, m, I.pix, I.sample, seg, kTmin, t1, tbest, hit_medium);
                }
              }
            } else if (S.C.prim >= 0) {  // exit hit of medium m
              medium_event(P, m, I.pix, I.sample, seg, t1, S.C.t, tbest, hit_medium);
            }
          }
          // media whose boundary is the surface set reuse the surface hit (DevMedium)
          while (next_m >= 0 && next_m < n_media && P.media[next_m].alias_surface) {
            if (best >= 0 && !prim_front(P, prims, best, R, t_surf))
              medium_event(P, next_m, I.pix, I.sample, seg, kTmin, t_surf, tbest, hit_medium);
            ++next_m;
          }
          if (next_m >= 0) {
            if (next_m < n_media) {
              q = 1 + 2 * next_m;
              trav_begin(S, P.media[next_m].root, kTmin);
            } else {
              state = ST_SHADE;
            }
          }
          // a query over a set that is a single leaf (e.g. a fog sphere) is tested right away;
          // with one-class leaves by the generic test (the host checks only the classes of the
          // leaves below BVH nodes: a single-leaf medium set may be any class, rt_build.cpp)
          if (state != ST_TRACE || S.node != RT_EMPTY_ROOT) break;
          if constexpr (kLeaf != 0)
            test_leaf_generic<kInst>(P, R, S);
          else
            trav_round<kInst, kLeaf>(P, R, S, TW, overflow RT_PROF_ARG);
        }
      }
    }
    RT_PROF_MARK(PF_TRAV);
    RT_PROF_ADD(PF_SHADING, RT_BALLOT_COUNT(state == ST_SHADE));
    // ---- shade the segments whose queries are complete
    if (state == ST_SHADE) {
      const KernelParams& P = RT_KARGS(P0);
      if constexpr (!kChain) {
        tbest = S.C.t;
        best = S.C.prim;
        best_inst = S.C.inst;
        hit_medium = -1;
      }
      if constexpr (kMedia == 2)  // (tbest is the surface hit's distance until the media events)
        media_events_late<kInst>(P, prims, R, I.pix, I.sample, seg, best, tbest, tbest, hit_medium);
      f3 L = mk3(RL(0.), RL(0.), RL(0.));
      if (shade<kTex, kMats, kInst>(P, prims, I.pix, I.sample, seg, tbest, best, hit_medium, R, L, T, best_inst)) {
        // the path ended: R and T are indeterminate until camera_ray (shade's invariant)
        RT_HOOK_SAMPLE(I.pix, I.sample, L);
        acc_sample(acc, L, bad);
        ++I.sample;
        state = I.sample < I.s_end ? ST_NEED_SAMPLE : ST_NEED_ITEM;
      } else {
        state = ST_START_SEG;
      }
    }
    RT_PROF_MARK(PF_SHADE);
  }
  RT_PROF_FLUSH
  return overflow;
}

}  // namespace RT_NS
