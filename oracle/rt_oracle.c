/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement (IEEE binary64) of the
 * UnaryPlus/raytrace per-pixel radiance loop.  It is the parity checker for the HIP
 * product path and the `cpu_baseline` leg of bench.py; nothing in raytrace_amd/
 * links, imports or calls it.
 *
 * What it restates (all paths relative to the reference tree, v0.2.0.0):
 *   camera setup ............ src/Graphics/Ray.hs:122-155
 *   getRay / samplePixel .... src/Graphics/Ray.hs:157-172
 *   rayColor ................ src/Graphics/Ray.hs:174-224 (incl. redirect mixture pdf)
 *   pixelColor / seeds ...... src/Graphics/Ray.hs:226-238
 *   randomUnitVector, randomInUnitDisk, reflect, overlapsBox ... src/Graphics/Ray/Core.hs:49-68, 95-152
 *   sphere, sphereUV, planeShape, parallelogram, triangle ...... src/Graphics/Ray/Geometry.hs:58-176
 *   constantMedium, group, bvhNode, transform, moving .......... src/Graphics/Ray/Geometry.hs:298-456
 *   the ten materials ....... src/Graphics/Ray/Material.hs:41-129
 *   textures (constant, checker, image, noise, marble) src/Graphics/Ray/Texture.hs:18-78
 *   Perlin noise, fractal noise, turbulence ..... src/Graphics/Ray/Noise.hs:15-53
 *
 * The scene arrives as the reference's own geometry TREE (group / bvhNode / transform /
 * moving / constantMedium / `<$` nodes over sphere and planeShape leaves), serialized by
 * raytrace_amd.scene.serialize_tree(); the traversal below walks it in the reference's
 * order (group fold with shrinking tmax, bvhNode left-then-right with overlapsBox), so
 * tie-breaking and the order of random draws inside media follow the reference.
 *
 * Arithmetic follows GHC's evaluation of the Haskell expressions: left-associative sums,
 * no FMA contraction (build with -ffp-contract=off), libm transcendentals, GHC.Float's
 * default atan2, Haskell min/max semantics, banker's rounding for `round`.
 *
 * RNG modes:
 *   ORACLE_RNG_SPLITMIX — restates the reference's StdGen stream: splitmix SMGen
 *     (mkSMGen/nextWord64/splitSMGen/mixGamma), random-1.3 `random :: Double` = 1 - w/(2^64-1),
 *     `randomR (l,h)` = x*l + (1-x)*h, per-pixel generators from massiv's randomArrayS with
 *     splitGen in row-major order, and the reference's rejection samplers.  Third-party
 *     algorithms (splitmix >=0.1, random >=1.3 <1.4, linear >=1.23.2, massiv >=1.0.5) are
 *     absent from /root/reference; they are restated from their published definitions and
 *     pinned by reproducing the pixels of the reference's committed PNG renders
 *     (tests/test_oracle_golden.py).
 *   ORACLE_RNG_PHILOX — the counter-based stream the GPU kernel uses (Philox4x32-10 keyed by
 *     the 64-bit seed, counter = (pixel, sample, segment, event)) with direct (non-rejection)
 *     samplers of the same distributions.  GPU and oracle then consume identical random
 *     numbers, so renders can be compared per pixel.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_RNG_SPLITMIX 0
#define ORACLE_RNG_PHILOX 1

/* node kinds (must match raytrace_amd/scene.py) */
enum { N_SPHERE = 0, N_PLANE = 1, N_GROUP = 2, N_BVH = 3, N_TRANSFORM = 4, N_MOVING = 5, N_MEDIUM = 6, N_MATERIAL = 7 };
/* plane-shape test kinds */
enum { P_PARALLELOGRAM = 0, P_TRIANGLE = 1 };
/* material kinds (Material.hs:41-129) */
enum { M_LIGHT = 0, M_BLACK = 1, M_LAMBERT = 2, M_LOMMEL = 3, M_MIRROR = 4, M_METAL = 5, M_DIELECTRIC = 6,
       M_TRANSPARENT = 7, M_ISOTROPIC = 8, M_ANISOTROPIC = 9 };
/* texture kinds */
enum { T_CONSTANT = 0, T_CHECKER = 1, T_IMAGE = 2, T_NOISE = 3, T_MARBLE = 4 };
/* background kinds */
enum { BG_CONST = 0, BG_LERPY = 1 };

#define NI 4   /* ints per node  */
#define ND 30  /* doubles per node */
#define PI_HS 3.141592653589793

/* counters (algorithmic-bytes model) */
enum { C_SEGMENTS = 0, C_BVH_NODES, C_SPHERES, C_PLANES, C_TRANSFORMS, C_MEDIA, C_REDIRECT_EVALS,
       C_MATERIAL_HITS, C_SAMPLES, C_COUNT };

typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 smul(double s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }   /* s *^ v */
static inline v3 muls(v3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }   /* v ^* s */
static inline v3 divs(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }   /* v ^/ s */
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double quadrance(v3 a) { return dot(a, a); }
/* linear's normalize: leaves v unchanged when quadrance is nearZero or nearZero (1 - quadrance) */
static inline v3 normalize(v3 v) {
  double l = quadrance(v);
  if (fabs(l) <= 1e-12 || fabs(1 - l) <= 1e-12) return v;
  return divs(v, sqrt(l));
}
/* Haskell's default Ord max/min for Double */
static inline double hmax(double x, double y) { return x <= y ? y : x; }
static inline double hmin(double x, double y) { return x <= y ? x : y; }
/* GHC.Float default atan2 */
static double hs_atan2(double y, double x) {
  if (x > 0) return atan(y / x);
  if (x == 0 && y > 0) return PI_HS / 2;
  if (x < 0 && y > 0) return PI_HS + atan(y / x);
  if ((x <= 0 && y < 0) || (x < 0 && signbit(y) && y == 0) || (signbit(x) && x == 0 && signbit(y) && y == 0))
    return -hs_atan2(-y, x);
  if (y == 0 && (x < 0 || (signbit(x) && x == 0))) return PI_HS;
  if (x == 0 && y == 0) return y;
  return x + y;
}
/* Core.hs:49-51 */
static inline v3 reflect(v3 n, v3 v) { return sub(v, smul(2 * dot(n, v), n)); }

/* ------------------------------------------------------------------ RNG */
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdULL;
  z = (z ^ (z >> 33)) * 0xc4ceb9fe1a85ec53ULL;
  return z ^ (z >> 33);
}
static inline uint64_t mix64v13(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static inline uint64_t mix_gamma(uint64_t z) {
  uint64_t z1 = mix64v13(z) | 1ULL;
  int n = __builtin_popcountll(z1 ^ (z1 >> 1));
  return n >= 24 ? z1 : (z1 ^ 0xaaaaaaaaaaaaaaaaULL);
}
/* mkStdGen n = StdGen (mkSMGen (fromIntegral n)) */
void oracle_mkstdgen(int64_t n, uint64_t* seed, uint64_t* gamma) {
  uint64_t s = (uint64_t)n;
  *seed = mix64(s);
  *gamma = mix_gamma(s + 0x9e3779b97f4a7c15ULL);
}
/* splitSMGen: (SMGen seed'' gamma, SMGen (mix64 seed') (mixGamma seed'')) */
static inline void split_smgen(uint64_t s, uint64_t g, uint64_t* s1, uint64_t* g1, uint64_t* s2, uint64_t* g2) {
  uint64_t sp = s + g, spp = sp + g;
  *s1 = spp; *g1 = g;
  *s2 = mix64(sp); *g2 = mix_gamma(spp);
}
void oracle_split(uint64_t s, uint64_t g, uint64_t* out4) { split_smgen(s, g, &out4[0], &out4[1], &out4[2], &out4[3]); }

static inline void philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; r++) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
void oracle_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { philox4x32_10(ctr, key, out); }

/* [0,1) with 24 bits — identical to the device's u01() */
static inline double u01(uint32_t w) { return (double)(w >> 8) * (1.0 / 16777216.0); }

/* Philox events (must match raytrace_amd/csrc/rt_kernel.hip) */
enum { EV_CAMERA0 = 0, EV_CAMERA1 = 1, EV_SCATTER = 2, EV_MEDIA = 3 };

typedef struct {
  int mode;
  /* splitmix state */
  uint64_t seed, gamma;
  /* philox */
  uint32_t key[2];
  uint32_t pix, sample;
  int variant; /* splitmix randomR variant: 0 = x*l + (1-x)*h (random-1.2/1.3), 1 = l + x*(h-l) */
} rng_t;

static inline uint64_t next_word(rng_t* r) { r->seed += r->gamma; return mix64(r->seed); }
/* uniformDouble01M: fromIntegral w64 / fromIntegral (maxBound :: Word64) */
static inline double uniform01(rng_t* r) {
  if (r->variant & 8) return (double)(next_word(r) >> 11) * (1.0 / 9007199254740992.0);
  return (double)next_word(r) / 18446744073709551615.0;
}
/* random :: Double (random >= 1.2): 1 - uniformDouble01M */
static inline double hs_random(rng_t* r) { return (r->variant & 2) ? uniform01(r) : 1 - uniform01(r); }
/* randomR (l, h) :: Double */
static inline double hs_randomR(rng_t* r, double l, double h) {
  if (l == h) return l;
  double x = uniform01(r);
  if (r->variant & 1) return l + x * (h - l);
  return x * l + (1 - x) * h;
}
static inline void philox_event(const rng_t* r, uint32_t segment, uint32_t event, uint32_t out[4]) {
  uint32_t ctr[4] = {r->pix, r->sample, segment, event};
  philox4x32_10(ctr, r->key, out);
}
/* direct samplers shared with the GPU */
static inline v3 unit_vector_direct(double u1, double u2) {
  double z = 1 - 2 * u1;
  double rr = sqrt(fmax(0.0, 1 - z * z));
  double phi = 2 * PI_HS * u2;
  return mk(rr * cos(phi), rr * sin(phi), z);
}
/* Core.hs:54-60 randomUnitVector (rejection) */
static v3 random_unit_vector_sm(rng_t* r) {
  for (;;) {
    double x = hs_randomR(r, -1, 1), y = hs_randomR(r, -1, 1), z = hs_randomR(r, -1, 1);
    v3 v = mk(x, y, z);
    double q = quadrance(v);
    if (1e-8 <= q && q <= 1) return divs(v, sqrt(q));
  }
}

/* Noise.hs:94-98 gradients = evalState (replicateM 256 randomUnitVector) (mkStdGen 666):
   the oracle's own restatement, used by the tests to check the product's table. */
void oracle_perlin_gradients(double* out /* 256 x 3 */) {
  rng_t r;
  memset(&r, 0, sizeof r);
  r.mode = ORACLE_RNG_SPLITMIX;
  oracle_mkstdgen(666, &r.seed, &r.gamma);
  for (int k = 0; k < 256; ++k) {
    v3 g = random_unit_vector_sm(&r);
    out[3 * k] = g.x;
    out[3 * k + 1] = g.y;
    out[3 * k + 2] = g.z;
  }
}

/* ------------------------------------------------------------------ scene */
typedef struct {
  double p, remprob_unused;
  v3 q, u, v, cr;
  double thresh;
  /* parallelogram precompute for rt_hit */
  v3 normal, normalS;
} target_t;

typedef struct {
  const int32_t* ni;
  const double* nd;
  const int32_t* children;
  const int32_t* mi;
  const double* md;
  const int32_t* ti;
  const double* td;
  const float* texels;      /* image textures: 3 floats per texel */
  const int32_t* perm;      /* Perlin permX / permY / permZ, 3 x 256 */
  const double* grad;       /* Perlin gradients, 256 x 3 */
  int root;
  /* camera */
  int width, height, spp, max_depth, bg_kind;
  v3 center, top_left, pixel_u, pixel_v, disk_u, disk_v, bg0, bg1;
  int nt;
  target_t* targets;
  double rem_prob;
  int rng_mode, variant;
  uint64_t seed, gamma;   /* splitmix StdGen for `raytrace`'s seed argument */
  uint32_t key[2];
  /* splitmix per-pixel generators (computed for pixel indices up to max requested) */
  uint64_t* pix_seed;
  uint64_t* pix_gamma;
} scene_t;

typedef struct {
  int valid;
  double t;
  v3 p, n;
  int front;
  double u, v;
  int mat;
} hit_t;

typedef struct {
  v3 o, d;
} ray_t;

static inline const int32_t* NIp(const scene_t* s, int i) { return s->ni + (size_t)i * NI; }
static inline const double* NDp(const scene_t* s, int i) { return s->nd + (size_t)i * ND; }

typedef struct {
  rng_t* rng;
  uint32_t segment;
  double* cnt;
} tctx_t;

static int hit_node(const scene_t* s, tctx_t* tc, int idx, double time, ray_t ray, double tmin, double tmax, hit_t* out);

/* Core.hs:95-106, 147-152 */
static inline int isect(double a, double b, double c, double d, double* lo, double* hi) {
  double imin = hmax(a, c), imax = hmin(b, d);
  if (imin > imax) return 0;
  *lo = imin; *hi = imax;
  return 1;
}
static inline void overlaps_interval(double lo, double hi, double x, double d, double* a, double* b) {
  double t0 = (lo - x) / d, t1 = (hi - x) / d;
  if (t0 < t1) { *a = t0; *b = t1; } else { *a = t1; *b = t0; }
}
static int overlaps_box(const double* box, ray_t r, double tmin, double tmax) {
  double a, b, lo, hi;
  overlaps_interval(box[0], box[1], r.o.x, r.d.x, &a, &b);
  if (!isect(tmin, tmax, a, b, &lo, &hi)) return 0;
  tmin = lo; tmax = hi;
  overlaps_interval(box[2], box[3], r.o.y, r.d.y, &a, &b);
  if (!isect(tmin, tmax, a, b, &lo, &hi)) return 0;
  tmin = lo; tmax = hi;
  overlaps_interval(box[4], box[5], r.o.z, r.d.z, &a, &b);
  return isect(tmin, tmax, a, b, &lo, &hi);
}

/* Geometry.hs:100-104 */
static inline void sphere_uv(v3 n, double* u, double* v) {
  *u = hs_atan2(n.x, n.z) / (2 * PI_HS) + 0.5;
  *v = acos(-n.y) / PI_HS;
}

/* Geometry.hs:58-94 */
static int hit_sphere(const double* p, ray_t r, double tmin, double tmax, hit_t* h) {
  v3 center = mk(p[0], p[1], p[2]);
  double radius = p[3];
  v3 oc = sub(center, r.o);
  double hh = dot(r.d, oc);
  double c = quadrance(oc) - radius * radius;
  double disc = hh * hh - c;
  if (!(disc >= 0)) return 0;
  double sq = sqrt(disc);
  double r1 = hh - sq, r2 = hh + sq, t;
  if (tmin < r1 && r1 < tmax) t = r1;
  else if (tmin < r2 && r2 < tmax) t = r2;
  else return 0;
  v3 point = add(r.o, smul(t, r.d));
  v3 outward = divs(sub(point, center), radius);
  int front = dot(r.d, outward) <= 0;
  h->valid = 1; h->t = t; h->p = point; h->n = front ? outward : neg(outward); h->front = front;
  sphere_uv(outward, &h->u, &h->v);
  return 1;
}

/* Geometry.hs:108-176.  p: q[0:3] u[3:6] v[6:9] uv0[9:11] uv1[11:13] uv2[13:15] */
static int hit_plane(const double* p, int kind, ray_t r, double tmin, double tmax, hit_t* h) {
  v3 q = mk(p[0], p[1], p[2]), u = mk(p[3], p[4], p[5]), v = mk(p[6], p[7], p[8]);
  v3 cp = cross(u, v);
  double norm_cp = sqrt(quadrance(cp));
  v3 normal = divs(cp, norm_cp);
  v3 normalS = divs(normal, norm_cp);
  double denom = dot(normal, r.d);
  if (!(fabs(denom) > 1e-8)) return 0;
  double t = dot(normal, sub(q, r.o)) / denom;
  if (!(tmin < t && t < tmax)) return 0;
  v3 pt = add(r.o, smul(t, r.d));
  v3 prel = sub(pt, q);
  double a = dot(normalS, cross(prel, v));
  double b = dot(normalS, cross(u, prel));
  double uu, vv;
  if (kind == P_PARALLELOGRAM) {
    if (!(0 <= a && a <= 1 && 0 <= b && b <= 1)) return 0;
    uu = a; vv = b;
  } else {
    if (!(a >= 0 && b >= 0 && a + b <= 1)) return 0;
    double w0 = 1 - a - b;
    uu = w0 * p[9] + a * p[11] + b * p[13];
    vv = w0 * p[10] + a * p[12] + b * p[14];
  }
  int front = denom < 0;
  h->valid = 1; h->t = t; h->p = pt; h->n = front ? normal : neg(normal); h->front = front;
  h->u = uu; h->v = vv;
  return 1;
}

/* 3x4 matrix (row-major) times V4 point / vector: linear's (!*) with V4 dot = ((ae+bf)+cg)+dh */
static inline v3 m34_point(const double* m, v3 p) {
  return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3] * 1.0,
            m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7] * 1.0,
            m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11] * 1.0);
}
static inline v3 m34_vector(const double* m, v3 p) {
  return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3] * 0.0,
            m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7] * 0.0,
            m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11] * 0.0);
}

static double draw_medium(const scene_t* s, tctx_t* tc, int medium_index) {
  rng_t* r = tc->rng;
  if (r->mode == ORACLE_RNG_SPLITMIX) return hs_random(r);
  uint32_t w[4];
  philox_event(r, tc->segment, EV_MEDIA + (uint32_t)(medium_index >> 2), w);
  (void)s;
  return 1.0 - u01(w[medium_index & 3]);
}

static int hit_node(const scene_t* s, tctx_t* tc, int idx, double time, ray_t ray, double tmin, double tmax, hit_t* out) {
  const int32_t* ni = NIp(s, idx);
  const double* nd = NDp(s, idx);
  switch (ni[0]) {
    case N_SPHERE:
      tc->cnt[C_SPHERES] += 1;
      if (hit_sphere(nd + 6, ray, tmin, tmax, out)) { out->mat = -1; return 1; }
      return 0;
    case N_PLANE:
      tc->cnt[C_PLANES] += 1;
      if (hit_plane(nd + 6, ni[1], ray, tmin, tmax, out)) { out->mat = -1; return 1; }
      return 0;
    case N_GROUP: { /* Geometry.hs:335-347 */
      double tcur = tmax;
      int found = 0;
      hit_t h;
      for (int k = 0; k < ni[2]; k++) {
        if (hit_node(s, tc, s->children[ni[1] + k], time, ray, tmin, tcur, &h)) {
          tcur = h.t; *out = h; found = 1;
        }
      }
      return found;
    }
    case N_BVH: { /* Geometry.hs:351-363 */
      tc->cnt[C_BVH_NODES] += 1;
      if (!overlaps_box(nd, ray, tmin, tmax)) return 0;
      hit_t hl, hr;
      if (!hit_node(s, tc, ni[1], time, ray, tmin, tmax, &hl)) return hit_node(s, tc, ni[2], time, ray, tmin, tmax, out);
      if (hit_node(s, tc, ni[2], time, ray, tmin, hl.t, &hr)) { *out = hr; return 1; }
      *out = hl;
      return 1;
    }
    case N_TRANSFORM: { /* Geometry.hs:382-391; nd[6:18] = m34, nd[18:30] = inv34 */
      tc->cnt[C_TRANSFORMS] += 1;
      const double* m = nd + 6;
      const double* inv = nd + 18;
      ray_t r2;
      r2.o = m34_point(inv, ray.o);
      r2.d = m34_vector(inv, ray.d);
      if (!hit_node(s, tc, ni[1], time, r2, tmin, tmax, out)) return 0;
      out->p = m34_point(m, out->p);
      out->n = m34_vector(m, out->n);
      return 1;
    }
    case N_MOVING: { /* Geometry.hs:449-456; nd[6:9] v0, nd[9:12] v1 */
      v3 v0 = mk(nd[6], nd[7], nd[8]), v1 = mk(nd[9], nd[10], nd[11]);
      v3 shift = add(smul(1 - time, v0), smul(time, v1));
      ray_t r2 = {sub(ray.o, shift), ray.d};
      if (!hit_node(s, tc, ni[1], time, r2, tmin, tmax, out)) return 0;
      out->p = add(out->p, shift);
      return 1;
    }
    case N_MEDIUM: { /* Geometry.hs:298-330; nd[6] density, ni[2] medium index */
      tc->cnt[C_MEDIA] += 1;
      hit_t h1, h2;
      double t1, t2;
      if (!hit_node(s, tc, ni[1], time, ray, tmin, INFINITY, &h1)) return 0;
      if (h1.front) {
        if (!(h1.t < tmax)) return 0;
        if (!hit_node(s, tc, ni[1], time, ray, h1.t, INFINITY, &h2)) return 0;
        t1 = h1.t; t2 = hmin(tmax, h2.t);
      } else {
        t1 = tmin; t2 = hmin(tmax, h1.t);
      }
      double rnd = draw_medium(s, tc, ni[2]);
      double neg_inv_density = -(1 / nd[6]);
      double in_dist = t2 - t1;
      double hit_dist = neg_inv_density * log(rnd);
      if (!(hit_dist < in_dist)) return 0;
      double t = t1 + hit_dist;
      out->valid = 1; out->t = t; out->p = add(ray.o, smul(t, ray.d)); out->n = neg(ray.d);
      out->front = 1; out->u = 0; out->v = 0; out->mat = -1;
      return 1;
    }
    case N_MATERIAL:
      if (!hit_node(s, tc, ni[1], time, ray, tmin, tmax, out)) return 0;
      out->mat = ni[2];
      return 1;
  }
  return 0;
}

/* Noise.hs:15-16 smoothstep */
static double smoothstep_hs(double x) { return x * x * (3 - 2 * x); }

/* Noise.hs:21-45 perlinNoise: the list comprehension over i, j, k in {0, 1}, summed left to right */
static double perlin_noise(const scene_t* s, v3 p) {
  long ix = (long)floor(p.x), iy = (long)floor(p.y), iz = (long)floor(p.z);
  double fx = p.x - (double)ix, fy = p.y - (double)iy, fz = p.z - (double)iz;
  double sum = 0;
  for (int i = 0; i <= 1; ++i)
    for (int j = 0; j <= 1; ++j)
      for (int k = 0; k <= 1; ++k) {
        double di = i, dj = j, dk = k;
        int g = s->perm[(ix + i) & 255] ^ s->perm[256 + ((iy + j) & 255)] ^ s->perm[512 + ((iz + k) & 255)];
        v3 grad = mk(s->grad[3 * g], s->grad[3 * g + 1], s->grad[3 * g + 2]);
        v3 rel = mk(fx - di, fy - dj, fz - dk);
        double coef = smoothstep_hs(di * fx + (1 - di) * (1 - fx)) * smoothstep_hs(dj * fy + (1 - dj) * (1 - fy)) *
                      smoothstep_hs(dk * fz + (1 - dk) * (1 - fz));
        sum = sum + coef * dot(grad, rel);
      }
  return sum;
}

/* Noise.hs:48-53 fractalNoise: sum (take depth (zipWith (*) coefs (map perlinNoise points))) */
static double fractal_noise(const scene_t* s, int depth, v3 p) {
  double sum = 0, coef = 1;
  for (int l = 0; l < depth; ++l) {
    sum = sum + coef * perlin_noise(s, p);
    coef = coef / 2;
    p = smul(2, p);
  }
  return sum;
}

/* Texture.hs:18-78 */
static v3 eval_texture(const scene_t* s, int tex, const hit_t* h) {
  const int32_t* ti = s->ti + (size_t)tex * 4;
  const double* td = s->td + (size_t)tex * 14;
  const double* prm = td + 6;
  v3 c0 = mk(td[0], td[1], td[2]);
  v3 c1 = mk(td[3], td[4], td[5]);
  switch (ti[0]) {
    case T_CONSTANT: return c0;
    case T_CHECKER: {
      long i = (long)floor(h->u * (double)ti[1]);
      long j = (long)floor(h->v * (double)ti[2]);
      return ((i + j) & 1) == 0 ? c0 : c1;
    }
    case T_IMAGE: {  /* Texture.hs:31-41: floor(u w) `mod` w, floor((1 - v) h) `mod` h, image ! (j :. i) */
      long w = ti[1], hh = ti[2];
      long i = (long)floor(h->u * (double)w) % w, j = (long)floor((1 - h->v) * (double)hh) % hh;
      if (i < 0) i += w;
      if (j < 0) j += hh;
      const float* t = s->texels + 3 * ((size_t)ti[3] + (size_t)j * w + i);
      return mk(t[0], t[1], t[2]);
    }
    case T_NOISE: {  /* Texture.hs:56-67 */
      double scale = 0.5 / 0.8;
      v3 q = add(smul(prm[0], h->p), mk(prm[1], prm[2], prm[3]));
      double n = fractal_noise(s, ti[1], q) * scale + 0.5;
      v3 diff = sub(c1, c0);
      return add(c0, smul(n, diff));
    }
    default: {  /* T_MARBLE, Texture.hs:70-78 */
      double freq = prm[3];
      double sin_arg = freq * dot(mk(prm[0], prm[1], prm[2]), h->p);
      double noise = 10 * fabs(fractal_noise(s, 7, add(smul(0.25 * freq, h->p), mk(prm[4], prm[5], prm[6]))));
      double m = 0.5 + 0.5 * sin(sin_arg + noise);
      return mk(m, m, m);
    }
  }
}

/* rt_hit of a redirect target: parallelogram hit on (0, infinity) (Ray.hs:143-145) */
static int target_hit(const target_t* tg, ray_t r, double* t_out) {
  double p[15] = {tg->q.x, tg->q.y, tg->q.z, tg->u.x, tg->u.y, tg->u.z, tg->v.x, tg->v.y, tg->v.z, 0, 0, 0, 0, 0, 0};
  hit_t h;
  if (!hit_plane(p, P_PARALLELOGRAM, r, 0, INFINITY, &h)) return 0;
  *t_out = h.t;
  return 1;
}

typedef struct {
  int kind; /* 0 absorb 1 scatter 2 hemisphere 3 sphere */
  v3 att, dir;
} matres_t;

static v3 ray_color(const scene_t* s, tctx_t* tc, int depth, double time, ray_t ray);

/* redirect direction choice + mixture pdf weighting (Ray.hs:187-224) */
static v3 scatter_f(const scene_t* s, tctx_t* tc, int depth, double time, const hit_t* h, int hemisphere,
                    const int32_t* mi, const double* md, v3 in_dir, const uint32_t* w) {
  rng_t* r = tc->rng;
  double choice_r = (r->mode == ORACLE_RNG_SPLITMIX) ? hs_random(r) : u01(w[0]);
  int choice = -1;
  for (int k = 0; k < s->nt; k++) if (!(choice_r >= s->targets[k].thresh)) { choice = k; break; }
  v3 dir;
  if (choice < 0) {
    v3 uu;
    if (r->mode == ORACLE_RNG_SPLITMIX) uu = random_unit_vector_sm(r);
    else uu = unit_vector_direct(u01(w[1]), u01(w[2]));
    dir = hemisphere ? normalize(add(h->n, uu)) : uu;
  } else {
    double i, j;
    if (r->mode == ORACLE_RNG_SPLITMIX) { i = hs_random(r); j = hs_random(r); }
    else { i = u01(w[1]); j = u01(w[2]); }
    const target_t* tg = &s->targets[choice];
    v3 light_pt = add(add(tg->q, smul(i, tg->u)), smul(j, tg->v));
    dir = normalize(sub(light_pt, h->p));
  }
  double pdf1 = hemisphere ? dot(dir, h->n) / PI_HS : 0.25 / PI_HS;
  if (hemisphere && pdf1 <= 0) return mk(0, 0, 0);
  double sum = 0;
  ray_t out_ray = {h->p, dir};
  for (int k = 0; k < s->nt; k++) {
    tc->cnt[C_REDIRECT_EVALS] += 1;
    double t, pk = 0;
    if (target_hit(&s->targets[k], out_ray, &t)) pk = t * t / fabs(dot(s->targets[k].cr, dir));
    sum = (k == 0) ? s->targets[k].p * pk : sum + s->targets[k].p * pk;
  }
  double pdf = s->rem_prob * pdf1 + sum;
  v3 c = ray_color(s, tc, depth - 1, time, out_ray);
  /* matF dir */
  v3 tex = eval_texture(s, mi[1], h);
  v3 f;
  switch (mi[0]) {
    case M_LOMMEL: {
      double mu0 = -dot(in_dir, h->n), mu1 = dot(dir, h->n);
      f = smul(0.25 / (mu0 + mu1), tex);
      break;
    }
    case M_ANISOTROPIC: {
      double g = md[0];
      double mu = dot(in_dir, dir);
      double hg = (1 - g * g) / pow(1 + g * g - 2 * g * mu, 1.5);
      f = smul(hg, tex);
      break;
    }
    default: f = tex;
  }
  return muls(mulv(f, c), pdf1 / pdf);
}

/* Ray.hs:174-224 */
static v3 ray_color(const scene_t* s, tctx_t* tc, int depth, double time, ray_t ray) {
  if (depth <= 0) return mk(0, 0, 0);
  tc->segment = (uint32_t)(s->max_depth - depth);
  tc->cnt[C_SEGMENTS] += 1;
  hit_t h;
  if (!hit_node(s, tc, s->root, time, ray, 0.0001, INFINITY, &h)) {
    if (s->bg_kind == BG_CONST) return s->bg0;
    double a = 0.5 * (ray.d.y + 1);
    return add(smul(1 - a, s->bg0), smul(a, s->bg1));
  }
  tc->cnt[C_MATERIAL_HITS] += 1;
  const int32_t* mi = s->mi + (size_t)h.mat * 4;
  const double* md = s->md + (size_t)h.mat * 2;
  rng_t* r = tc->rng;
  uint32_t w[4] = {0, 0, 0, 0};
  if (r->mode == ORACLE_RNG_PHILOX) philox_event(r, tc->segment, EV_SCATTER, w);
  v3 zero = mk(0, 0, 0), emitted = zero, res = zero;
  switch (mi[0]) {
    case M_LIGHT: emitted = eval_texture(s, mi[1], &h); break;
    case M_BLACK: break;
    case M_LAMBERT:
    case M_LOMMEL:
      res = scatter_f(s, tc, depth, time, &h, 1, mi, md, ray.d, w);
      break;
    case M_ISOTROPIC:
    case M_ANISOTROPIC:
      res = scatter_f(s, tc, depth, time, &h, 0, mi, md, ray.d, w);
      break;
    case M_MIRROR: {
      v3 att = eval_texture(s, mi[1], &h);
      ray_t nr = {h.p, reflect(h.n, ray.d)};
      res = mulv(att, ray_color(s, tc, depth - 1, time, nr));
      break;
    }
    case M_METAL: { /* Material.hs:72-78 */
      v3 u = (r->mode == ORACLE_RNG_SPLITMIX) ? random_unit_vector_sm(r) : unit_vector_direct(u01(w[1]), u01(w[2]));
      v3 d2 = add(reflect(h.n, ray.d), smul(md[0], u));
      if (dot(d2, h.n) > 0) {
        v3 att = eval_texture(s, mi[1], &h);
        ray_t nr = {h.p, normalize(d2)};
        res = mulv(att, ray_color(s, tc, depth - 1, time, nr));
      }
      break;
    }
    case M_DIELECTRIC: { /* Material.hs:89-106 */
      double ior = md[0];
      double ratio = h.front ? 1 / ior : ior;
      double cos_t = hmin(1, dot(h.n, neg(ray.d)));
      double sin_t = sqrt(1 - cos_t * cos_t);
      int cannot = ratio * sin_t > 1;
      double r0 = (1 - ratio) / (1 + ratio);
      double r0s = r0 * r0;
      double reflectance = r0s + (1 - r0s) * pow(1 - cos_t, 5);
      double x = (r->mode == ORACLE_RNG_SPLITMIX) ? hs_random(r) : u01(w[0]);
      v3 d2;
      if (cannot || x < reflectance) d2 = reflect(h.n, ray.d);
      else {
        v3 perp = smul(ratio, add(ray.d, smul(cos_t, h.n)));
        v3 para = neg(smul(sqrt(fabs(1 - quadrance(perp))), h.n));
        d2 = add(perp, para);
      }
      ray_t nr = {h.p, d2};
      res = mulv(mk(1, 1, 1), ray_color(s, tc, depth - 1, time, nr));
      break;
    }
    case M_TRANSPARENT: {
      v3 att = eval_texture(s, mi[1], &h);
      ray_t nr = {h.p, ray.d};
      res = mulv(att, ray_color(s, tc, depth - 1, time, nr));
      break;
    }
  }
  return add(emitted, res);
}

/* Ray.hs:226-232 for one pixel */
static v3 pixel_color(const scene_t* s, int i, int j, rng_t* r, double* cnt) {
  tctx_t tc = {r, 0, cnt};
  v3 sum = mk(0, 0, 0);
  for (int smp = 0; smp < s->spp; smp++) {
    double time, dx, dy, x, y;
    r->sample = (uint32_t)smp;
    if (r->mode == ORACLE_RNG_SPLITMIX) {
      time = hs_random(r);
      for (;;) { /* Core.hs:63-68 randomInUnitDisk */
        dx = hs_randomR(r, -1, 1);
        dy = hs_randomR(r, -1, 1);
        if (dx * dx + dy * dy <= 1) break;
      }
      x = hs_random(r);
      y = hs_random(r);
    } else {
      /* device stream: event 0 = (jitter x, jitter y, time, disk radius), event 1 = (disk angle) */
      uint32_t w0[4], w1[4];
      philox_event(r, 0, EV_CAMERA0, w0);
      philox_event(r, 0, EV_CAMERA1, w1);
      x = u01(w0[0]);
      y = u01(w0[1]);
      time = u01(w0[2]);
      double rad = sqrt(u01(w0[3])), th = 2 * PI_HS * u01(w1[0]);
      dx = rad * cos(th);
      dy = rad * sin(th);
    }
    v3 origin = add(add(s->center, smul(dx, s->disk_u)), smul(dy, s->disk_v));
    v3 target = add(add(s->top_left, smul((double)i + x, s->pixel_u)), smul((double)j + y, s->pixel_v));
    ray_t ray = {origin, normalize(sub(target, origin))};
    v3 c = ray_color(s, &tc, s->max_depth, time, ray);
    sum = (smp == 0) ? c : add(sum, c);
    cnt[C_SAMPLES] += 1;
  }
  return divs(sum, (double)s->spp);
}

/* ------------------------------------------------------------------ threading */
typedef struct {
  const scene_t* s;
  const int32_t* pixels;
  int n;
  double* out;
  volatile int next;
  pthread_mutex_t mu;
  double cnt[C_COUNT];
} job_t;

static void* worker(void* arg) {
  job_t* jb = (job_t*)arg;
  double cnt[C_COUNT] = {0};
  const scene_t* s = jb->s;
  for (;;) {
    int k = __atomic_fetch_add(&jb->next, 1, __ATOMIC_RELAXED);
    if (k >= jb->n) break;
    int pix = jb->pixels[k];
    int j = pix / s->width, i = pix % s->width;
    rng_t r;
    memset(&r, 0, sizeof r);
    r.mode = s->rng_mode;
    r.variant = s->variant;
    r.pix = (uint32_t)pix;
    r.key[0] = s->key[0]; r.key[1] = s->key[1];
    if (r.mode == ORACLE_RNG_SPLITMIX) { r.seed = s->pix_seed[pix]; r.gamma = s->pix_gamma[pix]; }
    v3 c = pixel_color(s, i, j, &r, cnt);
    jb->out[3 * (size_t)k + 0] = c.x;
    jb->out[3 * (size_t)k + 1] = c.y;
    jb->out[3 * (size_t)k + 2] = c.z;
  }
  pthread_mutex_lock(&jb->mu);
  for (int c = 0; c < C_COUNT; c++) jb->cnt[c] += cnt[c];
  pthread_mutex_unlock(&jb->mu);
  return 0;
}

/*
 * cam_d: center[0:3] lookAt[3:6] up[6:9] vfov[9] aspect[10] defocusAngle[11] focusDist[12] bg0[13:16] bg1[16:19]
 * cam_i: width, spp, maxDepth, bg_kind, n_targets
 * targets: n_targets x 10 doubles: p, q[3], U[3], V[3]
 * seed: splitmix mode -> (seed_a, seed_b) = SMGen (seed, gamma) of raytrace's StdGen argument;
 *       philox mode   -> seed_a is the 64-bit key.
 * Returns image height (>0) on success, negative on error.
 */
int oracle_render(const int32_t* node_i, const double* node_d, int n_nodes, int root, const int32_t* children,
                  const int32_t* mat_i, const double* mat_d, const int32_t* tex_i, const double* tex_d,
                  const double* cam_d, const int32_t* cam_i, const double* targets, int rng_mode, int variant,
                  uint64_t seed_a, uint64_t seed_b, const int32_t* pixels, int n_pixels, int nthreads, double* out_rgb,
                  double* counters, const float* texels, const int32_t* perlin_perm, const double* perlin_grad) {
  if (root < 0 || root >= n_nodes) return -1;
  scene_t s;
  memset(&s, 0, sizeof s);
  s.ni = node_i; s.nd = node_d; s.children = children; s.mi = mat_i; s.md = mat_d; s.ti = tex_i; s.td = tex_d;
  s.texels = texels; s.perm = perlin_perm; s.grad = perlin_grad;
  s.root = root;
  s.width = cam_i[0]; s.spp = cam_i[1]; s.max_depth = cam_i[2]; s.bg_kind = cam_i[3]; s.nt = cam_i[4];
  s.rng_mode = rng_mode; s.variant = variant;
  if (s.width <= 0 || s.spp <= 0) return -2;
  /* Ray.hs:122-155 */
  v3 center = mk(cam_d[0], cam_d[1], cam_d[2]), look = mk(cam_d[3], cam_d[4], cam_d[5]), up = mk(cam_d[6], cam_d[7], cam_d[8]);
  double vfov = cam_d[9], aspect = cam_d[10], defocus = cam_d[11], focus = cam_d[12];
  s.height = (int)llrint((double)s.width / aspect);
  double vh = focus * tan(vfov / 2) * 2;
  double vw = vh * (double)s.width / (double)s.height;
  v3 w = normalize(sub(center, look));
  v3 u = normalize(cross(up, w));
  v3 v = cross(w, u);
  v3 across = smul(vw, u);
  v3 down = neg(smul(vh, v));
  s.top_left = sub(sub(sub(center, muls(w, focus)), divs(across, 2)), divs(down, 2));
  s.pixel_u = divs(across, (double)s.width);
  s.pixel_v = divs(down, (double)s.height);
  double dr = focus * tan(defocus / 2);
  s.disk_u = muls(u, dr);
  s.disk_v = muls(v, dr);
  s.center = center;
  s.bg0 = mk(cam_d[13], cam_d[14], cam_d[15]);
  s.bg1 = mk(cam_d[16], cam_d[17], cam_d[18]);
  target_t tg[64];
  if (s.nt > 64) return -3;
  double acc = 0, psum = 0;
  for (int k = 0; k < s.nt; k++) {
    const double* t = targets + 10 * k;
    tg[k].p = t[0];
    tg[k].q = mk(t[1], t[2], t[3]); tg[k].u = mk(t[4], t[5], t[6]); tg[k].v = mk(t[7], t[8], t[9]);
    tg[k].cr = cross(tg[k].u, tg[k].v);
    acc = (k == 0) ? t[0] : acc + t[0];   /* scanl1 (+) probs */
    tg[k].thresh = acc;
    psum = (k == 0) ? t[0] : psum + t[0];
  }
  s.targets = tg;
  s.rem_prob = 1 - psum;
  if (s.height <= 0) return -2;
  int maxpix = -1;
  for (int k = 0; k < n_pixels; k++) {
    if (pixels[k] < 0 || pixels[k] >= s.width * s.height) return -4;
    if (pixels[k] > maxpix) maxpix = pixels[k];
  }
  if (rng_mode == ORACLE_RNG_SPLITMIX) {
    /* massiv randomArrayS seed sz splitGen: row-major, element = first component of the split */
    s.pix_seed = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(maxpix + 1));
    s.pix_gamma = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(maxpix + 1));
    uint64_t gs = seed_a, gg = seed_b;
    for (int k = 0; k <= maxpix; k++) {
      uint64_t s1, g1, s2, g2;
      split_smgen(gs, gg, &s1, &g1, &s2, &g2);
      if (variant & 4) { s.pix_seed[k] = s2; s.pix_gamma[k] = g2; gs = s1; gg = g1; continue; }
      s.pix_seed[k] = s1; s.pix_gamma[k] = g1;
      gs = s2; gg = g2;
    }
  } else {
    s.key[0] = (uint32_t)seed_a;
    s.key[1] = (uint32_t)(seed_a >> 32);
  }
  job_t jb;
  memset(&jb, 0, sizeof jb);
  jb.s = &s; jb.pixels = pixels; jb.n = n_pixels; jb.out = out_rgb; jb.next = 0;
  pthread_mutex_init(&jb.mu, 0);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, worker, &jb);
  worker(&jb);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
  pthread_mutex_destroy(&jb.mu);
  if (counters) for (int c = 0; c < C_COUNT; c++) counters[c] = jb.cnt[c];
  free(s.pix_seed);
  free(s.pix_gamma);
  return s.height;
}
