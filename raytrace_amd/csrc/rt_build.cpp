// rt_build.cpp — host-side scene image and launch parameters (no HIP calls).
//
//  * validates the flattened scene of include/rt.h,
//  * precomputes the plane-shape frame of Geometry.hs:117-131 (unit normal n, and the
//    vectors wa = v x nS, wb = nS x u so that a = nS.((p-q) x v) = (p-q).wa and
//    b = nS.(u x (p-q)) = (p-q).wb) in binary64 and rounds it once to FP32,
//  * builds one BVH per primitive set (surfaces, then each medium's boundary),
//  * evaluates the camera set-up of Ray.hs:122-155 in binary64, in the reference's order.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/rt.h"
#include "rt_bvh.h"
#include "rt_encode8_table.h"
#include "rt_internal.h"

const char* rt_knob(const char* name) {
  const char* on = std::getenv("RT_AMD_EXPERIMENTS");
  if (!on || !*on || std::atoi(on) == 0) return nullptr;
  return std::getenv(name);
}

namespace {

struct d3 {
  double x, y, z;
};
inline d3 D3(const double* p) { return {p[0], p[1], p[2]}; }
inline d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline d3 operator-(d3 a) { return {-a.x, -a.y, -a.z}; }
inline d3 smul(double s, d3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline d3 divs(d3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline d3 cross(d3 a, d3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline d3 normalize_hs(d3 v) {  // linear's normalize
  double l = dot(v, v);
  if (std::fabs(l) <= 1e-12 || std::fabs(1 - l) <= 1e-12) return v;
  return divs(v, std::sqrt(l));
}
template <class R>
inline void put3(R* dst, d3 v) {
  dst[0] = (R)v.x;
  dst[1] = (R)v.y;
  dst[2] = (R)v.z;
}
inline bool finite_n(const double* p, int n) {
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(p[i])) return false;
  return true;
}
// an int stored in an R array: its 32-bit pattern in the low word (rt_trace.h RT_R2I)
template <class R>
inline R ibits(int v);
template <>
inline float ibits<float>(int v) {
  float f;
  std::memcpy(&f, &v, 4);
  return f;
}
template <>
inline double ibits<double>(int v) {
  const uint64_t u = (uint32_t)v;
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

int fail(std::string& err, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(std::string& err, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  err = buf;
  return code;
}


// Box groups (rt_internal.h DevBox): parallelograms that are full faces of one rectangular box.
struct BoxFound {
  d3 c, a[3];       // corner, axis_k / L_k
  int face[6];      // caller primitive index of face f = 2 axis + side, -1 if absent
};

// Among `rects` (caller indices of static parallelograms of one set) find boxes with >= 3 faces;
// every primitive is used at most once.  Binary64, relative tolerance 1e-9 of the box size.
std::vector<BoxFound> find_boxes(const rt_scene* sc, const std::vector<int>& rects) {
  std::vector<BoxFound> out;
  const int n = (int)rects.size();
  std::vector<char> used(n, 0);
  auto corners = [&](int i, d3* c4) {
    const double* p = sc->prims[rects[i]].p;
    d3 q = D3(p), u = D3(p + 3), v = D3(p + 6);
    c4[0] = q;
    c4[1] = q + u;
    c4[2] = q + v;
    c4[3] = q + u + v;
  };
  auto is_rect = [&](int i) {
    const double* p = sc->prims[rects[i]].p;
    d3 u = D3(p + 3), v = D3(p + 6);
    double lu = std::sqrt(dot(u, u)), lv = std::sqrt(dot(v, v));
    return lu > 0 && lv > 0 && std::fabs(dot(u, v)) <= 1e-12 * lu * lv;
  };
  for (int i = 0; i < n; ++i) {
    if (used[i] || !is_rect(i)) continue;
    const double* pi = sc->prims[rects[i]].p;
    d3 ui = D3(pi + 3), vi = D3(pi + 6);
    d3 e0 = divs(ui, std::sqrt(dot(ui, ui))), e1 = divs(vi, std::sqrt(dot(vi, vi))), e2 = cross(e0, e1);
    e2 = divs(e2, std::sqrt(dot(e2, e2)));
    d3 ci[4];
    corners(i, ci);
    for (int j = 0; j < n; ++j) {
      if (j == i || used[j] || !is_rect(j)) continue;
      d3 cj[4];
      corners(j, cj);
      const double h = dot(e2, cj[0] - ci[0]);
      const double size = std::sqrt(std::max(dot(ui, ui), dot(vi, vi)));
      const double tol = 1e-9 * std::max(size, std::fabs(h));
      if (!(std::fabs(h) > tol)) continue;
      bool match = true;  // j = i translated by h e2, corner for corner (as sets)
      for (int a = 0; a < 4 && match; ++a) {
        d3 t = cj[a] - smul(h, e2);
        bool any = false;
        for (int b = 0; b < 4; ++b) {
          d3 d = t - ci[b];
          any = any || std::sqrt(dot(d, d)) <= tol;
        }
        match = any;
      }
      if (!match) continue;
      // the box spanned by i and j, in the frame (e0, e1, e2)
      const d3 E[3] = {e0, e1, e2};
      double lo[3], hi[3];
      for (int k = 0; k < 3; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
        for (int a = 0; a < 4; ++a) {
          for (const d3& p : {ci[a], cj[a]}) {
            double x = dot(E[k], p - ci[0]);
            lo[k] = std::min(lo[k], x);
            hi[k] = std::max(hi[k], x);
          }
        }
      }
      BoxFound B;
      B.c = ci[0] + smul(lo[0], e0) + smul(lo[1], e1) + smul(lo[2], e2);
      for (int k = 0; k < 3; ++k) B.a[k] = divs(E[k], hi[k] - lo[k]);
      for (int f = 0; f < 6; ++f) B.face[f] = -1;
      std::vector<int> members;
      for (int m = 0; m < n; ++m) {
        if (used[m] || !is_rect(m)) continue;
        d3 cm[4];
        corners(m, cm);
        double sc4[4][3];
        for (int a = 0; a < 4; ++a)
          for (int k = 0; k < 3; ++k) sc4[a][k] = dot(B.a[k], cm[a] - B.c);
        const double et = 1e-9;
        auto near01 = [&](double x, int& bit) {
          if (std::fabs(x) <= et) return bit = 0, true;
          if (std::fabs(x - 1) <= et) return bit = 1, true;
          return false;
        };
        int face = -1;
        for (int ax = 0; ax < 3 && face < 0; ++ax) {
          int side0 = -1, mask = 0;
          bool ok = true;
          for (int a = 0; a < 4 && ok; ++a) {
            int bits[3];
            for (int k = 0; k < 3 && ok; ++k) ok = near01(sc4[a][k], bits[k]);
            if (!ok) break;
            if (side0 < 0) side0 = bits[ax];
            ok = bits[ax] == side0;
            const int b1 = bits[(ax + 1) % 3], b2 = bits[(ax + 2) % 3];
            mask |= 1 << (b1 * 2 + b2);
          }
          if (ok && mask == 15) face = 2 * ax + side0;  // the four corners of that face
        }
        if (face >= 0 && B.face[face] < 0) {
          B.face[face] = rects[m];
          members.push_back(m);
        }
      }
      if (members.size() >= 3) {
        for (int m : members) used[m] = 1;
        out.push_back(B);
        break;
      }
    }
  }
  return out;
}

struct BoxCodes {
  int ord_base, ord_code, gid_base, gid_code, prim_base, prim_code;
};

// The device records of one precision (rt_internal.h layout): primitives in `order` (slot
// order for flat scenes, with class-grouped test copies), their materials, the textures,
// motions, sphereUV frames, Perlin gradients and box groups.  The plane-shape frame of
// Geometry.hs:117-131 (unit normal n, wa = v x nS, wb = nS x u, so that a = nS.((p-q) x v) =
// (p-q).wa and b = nS.(u x (p-q)) = (p-q).wb) is computed in binary64 and rounded once to R.
template <class R>
void fill_records(const rt_scene* sc, const std::vector<int>& order, const std::vector<int>& slot_of, bool flat,
                  const std::vector<BoxFound>& boxes, const std::vector<BoxCodes>& codes,
                  const std::vector<int>& prim_mat, HostArraysT<R>& A) {
  const int n = (int)order.size();
  A.boxes.clear();
  for (size_t b = 0; b < boxes.size(); ++b) {
    DevBoxT<R> d;
    std::memset(&d, 0, sizeof d);
    // the slab offsets a_k . c in binary64, rounded once (the kernel's s_k = a_k . o - sc[k], three
    // FMAs per axis instead of the ray origin relative to the corner and a dot product)
    for (int k = 0; k < 3; ++k) d.sc[k] = (R)dot(boxes[b].a[k], boxes[b].c);
    put3(d.a0, boxes[b].a[0]);
    put3(d.a1, boxes[b].a[1]);
    put3(d.a2, boxes[b].a[2]);
    d.ord_base = codes[b].ord_base;
    d.ord_code = codes[b].ord_code;
    d.gid_base = codes[b].gid_base;
    d.gid_code = codes[b].gid_code;
    d.prim_base = codes[b].prim_base;
    d.prim_code = codes[b].prim_code;
    A.boxes.push_back(d);
  }
  A.prims.assign((size_t)n * 16, (R)0);
  A.prim_uv.assign((size_t)n * 6, (R)0);
  for (int j = 0; j < n; ++j) {
    const rt_prim& p = sc->prims[order[j]];
    R* f = A.prims.data() + 16 * (size_t)j;
    int kf = (p.kind == RT_PRIM_SPHERE ? 0 : p.kind == RT_PRIM_PARALLELOGRAM ? 1 : 2) |
             (p.motion >= 0 ? RT_FLAG_MOTION : 0);
    if (p.kind == RT_PRIM_SPHERE) {
      f[0] = (R)p.p[0];
      f[1] = (R)p.p[1];
      f[2] = (R)p.p[2];
      f[4] = (R)p.p[3];
      f[5] = (R)(p.p[3] * p.p[3]);
      f[6] = ibits<R>(p.uvframe);
    } else {
      d3 q = D3(p.p), u = D3(p.p + 3), v = D3(p.p + 6);
      d3 cp = cross(u, v);
      double ncp = std::sqrt(dot(cp, cp));
      d3 nrm = divs(cp, ncp), nS = divs(nrm, ncp);
      put3(f, nrm);
      put3(f + 4, q);
      put3(f + 8, cross(v, nS));
      put3(f + 12, cross(nS, u));
      if (!(ncp > 0)) f[0] = f[1] = f[2] = (R)0;  // the reference's normal is NaN: never hit
      for (int k = 0; k < 6; ++k) A.prim_uv[6 * (size_t)j + k] = (R)p.uv[k];
    }
    f[3] = ibits<R>(kf);
    f[7] = ibits<R>(p.gid);
    f[11] = ibits<R>(flat ? slot_of[j] : p.order);
    f[15] = ibits<R>(p.motion);
  }
  A.flat_recs.clear();
  if (flat) {  // test order -> slot order for the shading arrays (prim index = slot)
    A.flat_recs = A.prims;
    std::vector<R> prims(A.prims.size()), uv(A.prim_uv.size());
    for (int j = 0; j < n; ++j) {
      const int k = slot_of[j];
      std::copy(A.flat_recs.begin() + 16 * (size_t)j, A.flat_recs.begin() + 16 * (size_t)(j + 1),
                prims.begin() + 16 * (size_t)k);
      std::copy(A.prim_uv.begin() + 6 * (size_t)j, A.prim_uv.begin() + 6 * (size_t)(j + 1), uv.begin() + 6 * (size_t)k);
    }
    A.prims.swap(prims);
    A.prim_uv.swap(uv);
  }
  A.mats.assign(sc->n_materials, DevMaterialT<R>{});
  for (int i = 0; i < sc->n_materials; ++i) {
    DevMaterialT<R>& d = A.mats[i];
    d.kind = sc->materials[i].kind;
    d.tex = sc->materials[i].texture;
    d.param = (R)sc->materials[i].param;
    const rt_texture& t = sc->textures[d.tex];
    d.tex_const = t.kind == RT_TEX_CONSTANT ? 1 : 0;
    for (int a = 0; a < 3; ++a) d.c0[a] = (R)t.c0[a];
  }
  A.prim_shade.assign(prim_mat.size(), DevMaterialT<R>{});
  for (size_t j = 0; j < prim_mat.size(); ++j)
    if (prim_mat[j] >= 0) A.prim_shade[j] = A.mats[prim_mat[j]];
  A.texs.assign(sc->n_textures, DevTextureT<R>{});
  for (int i = 0; i < sc->n_textures; ++i) {
    const rt_texture& t = sc->textures[i];
    DevTextureT<R>& d = A.texs[i];
    d.kind = t.kind;
    d.nu = t.nu;
    d.nv = t.nv;
    d.off = t.kind == RT_TEX_IMAGE ? t.image : 0;
    for (int a = 0; a < 3; ++a) {
      d.c0[a] = (R)t.c0[a];
      d.c1[a] = (R)t.c1[a];
    }
    for (int a = 0; a < 8; ++a) d.prm[a] = (R)t.params[a];
  }
  A.texels.assign((size_t)sc->n_texels * 4, (R)0);
  for (int i = 0; i < sc->n_texels; ++i)
    for (int a = 0; a < 3; ++a) A.texels[4 * (size_t)i + a] = (R)sc->texels[3 * (size_t)i + a];
  A.perlin_grad.assign(256 * 4, (R)0);
  if (sc->perlin)
    for (int k = 0; k < 256; ++k)
      for (int a = 0; a < 3; ++a) A.perlin_grad[4 * k + a] = (R)sc->perlin->grad[k][a];
  A.motions.assign((size_t)sc->n_motions * 8, (R)0);
  for (int i = 0; i < sc->n_motions; ++i)
    for (int a = 0; a < 3; ++a) {
      A.motions[8 * (size_t)i + a] = (R)sc->motions[i].v0[a];
      A.motions[8 * (size_t)i + 4 + a] = (R)sc->motions[i].v1[a];
    }
  A.uvframes.assign((size_t)sc->n_uvframes * 12, (R)0);
  for (int i = 0; i < sc->n_uvframes; ++i)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) A.uvframes[12 * (size_t)i + 4 * r + c] = (R)sc->uvframes[i].r[3 * r + c];
}

template <class R>
void fill_instances(const rt_scene* sc, const std::vector<int>& blas_root, HostArraysT<R>& A) {
  A.instances.assign(sc->n_instances, DevInstanceT<R>{});
  for (int k = 0; k < sc->n_instances; ++k) {
    const rt_instance& I = sc->instances[k];
    DevInstanceT<R>& d = A.instances[k];
    for (int a = 0; a < 12; ++a) d.m[a] = (R)I.m[a];
    d.root = blas_root[I.blas];
    d.material = I.material;
    d.order = I.order;
    d.pad = 0;
  }
}

}  // namespace

int rt_host_image_height(const rt_camera_settings* cs) {
  double h = (double)cs->image_width / cs->aspect_ratio;
  if (!std::isfinite(h) || h > 1e9) return -1;
  return (int)std::nearbyint(h);  // round-half-even under the default rounding mode (Ray.hs:123)
}

int rt_host_shard_rows(int height, const rt_exec* ex) {
  if (!ex || ex->n_shards < 1 || ex->row_block < 1 || ex->shard < 0 || ex->shard >= ex->n_shards || height < 0)
    return RT_E_INVALID;
  if (ex->n_shards == 1) return height;  // the whole image, unpadded
  int blocks = (height + ex->row_block - 1) / ex->row_block;
  int per = (blocks + ex->n_shards - 1) / ex->n_shards;
  return per * ex->row_block;
}

int rt_host_build_scene(const rt_scene* sc, HostScene& S, std::string& err) {
  if (!sc) return fail(err, RT_E_INVALID, "null scene");
  if (sc->n_prims < 0 || sc->n_media < 0 || sc->n_materials < 0 || sc->n_textures < 0 || sc->n_motions < 0 ||
      sc->n_uvframes < 0)
    return fail(err, RT_E_INVALID, "negative count");
  if (sc->n_media > RT_MAX_MEDIA)
    return fail(err, RT_E_UNSUPPORTED, "%d media (at most %d)", sc->n_media, RT_MAX_MEDIA);
  if ((sc->n_prims && !sc->prims) || (sc->n_media && !sc->media) || (sc->n_materials && !sc->materials) ||
      (sc->n_textures && !sc->textures) || (sc->n_motions && !sc->motions) || (sc->n_uvframes && !sc->uvframes))
    return fail(err, RT_E_INVALID, "null array with nonzero count");
  if (sc->n_texels < 0 || (sc->n_texels && !sc->texels)) return fail(err, RT_E_INVALID, "bad texel array");
  bool need_perlin = false;
  for (int i = 0; i < sc->n_textures; ++i) {
    const rt_texture& t = sc->textures[i];
    if (t.kind < RT_TEX_CONSTANT || t.kind > RT_TEX_MARBLE)
      return fail(err, RT_E_UNSUPPORTED, "texture %d: kind %d is not evaluated on the device", i, t.kind);
    if (!finite_n(t.c0, 3) || !finite_n(t.c1, 3)) return fail(err, RT_E_INVALID, "texture %d: non-finite colour", i);
    if (!finite_n(t.params, 8)) return fail(err, RT_E_INVALID, "texture %d: non-finite parameters", i);
    if (t.kind == RT_TEX_IMAGE &&
        (t.nu <= 0 || t.nv <= 0 || t.image < 0 || (long long)t.image + (long long)t.nu * t.nv > sc->n_texels))
      return fail(err, RT_E_INVALID, "texture %d: image %dx%d at texel %d exceeds the %d texels", i, t.nu, t.nv,
                  t.image, sc->n_texels);
    if (t.kind == RT_TEX_NOISE && t.nu < 0) return fail(err, RT_E_INVALID, "texture %d: negative noise layers", i);
    if (t.kind == RT_TEX_NOISE || t.kind == RT_TEX_MARBLE) need_perlin = true;
  }
  S.noise = need_perlin;
  if (need_perlin) {
    if (!sc->perlin) return fail(err, RT_E_INVALID, "noise / marble textures need rt_scene.perlin");
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 256; ++k)
        if (sc->perlin->perm[a][k] < 0 || sc->perlin->perm[a][k] > 255)
          return fail(err, RT_E_INVALID, "perlin permutation entry out of [0, 255]");
    for (int k = 0; k < 256; ++k)
      if (!finite_n(sc->perlin->grad[k], 3)) return fail(err, RT_E_INVALID, "non-finite perlin gradient");
  }
  S.full_mats = false;
  S.uv_tex = false;
  for (int i = 0; i < sc->n_materials; ++i) {
    const rt_material& m = sc->materials[i];
    if (m.kind != RT_MAT_LIGHT_SOURCE && m.kind != RT_MAT_PITCH_BLACK && m.kind != RT_MAT_LAMBERTIAN) S.full_mats = true;
    if (m.texture >= 0 && m.texture < sc->n_textures && sc->textures[m.texture].kind != RT_TEX_CONSTANT) S.uv_tex = true;
    if (m.kind < 0 || m.kind > RT_MAT_ANISOTROPIC)
      return fail(err, RT_E_UNSUPPORTED, "material %d: kind %d", i, m.kind);
    if (m.texture < 0 || m.texture >= sc->n_textures)
      return fail(err, RT_E_INVALID, "material %d: bad texture index", i);
  }
  for (int k = 0; k < sc->n_media; ++k) {
    const rt_medium& m = sc->media[k];
    if (!(m.density > 0) || !std::isfinite(m.density))
      return fail(err, RT_E_INVALID, "medium %d: density must be > 0", k);
    if (m.material < 0 || m.material >= sc->n_materials) return fail(err, RT_E_INVALID, "medium %d: bad material", k);
  }
  const int n_sets = 1 + sc->n_media;
  // two-level instancing: instanced objects (prims with set RT_SET_BLAS(b)) and their placements
  if (sc->n_instances < 0 || (sc->n_instances && !sc->instances)) return fail(err, RT_E_INVALID, "bad instance array");
  int n_blas = 0;
  for (int i = 0; i < sc->n_prims; ++i)
    if (sc->prims[i].set < 0) n_blas = std::max(n_blas, -sc->prims[i].set);
  for (int k = 0; k < sc->n_instances; ++k) {
    const rt_instance& I = sc->instances[k];
    if (I.blas < 0 || I.blas >= n_blas) return fail(err, RT_E_INVALID, "instance %d: object %d has no leaves", k, I.blas);
    if (I.material < -1 || I.material >= sc->n_materials) return fail(err, RT_E_INVALID, "instance %d: bad material", k);
    if (!finite_n(I.m, 12)) return fail(err, RT_E_INVALID, "instance %d: non-finite transform", k);
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        const double d = I.m[a] * I.m[b] + I.m[4 + a] * I.m[4 + b] + I.m[8 + a] * I.m[8 + b];
        if (std::fabs(d - (a == b ? 1.0 : 0.0)) > 1e-9)
          return fail(err, RT_E_UNSUPPORTED, "instance %d: transform is not rigid (Geometry.hs:379-381)", k);
      }
  }
  std::vector<std::vector<BuildPrim>> sets(n_sets), blas_sets(n_blas);
  std::vector<char> blas_all_mats(n_blas, 1);
  for (int i = 0; i < sc->n_prims; ++i) {
    const rt_prim& p = sc->prims[i];
    if (p.kind < RT_PRIM_SPHERE || p.kind > RT_PRIM_TRIANGLE) return fail(err, RT_E_INVALID, "prim %d: bad kind", i);
    if (p.set >= n_sets) return fail(err, RT_E_INVALID, "prim %d: bad set %d", i, p.set);
    if (p.set == 0 && (p.material < 0 || p.material >= sc->n_materials))
      return fail(err, RT_E_INVALID, "prim %d: surface without a valid material", i);
    if (p.set < 0 && (p.material < -1 || p.material >= sc->n_materials))
      return fail(err, RT_E_INVALID, "prim %d: bad material", i);
    if (p.set < 0 && p.material < 0) blas_all_mats[-1 - p.set] = 0;
    if (p.motion >= sc->n_motions || p.uvframe >= sc->n_uvframes)
      return fail(err, RT_E_INVALID, "prim %d: bad motion/uvframe index", i);
    if (!finite_n(p.p, p.kind == RT_PRIM_SPHERE ? 4 : 9))
      return fail(err, RT_E_INVALID, "prim %d: non-finite geometry", i);
    BuildPrim bp;
    bp.index = i;
    if (p.kind == RT_PRIM_SPHERE) {
      double r = std::fabs(p.p[3]);
      for (int a = 0; a < 3; ++a) {
        bp.lo[a] = p.p[a] - r;
        bp.hi[a] = p.p[a] + r;
      }
    } else {
      for (int a = 0; a < 3; ++a) {
        double q = p.p[a], u = p.p[3 + a], v = p.p[6 + a];
        double c[4] = {q, q + u, q + v, q + u + v};
        int nc = p.kind == RT_PRIM_PARALLELOGRAM ? 4 : 3;
        bp.lo[a] = bp.hi[a] = c[0];
        for (int k = 1; k < nc; ++k) {
          bp.lo[a] = std::fmin(bp.lo[a], c[k]);
          bp.hi[a] = std::fmax(bp.hi[a], c[k]);
        }
      }
    }
    if (p.motion >= 0) {
      const rt_motion& m = sc->motions[p.motion];
      if (!finite_n(m.v0, 3) || !finite_n(m.v1, 3)) return fail(err, RT_E_INVALID, "motion %d non-finite", p.motion);
      for (int a = 0; a < 3; ++a) {
        double lo = bp.lo[a], hi = bp.hi[a];
        bp.lo[a] = std::fmin(lo + m.v0[a], lo + m.v1[a]);
        bp.hi[a] = std::fmax(hi + m.v0[a], hi + m.v1[a]);
      }
    }
    if (p.set < 0)
      blas_sets[-1 - p.set].push_back(bp);
    else
      sets[p.set].push_back(bp);
  }
  for (int k = 0; k < sc->n_media; ++k)
    if (sets[k + 1].empty()) return fail(err, RT_E_INVALID, "medium %d has an empty boundary", k);
  // every placement is one item of the surface set, boxed by its object's box under the transform
  for (int k = 0; k < sc->n_instances; ++k) {
    const rt_instance& I = sc->instances[k];
    if (blas_sets[I.blas].empty()) return fail(err, RT_E_INVALID, "instance %d: object %d has no leaves", k, I.blas);
    if (I.material < 0 && !blas_all_mats[I.blas])
      return fail(err, RT_E_INVALID, "instance %d: a leaf of object %d has no material", k, I.blas);
    double olo[3] = {INFINITY, INFINITY, INFINITY}, ohi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const BuildPrim& b : blas_sets[I.blas])
      for (int a = 0; a < 3; ++a) {
        olo[a] = std::min(olo[a], b.lo[a]);
        ohi[a] = std::max(ohi[a], b.hi[a]);
      }
    BuildPrim bp;
    bp.index = -1;
    bp.inst = k;
    for (int a = 0; a < 3; ++a) {
      bp.lo[a] = INFINITY;
      bp.hi[a] = -INFINITY;
    }
    for (int c = 0; c < 8; ++c) {
      const double x[3] = {(c & 1) ? ohi[0] : olo[0], (c & 2) ? ohi[1] : olo[1], (c & 4) ? ohi[2] : olo[2]};
      for (int a = 0; a < 3; ++a) {
        const double w = I.m[4 * a] * x[0] + I.m[4 * a + 1] * x[1] + I.m[4 * a + 2] * x[2] + I.m[4 * a + 3];
        bp.lo[a] = std::min(bp.lo[a], w);
        bp.hi[a] = std::max(bp.hi[a], w);
      }
    }
    sets[0].push_back(bp);
  }

  // media whose boundary is, leaf for leaf in depth-first order, the surface set (DevMedium)
  std::vector<int> alias(sc->n_media, 0);
  {
    std::vector<std::vector<int>> by_set(n_sets);
    for (int i = 0; i < sc->n_prims; ++i)
      if (sc->prims[i].set >= 0) by_set[sc->prims[i].set].push_back(i);  // instanced objects' leaves: not a set
    for (auto& v : by_set)
      std::stable_sort(v.begin(), v.end(), [&](int x, int y) { return sc->prims[x].order < sc->prims[y].order; });
    auto same = [&](const rt_prim& a, const rt_prim& b) {
      if (a.kind != b.kind || a.motion != b.motion || a.gid != b.gid || a.uvframe != b.uvframe) return false;
      for (int j = 0; j < 9; ++j)
        if (a.p[j] != b.p[j]) return false;
      return true;
    };
    for (int k = 0; k < sc->n_media; ++k) {
      const auto& a = by_set[0];
      const auto& b = by_set[k + 1];
      bool eq = !a.empty() && a.size() == b.size();
      for (size_t j = 0; eq && j < a.size(); ++j) eq = same(sc->prims[a[j]], sc->prims[b[j]]);
      alias[k] = eq ? 1 : 0;
    }
  }
  if (const char* e = rt_knob("RT_AMD_NO_ALIAS"))  // experiments: always traverse boundaries
    if (atoi(e)) std::fill(alias.begin(), alias.end(), 0);
  if (sc->n_instances > 0) std::fill(alias.begin(), alias.end(), 0);  // the surface set also holds placements

  // Large-primitive prefix of the surface set (BVH scenes).  Primitives whose box is a large
  // fraction of the whole set's (the Cornell walls around a mesh, demo1's ground sphere) overlap
  // almost every ray and sit at the top of any BVH; taken out of it, they are tested first by
  // the whole wave with wave-uniform records (scalar loads, like the flat kernel), and their
  // closest hit then bounds the traversal of the remaining BVH (rt_trace.h prefix_hits).  The
  // 64-bit closest-hit key carries each leaf's global depth-first order, so the result is the
  // same closest hit, tie for tie.  Only static primitives; grouped by class like a flat set.
  std::vector<int> prefix;  // caller indices, class-grouped
  int prefix_cnt[3] = {0, 0, 0};
  {
    bool want = (int)sets[0].size() > RT_FLAT_MAX + RT_PREFIX_MAX;
    if (const char* e = rt_knob("RT_AMD_NO_PREFIX"))  // experiments: everything in the BVH
      if (atoi(e)) want = false;
    if (want) {
      auto area = [](const double* lo, const double* hi) {
        double d[3];
        for (int a = 0; a < 3; ++a) d[a] = std::max(0.0, hi[a] - lo[a]);
        return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
      };
      double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (const BuildPrim& b : sets[0])
        for (int a = 0; a < 3; ++a) {
          lo[a] = std::min(lo[a], b.lo[a]);
          hi[a] = std::max(hi[a], b.hi[a]);
        }
      const double root_area = area(lo, hi);
      double frac = RT_PREFIX_AREA;
      if (const char* e = rt_knob("RT_AMD_PREFIX_AREA")) frac = atof(e);  // experiments
      std::vector<std::pair<double, int>> big;  // (area, position in sets[0])
      for (size_t j = 0; j < sets[0].size(); ++j) {
        const BuildPrim& b = sets[0][j];
        const double a = area(b.lo, b.hi);
        if (b.inst < 0 && sc->prims[b.index].motion < 0 && a >= frac * root_area) big.push_back({-a, (int)j});
      }
      std::stable_sort(big.begin(), big.end());
      if (big.size() > RT_PREFIX_MAX) big.resize(RT_PREFIX_MAX);
      std::vector<char> taken(sets[0].size(), 0);
      for (auto& b : big) taken[b.second] = 1;
      // then outliers: a primitive that alone holds a face of the remaining set's box out by a
      // lot (the Cornell light above the bunny: without it the BVH root shrinks to the bunny)
      double shrink = RT_PREFIX_SHRINK;
      if (const char* e = rt_knob("RT_AMD_PREFIX_SHRINK")) shrink = atof(e);  // experiments
      for (int added = (int)big.size(); added < RT_PREFIX_MAX && shrink < 1.0; ++added) {
        auto bounds_without = [&](int skip, double* l, double* h) {
          for (int a = 0; a < 3; ++a) {
            l[a] = INFINITY;
            h[a] = -INFINITY;
          }
          for (size_t j = 0; j < sets[0].size(); ++j) {
            if (taken[j] || (int)j == skip) continue;
            for (int a = 0; a < 3; ++a) {
              l[a] = std::min(l[a], sets[0][j].lo[a]);
              h[a] = std::max(h[a], sets[0][j].hi[a]);
            }
          }
        };
        double l0[3], h0[3];
        bounds_without(-1, l0, h0);
        const double a0 = area(l0, h0);
        int best_j = -1;
        double best_a = a0;
        for (size_t j = 0; j < sets[0].size(); ++j) {  // candidates: the primitives on the box's faces
          const BuildPrim& b = sets[0][j];
          bool extreme = false;
          for (int a = 0; a < 3; ++a) extreme = extreme || b.lo[a] == l0[a] || b.hi[a] == h0[a];
          if (taken[j] || !extreme || b.inst >= 0 || sc->prims[b.index].motion >= 0) continue;
          double l[3], h[3];
          bounds_without((int)j, l, h);
          const double a = area(l, h);
          if (a < best_a) {
            best_a = a;
            best_j = (int)j;
          }
        }
        if (best_j < 0 || !(best_a <= (1.0 - shrink) * a0)) break;
        taken[best_j] = 1;
      }
      auto cls = [&](int i) {
        const int k = sc->prims[i].kind;
        return k == RT_PRIM_PARALLELOGRAM ? 0 : k == RT_PRIM_TRIANGLE ? 1 : 2;
      };
      std::vector<BuildPrim> rest;
      for (size_t j = 0; j < sets[0].size(); ++j) {
        if (taken[j])
          prefix.push_back(sets[0][j].index);
        else
          rest.push_back(sets[0][j]);
      }
      std::stable_sort(prefix.begin(), prefix.end(), [&](int x, int y) { return cls(x) < cls(y); });
      for (int i : prefix) prefix_cnt[cls(i)]++;
      sets[0].swap(rest);
    }
  }

  // one BVH per set; primitives stored in leaf order, set after set (the prefix first)
  std::vector<int> order(prefix);
  std::vector<int> roots(n_sets), set_begin(n_sets + 1, 0);
  int surface_depth = 0;
  set_begin[0] = (int)prefix.size();
  S.nodes.clear();
  S.max_depth = 0;
  for (int s = 0; s < n_sets; ++s) {
    BvhOut bo;
    // leaves of at most 2 triangles / quads (bunny-Cornell 112 -> 107 ms, pawn+fog -1.2 % against
    // 8 under the leaf-exit policy); sphere sets keep 8 (demo1 +0.6 % at 2)
    bool spheres = true;
    for (const BuildPrim& b : sets[s]) spheres = spheres && b.inst < 0 && sc->prims[b.index].kind == RT_PRIM_SPHERE;
    int leaf_max = spheres ? RT_LEAF_MAX : 2;
    if (const char* e = rt_knob("RT_AMD_LEAF_MAX")) leaf_max = std::max(1, std::min(RT_FLAT_MAX, atoi(e)));
    rt_build_bvh(sets[s], (int)(S.nodes.size() / 16), (int)order.size(), bo, leaf_max);
    S.nodes.insert(S.nodes.end(), bo.nodes.begin(), bo.nodes.end());
    order.insert(order.end(), bo.order.begin(), bo.order.end());
    roots[s] = bo.root;
    S.max_depth = std::max(S.max_depth, bo.max_depth);
    set_begin[s + 1] = (int)order.size();
    if (s == 0) {
      S.surface_nodes = (int)(S.nodes.size() / 16);
      surface_depth = bo.max_depth;
    }
  }
  // instanced objects: one object-space BVH each (leaves of at most 2 primitives, as meshes),
  // after the sets; the stack holds the world levels, the exit marker and the object's levels
  std::vector<int> blas_root(n_blas, RT_EMPTY_ROOT);
  int blas_depth = 0;
  for (int b = 0; b < n_blas && sc->n_instances > 0; ++b) {
    BvhOut bo;
    rt_build_bvh(blas_sets[b], (int)(S.nodes.size() / 16), (int)order.size(), bo, 2);
    S.nodes.insert(S.nodes.end(), bo.nodes.begin(), bo.nodes.end());
    order.insert(order.end(), bo.order.begin(), bo.order.end());
    blas_root[b] = bo.root;
    blas_depth = std::max(blas_depth, bo.max_depth);
  }
  if (sc->n_instances > 0) S.max_depth = std::max(S.max_depth, surface_depth + 1 + blas_depth + 1);
  if (S.nodes.size() / 16 >= (size_t)RT_MAX_NODES)
    return fail(err, RT_E_UNSUPPORTED, "%zu BVH nodes exceed the kernels' 32-bit node offsets (%d)", S.nodes.size() / 16,
                RT_MAX_NODES);
  if (S.max_depth > RT_STACK_DEPTH)
    return fail(err, RT_E_STACK, "BVH depth %d exceeds the traversal stack (%d)", S.max_depth, RT_STACK_DEPTH);
  const int n = (int)order.size();
  S.flat = S.nodes.empty() && n <= RT_LDS_PRIMS_MAX && prefix.empty() && sc->n_instances == 0;
  if (!prefix.empty()) {  // BVH scenes: flat_sets[0] describes the surface prefix
    DevFlatSet& F = S.flat_sets[0];
    F.first = 0;
    F.end_quad = prefix_cnt[0];
    F.end_tri = F.end_quad + prefix_cnt[1];
    F.end_sphere = F.end_tri + prefix_cnt[2];
    F.end = F.end_sphere;
  }
  if (S.flat) {
    // group each set's single leaf by class (rt_internal.h DevFlatSet); stable within a class
    auto cls = [&](int i) {
      const rt_prim& p = sc->prims[i];
      if (p.motion >= 0) return 3;
      return p.kind == RT_PRIM_PARALLELOGRAM ? 0 : p.kind == RT_PRIM_TRIANGLE ? 1 : 2;
    };
    for (int s = 0; s < n_sets; ++s) {
      int* b = order.data() + set_begin[s];
      int* e = order.data() + set_begin[s + 1];
      std::stable_sort(b, e, [&](int x, int y) { return cls(x) < cls(y); });
      int cnt[4] = {0, 0, 0, 0};
      for (int* it = b; it != e; ++it) cnt[cls(*it)]++;
      DevFlatSet& F = S.flat_sets[s];
      F.first = set_begin[s];
      F.end_quad = F.first + cnt[0];
      F.end_tri = F.end_quad + cnt[1];
      F.end_sphere = F.end_tri + cnt[2];
      F.end = F.end_sphere + cnt[3];
      F.box_first = F.box_end = 0;
      F.pad = 0;
    }
  }
  // box groups among each flat set's static parallelograms (and the surface prefix): their
  // faces move to the end of the set's range, after the tested classes (DevBox)
  std::vector<BoxFound> boxes;
  std::vector<int> box_face_pos;  // per box: position in `order` of its first face
  {
    bool want = true;
    if (const char* e = rt_knob("RT_AMD_NO_BOX"))  // experiments: every face its own test
      if (atoi(e)) want = false;
    for (int s = 0; s < n_sets && want; ++s) {
      if (!S.flat && !(s == 0 && !prefix.empty())) break;
      DevFlatSet& F = S.flat_sets[s];
      const int set_end = S.flat ? set_begin[s + 1] : (int)prefix.size();
      std::vector<int> quads(order.begin() + F.first, order.begin() + F.end_quad);
      std::vector<BoxFound> found;
      for (const BoxFound& B : find_boxes(sc, quads)) {
        // the faces' key orders and gids must fit the 5-bit offset codes (slot spans are at
        // most the order spans)
        int olo = INT32_MAX, ohi = INT32_MIN, glo = INT32_MAX, ghi = INT32_MIN;
        for (int f = 0; f < 6; ++f) {
          if (B.face[f] < 0) continue;
          const rt_prim& p = sc->prims[B.face[f]];
          olo = std::min(olo, p.order);
          ohi = std::max(ohi, p.order);
          glo = std::min(glo, p.gid);
          ghi = std::max(ghi, p.gid);
        }
        if ((long long)ohi - olo < RT_BOX_NO_FACE && (long long)ghi - glo < RT_BOX_NO_FACE) found.push_back(B);
      }
      F.box_first = F.box_end = (int)boxes.size();
      if (found.empty()) continue;
      std::vector<char> in_box(sc->n_prims, 0);
      for (const BoxFound& B : found)
        for (int f = 0; f < 6; ++f)
          if (B.face[f] >= 0) in_box[B.face[f]] = 1;
      std::vector<int> rest, faces;
      int removed = 0;
      for (int j = F.first; j < set_end; ++j) {
        if (in_box[order[j]]) {
          ++removed;
          continue;
        }
        rest.push_back(order[j]);
      }
      for (const BoxFound& B : found) {
        box_face_pos.push_back(F.first + (int)rest.size() + (int)faces.size());
        for (int f = 0; f < 6; ++f)
          if (B.face[f] >= 0) faces.push_back(B.face[f]);
        boxes.push_back(B);
      }
      std::copy(rest.begin(), rest.end(), order.begin() + F.first);
      std::copy(faces.begin(), faces.end(), order.begin() + F.first + rest.size());
      F.end_quad -= removed;
      F.end_tri -= removed;
      F.end_sphere -= removed;
      F.end -= removed;
      F.box_end = (int)boxes.size();
    }
  }
  // flat scenes: slot of each primitive (rank of its order within the set) and slot -> index
  std::vector<int> slot_of(n, 0);
  if (S.flat) {
    for (int s = 0; s < n_sets; ++s) {
      std::vector<int> pos;
      for (int j = set_begin[s]; j < set_begin[s + 1]; ++j) pos.push_back(j);
      std::stable_sort(pos.begin(), pos.end(),
                       [&](int x, int y) { return sc->prims[order[x]].order < sc->prims[order[y]].order; });
      for (size_t r = 0; r < pos.size(); ++r) {
        slot_of[pos[r]] = set_begin[s] + (int)r;
      }
    }
  }
  // box groups: the faces' key orders, gids and primitive indices as base + 5-bit codes
  std::vector<BoxCodes> box_codes;
  {
    std::vector<int> pos_of(sc->n_prims, -1);
    for (int j = 0; j < n; ++j) pos_of[order[j]] = j;
    for (size_t b = 0; b < boxes.size(); ++b) {
      const BoxFound& B = boxes[b];
      BoxCodes d{};
      int ord[6], gid[6], prm[6];
      int ob = INT32_MAX, gb = INT32_MAX, pb = INT32_MAX;
      for (int f = 0; f < 6; ++f) {
        if (B.face[f] < 0) continue;
        const int j = pos_of[B.face[f]];
        ord[f] = S.flat ? slot_of[j] : sc->prims[B.face[f]].order;
        gid[f] = sc->prims[B.face[f]].gid;
        prm[f] = S.flat ? slot_of[j] : j;
        ob = std::min(ob, ord[f]);
        gb = std::min(gb, gid[f]);
        pb = std::min(pb, prm[f]);
      }
      d.ord_base = ob;
      d.gid_base = gb;
      d.prim_base = pb;
      bool fits = true;
      for (int f = 0; f < 6; ++f) {
        int oo = RT_BOX_NO_FACE, go = RT_BOX_NO_FACE, po = RT_BOX_NO_FACE;
        if (B.face[f] >= 0) {
          oo = ord[f] - ob;
          go = gid[f] - gb;
          po = prm[f] - pb;
          fits = fits && oo < RT_BOX_NO_FACE && go < RT_BOX_NO_FACE && po < RT_BOX_NO_FACE;
        }
        d.ord_code |= oo << (5 * f);
        d.gid_code |= go << (5 * f);
        d.prim_code |= po << (5 * f);
      }
      if (!fits) return fail(err, RT_E_GENERIC, "box group %d: face offsets exceed the 5-bit codes", (int)b);
      box_codes.push_back(d);
    }
  }
  S.prim_mat.assign(n, -1);
  for (int j = 0; j < n; ++j) S.prim_mat[j] = sc->prims[order[j]].set <= 0 ? sc->prims[order[j]].material : -1;
  if (S.flat) {  // test order -> slot order for the shading arrays (prim index = slot)
    std::vector<int> mat(S.prim_mat.size());
    for (int j = 0; j < n; ++j) mat[slot_of[j]] = S.prim_mat[j];
    S.prim_mat.swap(mat);
  }
  fill_records(sc, order, slot_of, S.flat, boxes, box_codes, S.prim_mat, S.f32);
  fill_records(sc, order, slot_of, S.flat, boxes, box_codes, S.prim_mat, S.f64);
  fill_instances(sc, blas_root, S.f32);
  fill_instances(sc, blas_root, S.f64);
  S.n_instances = sc->n_instances;
  S.n_boxes = (int)boxes.size();
  S.perlin_perm.assign(3 * 256, 0);
  if (sc->perlin)
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 256; ++k) S.perlin_perm[256 * a + k] = sc->perlin->perm[a][k];
  S.surface_root = roots[0];
  S.n_media = sc->n_media;
  for (int k = 0; k < sc->n_media; ++k) {
    S.f32.media[k] = DevMedium{(float)(-(1.0 / sc->media[k].density)), sc->media[k].material, roots[k + 1], alias[k]};
    S.f64.media[k] = DevMediumT<double>{-(1.0 / sc->media[k].density), sc->media[k].material, roots[k + 1], alias[k]};
  }
  S.n_nodes = (int)(S.nodes.size() / 16);
  // BVH traversal policy (KernelParams::leaf_exit_pct), measured per scene class on MI355X:
  // testing leaves once a fifth to a third of the lanes hold one beats waiting for all of them
  // on triangle meshes (bunny-Cornell 138 -> 113 ms at 20-30 %, 124 at 10); with media in the queries 50-60 %
  // (pawn+fog 415 -> 385 ms; 30 % is no gain there); sphere-only leaves are cheapest tested all
  // together (demo1: 100 % best, 60 % +1 %)
  {
    bool spheres_only = true, static_tris = true, static_spheres = true;
    for (int j = (int)prefix.size(); j < n; ++j) {
      const rt_prim& p = sc->prims[order[j]];
      spheres_only = spheres_only && p.kind == RT_PRIM_SPHERE;
    }
    // one-class leaves: the classes of the leaves the traversal reaches through BVH nodes (the
    // surface set, and the media sets with a BVH); a medium set that is a single leaf (a fog
    // sphere) is tested by the generic test (rt_trace.h test_leaf_generic)
    for (int s = 0; s < n_sets; ++s) {
      if (s > 0 && roots[s] < 0) continue;
      for (int j = set_begin[s]; j < set_begin[s + 1]; ++j) {
        const rt_prim& p = sc->prims[order[j]];
        static_tris = static_tris && p.kind == RT_PRIM_TRIANGLE && p.motion < 0;
        static_spheres = static_spheres && p.kind == RT_PRIM_SPHERE && p.motion < 0;
      }
    }
    // the leaf tests of the BVH kernel specialised to one primitive class (rt_trace.h trav_round
    // kLeaf): bunny-Cornell 144.0 -> 139.7 ms binary64, demo1 63.9 -> 61.6 (profiles/r3/agg)
    S.leaf_kind = n == (int)prefix.size() ? 0 : static_tris ? 1 : static_spheres ? 2 : 0;
    // With media: round 5's media kernels (shading-phase events, binary64 in one 1024-lane
    // workgroup per CU with the whole pawn BVH staged, FP32 at 6 waves) re-swept with the lane-loop
    // exit below (profiles/r5/policy): FP32 leaves at 40 % and lane-loop exit 50 %, pawn+fog
    // 275.5 -> 260.5 ms; binary64 55 % and 40 %, 428.3 -> 398.9 ms (round 4: 55 / 70 and 75).
    // Sphere-only leaves: binary64 100 %; FP32 70 % since round 5 (demo1 37.73 -> 37.44 ms; binary64
    // at 70 %: +0.6 %).
    S.leaf_exit_pct = spheres_only ? 70 : sc->n_media > 0 ? 40 : 25;
    S.leaf_exit_pct64 = spheres_only ? 100 : sc->n_media > 0 ? 55 : S.leaf_exit_pct;
    if (const char* e = rt_knob("RT_AMD_LEAF_EXIT_PCT"))
      S.leaf_exit_pct = S.leaf_exit_pct64 = std::max(1, std::min(100, atoi(e)));
    // and the decoupled lane loop's exit (KernelParams::trav_exit_pct): demo1 49.2 -> 48.5 ms at 25 %
    // (round 3), the bunny flat between 50 and 75, FP32 pawn+fog best at 50 since round 5's re-sweep
    // (profiles/r5/policy; binary64 media scenes at 40 %, below)
    S.trav_exit_pct = spheres_only ? 25 : 50;
    S.trav_exit_pct64 = !spheres_only && sc->n_media > 0 ? 40 : S.trav_exit_pct;
    if (const char* e = rt_knob("RT_AMD_TRAV_PCT"))
      S.trav_exit_pct = S.trav_exit_pct64 = std::max(0, std::min(100, atoi(e)));
  }
  S.n_prims = n;
  return RT_OK;
}

int rt_host_variant(bool flat, int n_media, bool noise, bool mats, bool tex, bool inst, int leaf_kind, bool media_late,
                    int stack_depth) {
  int v = flat ? RT_VAR_FLAT : RT_VAR_BVH;
  // the BVH kernels' 1024-lane classes (rt_render_kernel.h RT_BLOCK_BVH_OF) hold RT_WIDE_STACK_ROWS
  // stack rows per lane; a deeper BVH takes the 512-lane twin of its class
  const int narrow = !flat && stack_depth + 1 > RT_WIDE_STACK_ROWS ? RT_VAR_NARROW : 0;
  // media events in the shading phase; env RT_AMD_MEDIA_LATE=0 keeps them in the traversal loop's
  // query chain (A/B, tests: the images are bit-identical)
  if (const char* e = rt_knob("RT_AMD_MEDIA_LATE")) media_late = media_late && atoi(e) != 0;
  const int late = n_media > 0 && media_late ? RT_VAR_MEDIA_LATE : 0;
  if (inst) return RT_VAR_BVH | RT_VAR_INST | (noise ? RT_VAR_NOISE : 0) | (n_media > 0 ? RT_VAR_MEDIA : 0) |
                   (mats ? RT_VAR_MATS : 0) | (tex ? RT_VAR_TEX : 0) | late | narrow;  // two-level traversal: the decoupled BVH loop
  if (const char* e = rt_knob("RT_AMD_VARIANT")) {
    const int f = atoi(e);
    // (the lockstep kernels exist only in experiment builds, RT_LOCKSTEP_KERNELS)
    const bool ok = f == RT_VAR_BVH || (RT_LOCKSTEP_KERNELS && f == RT_VAR_BVH_LOCKSTEP) || (flat && f == RT_VAR_FLAT);
    if (ok) v = f;  // flat scenes run on any variant
  }
  // one-class BVH leaves: the decoupled kernel (leaf_kind covers the leaves below BVH nodes of the
  // surface and media sets; the kernel dispatch keeps the generic test where no one-class
  // instantiation exists; env RT_AMD_LEAF_KIND=0 keeps the generic test)
  int leaf = 0;
  if (v == RT_VAR_BVH) leaf = leaf_kind == 1 ? RT_VAR_LEAF_TRI : leaf_kind == 2 ? RT_VAR_LEAF_SPHERE : 0;
  if (const char* e = rt_knob("RT_AMD_LEAF_KIND"))
    if (atoi(e) == 0) leaf = 0;
  return v | (noise ? RT_VAR_NOISE : 0) | (n_media > 0 ? RT_VAR_MEDIA : 0) | (mats ? RT_VAR_MATS : 0) |
         (tex ? RT_VAR_TEX : 0) | leaf | (v == RT_VAR_BVH ? late : 0) | narrow;
}

template <class R>
int rt_host_make_params(const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex, KernelParamsT<R>& P,
                        std::string& err) {
  if (!cs || !ex) return fail(err, RT_E_INVALID, "null argument");
  if (cs->image_width <= 0) return fail(err, RT_E_INVALID, "image width must be positive");
  if (cs->samples_per_pixel <= 0) return fail(err, RT_E_INVALID, "samples per pixel must be positive");
  if (!(cs->aspect_ratio > 0)) return fail(err, RT_E_INVALID, "aspect ratio must be positive");
  int h = rt_host_image_height(cs);
  if (h <= 0) return fail(err, RT_E_INVALID, "image height %d must be positive", h);
  // the kernels carry a pixel's column and row in 16 bits each (rt_trace.h ItemCtx)
  if (cs->image_width > 65535 || h > 65535)
    return fail(err, RT_E_UNSUPPORTED, "image %dx%d exceeds 65535 x 65535", cs->image_width, h);
  if (cs->background_kind != RT_BG_CONST && cs->background_kind != RT_BG_LERP_Y)
    return fail(err, RT_E_UNSUPPORTED, "background kind %d", cs->background_kind);
  if (cs->n_redirect_targets < 0 || cs->n_redirect_targets > RT_MAX_TARGETS)
    return fail(err, RT_E_UNSUPPORTED, "%d redirect targets (at most %d)", cs->n_redirect_targets, RT_MAX_TARGETS);
  if (cs->n_redirect_targets && !cs->redirect_targets) return fail(err, RT_E_INVALID, "null redirect targets");
  if (!finite_n(cs->center, 3) || !finite_n(cs->look_at, 3) || !finite_n(cs->up, 3) || !std::isfinite(cs->vfov) ||
      !std::isfinite(cs->focus_dist) || !std::isfinite(cs->defocus_angle))
    return fail(err, RT_E_INVALID, "non-finite camera settings");
  int rows = rt_host_shard_rows(h, ex);
  if (rows < 0) return fail(err, RT_E_INVALID, "invalid rt_exec");
  // pixel and work-item ids are 32-bit ints: one render's tile holds at most 0x7fffff00 pixels
  if ((long long)rows * cs->image_width > 0x7fffff00LL)
    return fail(err, RT_E_UNSUPPORTED, "a tile of %d x %d pixels exceeds 2^31 (split it over shards)", cs->image_width,
                rows);
  // Ray.hs:122-136, 153-155 in binary64, rounded once to R
  d3 center = D3(cs->center), look = D3(cs->look_at), up = D3(cs->up);
  double vh = cs->focus_dist * std::tan(cs->vfov / 2) * 2;
  double vw = vh * (double)cs->image_width / (double)h;
  d3 w = normalize_hs(center - look);
  d3 u = normalize_hs(cross(up, w));
  d3 v = cross(w, u);
  d3 across = smul(vw, u);
  d3 down = -smul(vh, v);
  d3 top_left = ((center - smul(cs->focus_dist, w)) - divs(across, 2)) - divs(down, 2);
  double dr = cs->focus_dist * std::tan(cs->defocus_angle / 2);
  std::memset(&P.cam, 0, sizeof P.cam);
  put3(P.cam.center, center);
  put3(P.cam.top_left, top_left);
  put3(P.cam.pixel_u, divs(across, (double)cs->image_width));
  put3(P.cam.pixel_v, divs(down, (double)h));
  put3(P.cam.disk_u, smul(dr, u));
  put3(P.cam.disk_v, smul(dr, v));
  put3(P.cam.bg0, D3(cs->background_c0));
  put3(P.cam.bg1, D3(cs->background_c1));
  P.cam.width = cs->image_width;
  P.cam.height = h;
  P.cam.spp = cs->samples_per_pixel;
  P.cam.max_depth = cs->max_recursion_depth;
  P.cam.bg_kind = cs->background_kind;
  // redirect targets (Ray.hs:138-151)
  double cum = 0, psum = 0;
  P.n_targets = cs->n_redirect_targets;
  std::memset(P.targets, 0, sizeof P.targets);
  for (int k = 0; k < cs->n_redirect_targets; ++k) {
    const rt_redirect_target& t = cs->redirect_targets[k];
    DevTargetT<R>& T = P.targets[k];
    d3 q = D3(t.q), uu = D3(t.u), vv = D3(t.v);
    d3 cp = cross(uu, vv);
    double ncp = std::sqrt(dot(cp, cp));
    if (!(ncp > 0) || !std::isfinite(t.prob)) return fail(err, RT_E_INVALID, "redirect target %d is degenerate", k);
    d3 nrm = divs(cp, ncp), nS = divs(nrm, ncp);
    put3(T.q, q);
    put3(T.u, uu);
    put3(T.v, vv);
    put3(T.n, nrm);
    put3(T.wa, cross(vv, nS));
    put3(T.wb, cross(nS, uu));
    put3(T.cr, cp);
    cum = (k == 0) ? t.prob : cum + t.prob;
    psum = (k == 0) ? t.prob : psum + t.prob;
    T.prob = (R)t.prob;
    T.thresh = (R)cum;
    T.prob_icr = (R)(t.prob / ncp);
  }
  P.rem_prob = (R)(1.0 - psum);
  P.key0 = (uint32_t)seed;
  P.key1 = (uint32_t)(seed >> 32);
  P.n_shards = ex->n_shards;
  P.shard = ex->shard;
  P.row_block = ex->row_block;
  P.tile_rows = rows;
  return RT_OK;
}

bool rt_host_media_late(const HostScene& H) {
  if (H.n_media == 0) return false;
  for (int m = 0; m < H.n_media; ++m) {  // (the roots and aliases are the same in both precisions)
    const DevMediumT<double>& M = H.f64.media[m];
    if (!M.alias_surface && !(M.root < 0 && M.root != RT_EMPTY_ROOT)) return false;
  }
  return true;
}

FastDiv rt_host_fastdiv(uint32_t d) {
  FastDiv f{0u, 0, d, 0};
  if (d <= 1) return f;
  int l = 0;
  while ((1ull << l) < d) ++l;  // ceil(log2 d)
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  f.s = l - 1;
  return f;
}

template <class R>
void rt_host_plan_work(KernelParamsT<R>& P, long long resident_lanes, bool two_sizes, bool lone) {
  P.div_width = rt_host_fastdiv((uint32_t)P.cam.width);
  P.div_block = rt_host_fastdiv((uint32_t)P.row_block);
  const bool pool_given = P.pool_shift >= 4;  // (the caller may set 4-10: 16- to 1024-id pools)
  if (!pool_given) P.pool_shift = __builtin_ctz(RT_POOL);
  P.trav_exit_pct = 50;  // the caller sets the scene's policy (HostScene::trav_exit_pct) afterwards
  // Items = (tile pixel, chunk of consecutive samples), claimed in pixel order.  Small chunks
  // keep the 64 lanes of a wave on neighbouring pixels (coherent rays) and make the queue tail
  // short; below ~2 samples the per-item commit (3 atomics) dominates.  Measured on MI355X,
  // Cornell 600x600x200 (tools/sweep_chunk.sh, an early kernel): 1 -> 14.3 ms, 2 -> 8.70, 4 -> 8.79, 8 -> 8.97,
  // 34 -> 10.3, 200 -> 16.5.  The image does not depend on this choice (fixed-point sums).
  const long long tile_pixels = (long long)P.tile_rows * P.cam.width;
  const int spp = P.cam.spp;
  // 16-sample items cut the commit atomics 4x where every lane still runs many items (bunny-
  // Cornell / pawn+fog at 1 GPU: -2.4 % / -1 %); with fewer than ~64 items per resident lane (an
  // 8-GPU rank's share, the Cornell box) the longer last items cost more than that (bunny at 8
  // shards: 20.7 -> 22.0 ms), so those keep 4.
  // The flat kernel's small (tail) items hold 3 samples since round 4 (one-wave workgroups, 5 / 8
  // waves per SIMD): Cornell 5.045 -> 4.992 ms binary64 at 1 GPU, one rank's share of 8 0.715 ->
  // 0.706, README's share of 8 0.161 -> 0.134, README at 1 GPU 0.620 -> 0.628 (+1.3 %);
  // profiles/r4/chunk_sweep.  The BVH kernels keep 4.
  const int small = two_sizes ? 3 : 4;
  int chunk = spp < small ? spp : small;
  if (resident_lanes > 0 && (long long)P.tile_rows * P.cam.width * spp / 16 >= 64 * resident_lanes) chunk = 16;
  if (const char* env = rt_knob("RT_AMD_CHUNK")) {  // tuning knob for experiments
    int c = std::atoi(env);
    if (c > 0) chunk = c;
  }
  // Big items for the bulk of the samples, small ones for the tail: the last T samples of every
  // pixel go in `chunk`-sample items, T such that the tail alone still gives every resident lane
  // `tail_items` items, and the first spp - T in as few items of at most `big` samples as cover
  // them exactly.  Two policies since the tail sample stealing (round 6, profiles/r6/sweeps/big):
  // * renders whose frames overlap (rt_render_async: the bench line) take up to 64-sample big items
  //   and 8 tail items per lane — fewer item openings and commits, and the next frame fills the
  //   longer end: Cornell binary64 4.858 -> 4.761 ms, FP32 2.950 -> 2.800, README binary64 0.407
  //   -> 0.392, the 8-GPU share unchanged (its tail covers every sample);
  // * a synchronous call's one launch ends on its last big items, so it keeps 16-sample items and
  //   16 / 32 tail items (one Cornell call 5.25 ms against 5.49 with 48-sample items).
  int big = lone ? RT_BIG_CHUNK_MAX : RT_BIG_CHUNK_MAX_ASYNC, n_big = 0;
  if (const char* env = rt_knob("RT_AMD_BIG_CHUNK")) big = std::max(1, std::atoi(env));
  int tail_items = !lone ? RT_TAIL_ITEMS_ASYNC : sizeof(R) == 8 ? RT_TAIL_ITEMS_F64 : RT_TAIL_ITEMS_F32;
  if (const char* env = rt_knob("RT_AMD_TAIL_ITEMS")) tail_items = std::atoi(env);
  if (two_sizes && chunk < big && tail_items > 0 && resident_lanes > 0 && tile_pixels > 0) {
    long long t = ((long long)tail_items * chunk * resident_lanes + tile_pixels - 1) / tile_pixels;
    if (const char* env = rt_knob("RT_AMD_TAIL_SAMPLES")) t = std::max(0, std::atoi(env));  // tests
    const long long tail = ((t + chunk - 1) / chunk) * chunk;  // tail samples, a multiple of chunk
    if (tail < spp) {
      const long long bulk = spp - tail;
      auto split = [&](int cap) {
        n_big = (int)((bulk + cap - 1) / cap);
        big = (int)((bulk + n_big - 1) / n_big);  // <= cap; n_big items cover the bulk
        big = std::min(big, spp / n_big);          // the small items cover [n_big big, spp)
      };
      split(big);
      // the waves' first pools are static (rt_render_kernel.h WaveWork): a lane's share of its
      // first pool's big items must stay below the mean work per lane, or the lanes of the first
      // waves end the frame alone (README with 26-sample items from 6 tail items: 0.39 -> 0.51 ms)
      const double per_lane = (double)spp * (double)tile_pixels / (double)resident_lanes;
      for (int pass = 0; pass < 2 && !lone; ++pass) {  // (the pool follows the item size: below)
        const int pool_items = (pool_given ? 1 << P.pool_shift : big >= 32 ? 64 : RT_POOL) / 64;
        const int cap = (int)(0.9 * per_lane / pool_items);
        if (cap >= 1 && big > cap) split(cap);
      }
      if (big <= chunk) n_big = 0;
    }
  }
  const int n_chunks = (spp - n_big * big + chunk - 1) / chunk;
  long long items = (long long)(n_big + n_chunks) * tile_pixels;
  if (items > 0x7fffff00LL) {  // keep item ids in int: one item size, grow the chunk
    n_big = 0;
    chunk = (int)((long long)spp * tile_pixels / 0x7fffff00LL) + 1;
    items = (long long)((spp + chunk - 1) / chunk) * tile_pixels;
  }
  P.chunk = chunk;
  P.n_chunks = (spp - n_big * big + chunk - 1) / chunk;
  P.big_chunk = big;
  P.n_big_chunks = n_big;
  P.big_items = (int)((long long)n_big * tile_pixels);
  P.small_start = n_big * big;
  // long big items (>= 32 samples): 64-id pools, one item per lane, so the waves' last pools are
  // even (Cornell binary64 4.760 -> 4.730 ms, FP32 2.803 -> 2.782); shorter ones keep RT_POOL ids
  // per refill (README's 17-sample items: 0.392 -> 0.402 with 64)
  if (!pool_given && !lone && n_big > 0 && big >= 32) P.pool_shift = 6;
  P.div_big = rt_host_fastdiv((uint32_t)std::max(1, n_big));
  P.div_small = rt_host_fastdiv((uint32_t)std::max(1, P.n_chunks));
  P.n_items = (int)items;
  // commit aggregation: a phase qualifies when a pool of RT_POOL consecutive ids spans at most a
  // slot's pixels (rt_render_kernel.h WaveWork); env RT_AMD_AGG=0 turns it off (A/B, same LDS)
  const int slot_pix = !two_sizes                          ? RT_AGG_PIX_BVH
                       : sizeof(R) == 8 || P.n_media == 0 ? RT_AGG_PIX_FLAT_F64  // (rt_render_kernel.h RT_AGG_WIDE_OF)
                                                          : RT_AGG_PIX_FLAT;
  const int pool = 1 << P.pool_shift;
  auto spans = [&](int n) { return n > 0 && (pool - 1 + n - 1) / n + 1 <= slot_pix; };
  bool agg = tile_pixels < (1ll << 24);  // the item's aggregation code shares its tile-pixel word
  if (const char* env = rt_knob("RT_AMD_AGG")) agg = agg && std::atoi(env) != 0;
  P.agg_big = agg && spans(n_big);
  P.agg_small = agg && spans(P.n_chunks);
}

template int rt_host_make_params<float>(const rt_camera_settings*, uint64_t, const rt_exec*, KernelParamsT<float>&,
                                        std::string&);
template int rt_host_make_params<double>(const rt_camera_settings*, uint64_t, const rt_exec*, KernelParamsT<double>&,
                                         std::string&);
template void rt_host_plan_work<float>(KernelParamsT<float>&, long long, bool, bool);
template void rt_host_plan_work<double>(KernelParamsT<double>&, long long, bool, bool);

// The 8-bit code thresholds of writeImage / writeImageSqrt's quantisation (rt_encode8_table.h,
// generated with the transfer evaluated exactly; raytrace_amd.ray.encode8 reads the same table).
void rt_host_encode8_thresholds(int encoding, double* thr) {
  const double* t = encoding == 1 ? kEnc8Sqrt : kEnc8Srgb;
  for (int k = 0; k < 256; ++k) thr[k] = t[k];
}
