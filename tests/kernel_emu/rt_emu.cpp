// rt_emu.cpp — TEST TOOLING: the device logic of raytrace_amd/csrc/rt_trace.h compiled for
// the host, so the kernel's algorithm can be checked against the FP64 oracle without a GPU
// and kernel faults can be reproduced on the CPU.  Never linked into librt_amd.so.
#define RT_HOST_EMU 1
#include <pthread.h>

#include <atomic>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../raytrace_amd/csrc/rt_internal.h"
#include "../../raytrace_amd/csrc/rt_trace.h"

namespace rt_emu {
thread_local long long counters[4];
}

namespace {
thread_local std::string g_err;

struct Shared {
  const KernelParams* P;
  int variant;
  std::atomic<int> next{0};
  std::atomic<int> overflow{0};
  std::vector<std::atomic<long long>>* accum;
  std::vector<std::atomic<unsigned>>* flags;
  std::atomic<long long> cnt[4];
};

struct Grab {
  Shared* s;
  int operator()(bool need) { return need ? s->next.fetch_add(1) : 0; }
};
struct Commit {
  Shared* s;
  void operator()(int tp, long long x, long long y, long long z, bool bad) {
    (*s->accum)[3 * (size_t)tp] += x;
    (*s->accum)[3 * (size_t)tp + 1] += y;
    (*s->accum)[3 * (size_t)tp + 2] += z;
    if (bad) (*s->flags)[tp] |= 1u;
  }
};

template <int kTex, bool kMedia, bool kMats, class G, class Cm>
int run_loop(const KernelParams& P, int base, G& g, Cm& c, const rtk::Trav& W) {
  switch (base) {
    case RT_VAR_FLAT: return rtk::lane_loop_lockstep<true, kTex, kMedia, kMats>(P, g, c, W, P.prims);
    case RT_VAR_BVH_LOCKSTEP: return rtk::lane_loop_lockstep<false, kTex, kMedia, kMats>(P, g, c, W, P.prims);
    default: return rtk::lane_loop_bvh<kTex, kMedia, kMats>(P, g, c, W, P.prims);
  }
}
template <int kTex, class G, class Cm>
int run_flags(const KernelParams& P, int variant, G& g, Cm& c, const rtk::Trav& W) {
  const int base = variant & RT_VAR_BASE;
  const bool media = (variant & RT_VAR_MEDIA) != 0, mats = (variant & RT_VAR_MATS) != 0;
  if (media) return mats ? run_loop<kTex, true, true>(P, base, g, c, W) : run_loop<kTex, true, false>(P, base, g, c, W);
  return mats ? run_loop<kTex, false, true>(P, base, g, c, W) : run_loop<kTex, false, false>(P, base, g, c, W);
}
template <class G, class Cm>
int run_variant(const KernelParams& P, int variant, G& g, Cm& c, const rtk::Trav& W) {
  if (variant & RT_VAR_NOISE) return run_flags<2>(P, variant, g, c, W);
  if (variant & RT_VAR_TEX) return run_flags<1>(P, variant, g, c, W);
  return run_flags<0>(P, variant, g, c, W);
}

void* worker(void* arg) {
  Shared* s = (Shared*)arg;
  std::vector<int> stack(s->P->stack_depth + 1);
  for (auto& c : rt_emu::counters) c = 0;
  Grab g{s};
  Commit c{s};
  const rtk::Trav W{stack.data(), 1, nullptr};  // the emulator reads every node from memory
  int ov = 0;
  ov = run_variant(*s->P, s->variant, g, c, W);
  if (ov)
    s->overflow = 1;
  for (int i = 0; i < 4; ++i) s->cnt[i] += rt_emu::counters[i];
  return nullptr;
}
}  // namespace

extern "C" {
const char* rt_emu_last_error(void) { return g_err.c_str(); }

// counters (optional, 4 values): BVH nodes visited, primitives tested, segments, samples
int rt_emu_render(const rt_camera_settings* cs, const rt_scene* sc, uint64_t seed, const rt_exec* ex, float* out,
                  int nthreads, int chunk, long long* counters) {
  HostScene H;
  int rc = rt_host_build_scene(sc, H, g_err);
  if (rc) return rc;
  KernelParams P = {};
  rc = rt_host_make_params(cs, seed, ex, P, g_err);
  if (rc) return rc;
  P.nodes = H.nodes.data();
  P.prims = H.prims.data();
  P.prim_shade = H.prim_shade.data();
  P.prim_uv = H.prim_uv.data();
  P.mats = H.mats.data();
  P.texs = H.texs.data();
  P.motions = H.motions.data();
  P.uvframes = H.uvframes.data();
  P.texels = H.texels.data();
  P.perlin_perm = H.perlin_perm.data();
  P.perlin_grad = H.perlin_grad.data();
  P.flat_recs = H.flat_recs.data();
  P.boxes = H.boxes.data();
  P.out = out;
  P.surface_root = H.surface_root;
  P.leaf_exit_pct = H.leaf_exit_pct;
  P.surface_prefix = H.flat ? 0 : 1;
  P.n_media = H.n_media;
  for (int k = 0; k < H.n_media; ++k) P.media[k] = H.media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) P.flat_sets[k] = H.flat_sets[k];
  P.stack_depth = H.max_depth > 1 ? H.max_depth : 1;
  P.n_prims = H.n_prims;
  rt_host_plan_work(P, 4096);
  P.trav_exit_pct = H.trav_exit_pct;
  if (chunk > 0) {
    P.chunk = chunk;
    P.n_chunks = (P.cam.spp + chunk - 1) / chunk;
    P.n_items = P.n_chunks * P.tile_rows * P.cam.width;
  }
  const size_t tile_pixels = (size_t)P.tile_rows * P.cam.width;
  std::vector<std::atomic<long long>> accum(tile_pixels * 3);
  std::vector<std::atomic<unsigned>> flags(tile_pixels);
  for (auto& a : accum) a = 0;
  for (auto& f : flags) f = 0;
  Shared s;
  s.P = &P;
  s.variant = rt_host_variant(H.flat, H.n_media, H.noise, H.full_mats, H.uv_tex);
  s.accum = &accum;
  s.flags = &flags;
  for (auto& c : s.cnt) c = 0;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pthread_t th[64];
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], nullptr, worker, &s);
  worker(&s);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], nullptr);
  const double scale = 1.0 / (RT_FIX_SCALE * (double)P.cam.spp);
  for (size_t i = 0; i < tile_pixels; ++i)
    for (int c = 0; c < 3; ++c)
      out[3 * i + c] = flags[i] ? NAN : (float)((double)accum[3 * i + c].load() * scale);
  if (counters) {
    for (int i = 0; i < 3; ++i) counters[i] = s.cnt[i];
    counters[3] = (long long)tile_pixels * P.cam.spp;
  }
  if (s.overflow) {
    g_err = "BVH traversal stack overflow";
    return RT_E_STACK;
  }
  return RT_OK;
}
}

extern "C" {
// scene summary of the host build (test tooling): n_nodes, surface_nodes, max_depth, n_prims, flat
int rt_emu_scene_info(const rt_scene* sc, int* info) {
  HostScene H;
  int rc = rt_host_build_scene(sc, H, g_err);
  if (rc) return rc;
  info[0] = H.n_nodes;
  info[1] = H.surface_nodes;
  info[2] = H.max_depth;
  info[3] = H.n_prims;
  info[4] = H.flat ? 1 : 0;
  info[5] = (int)H.boxes.size();
  // BVH scenes: primitives tested before the surface BVH (prefix records + box-group faces)
  int pre = 0;
  if (!H.flat) {
    const DevFlatSet& F = H.flat_sets[0];
    pre = F.end - F.first;
    for (int b = F.box_first; b < F.box_end; ++b)
      for (int f = 0; f < 6; ++f) pre += ((H.boxes[b].ord_code >> (5 * f)) & 31) != RT_BOX_NO_FACE;
  }
  info[6] = pre;
  return RT_OK;
}
}
