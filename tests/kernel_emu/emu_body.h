// emu_body.h — TEST TOOLING: the host emulator's render loop for ONE precision (included by
// rt_emu.cpp once per precision, after rt_trace.h of the same RT_F64).

struct Shared {
  const RT_NS::KernelParams* P;
  int variant;
  std::atomic<int> next{0};
  std::atomic<int> overflow{0};
  std::vector<std::atomic<long long>>* accum;
  std::vector<std::atomic<unsigned>>* flags;
  std::atomic<long long> cnt[4];
};

// the device kernel's WaveWork without waves: one shared counter, every item committed directly
struct Work {
  Shared* s;
  int grab(bool need, int& slot) {
    slot = -1;
    return need ? s->next.fetch_add(1) : 0;
  }
  int tag(int tp, int slot) const {
    (void)slot;
    return tp;
  }
  template <class AccT>
  void commit(bool c, int tp, const AccT& acc, bool bad) {
    if (!c) return;
    const RT_NS::Acc A = RT_NS::acc_words(acc);
    const size_t w = RT_ACC_WORDS(RT_NS::real);
    for (int k = 0; k < 3; ++k) (*s->accum)[w * (size_t)tp + k] += A.hi[k];
#if RT_F64
    for (int k = 0; k < 3; ++k) (*s->accum)[w * (size_t)tp + 3 + k] += (long long)A.lo[k];
#endif
    if (bad) (*s->flags)[tp] |= 1u;
  }
};

template <int kTex, int kMedia, bool kMats, class G>
int run_loop(const RT_NS::KernelParams& P, int variant, G& g, const RT_NS::Trav& W) {
  // the item sums through the device kernels' LDS accumulator (one lane: stride 1)
  unsigned long long words[6] = {0, 0, 0, 0, 0, 0};
  RT_NS::AccLds acc{words, 1};
  if (variant & RT_VAR_INST) return RT_NS::lane_loop_bvh<kTex, kMedia, kMats, true, 0>(P, g, W, P.prims, acc);
  if ((variant & RT_VAR_BASE) == RT_VAR_BVH) {  // one-class leaves, as the device kernels
    if (variant & RT_VAR_LEAF_TRI) return RT_NS::lane_loop_bvh<kTex, kMedia, kMats, false, 1>(P, g, W, P.prims, acc);
    if ((variant & RT_VAR_LEAF_SPHERE) && !kMedia)
      return RT_NS::lane_loop_bvh<kTex, kMedia, kMats, false, 2>(P, g, W, P.prims, acc);
  }
  switch (variant & RT_VAR_BASE) {
    case RT_VAR_FLAT: return RT_NS::lane_loop_lockstep<true, kTex, kMedia != 0, kMats>(P, g, W, P.prims, acc);
    case RT_VAR_BVH_LOCKSTEP:
      return RT_NS::lane_loop_lockstep<false, kTex, kMedia != 0, kMats>(P, g, W, P.prims, acc);
    default: return RT_NS::lane_loop_bvh<kTex, kMedia, kMats, false, 0>(P, g, W, P.prims, acc);
  }
}
template <int kTex, class G>
int run_flags(const RT_NS::KernelParams& P, int variant, G& g, const RT_NS::Trav& W) {
  const int base = variant;
  const bool media = (variant & RT_VAR_MEDIA) != 0, mats = (variant & RT_VAR_MATS) != 0;
  // kMedia as the device kernels (rt_render_kernel.h RT_MEDIA_OF): 2 media events in the shading phase
  if (media && (variant & RT_VAR_MEDIA_LATE) && (variant & RT_VAR_BASE) == RT_VAR_BVH)
    return mats ? run_loop<kTex, 2, true>(P, base, g, W) : run_loop<kTex, 2, false>(P, base, g, W);
  if (media) return mats ? run_loop<kTex, 1, true>(P, base, g, W) : run_loop<kTex, 1, false>(P, base, g, W);
  return mats ? run_loop<kTex, 0, true>(P, base, g, W) : run_loop<kTex, 0, false>(P, base, g, W);
}
template <class G>
int run_variant(const RT_NS::KernelParams& P, int variant, G& g, const RT_NS::Trav& W) {
  if (variant & RT_VAR_NOISE) return run_flags<2>(P, variant, g, W);
  if (variant & RT_VAR_TEX) return run_flags<1>(P, variant, g, W);
  return run_flags<0>(P, variant, g, W);
}

void* worker(void* arg) {
  Shared* s = (Shared*)arg;
  std::vector<int> stack(s->P->stack_depth + 1);
  for (auto& c : rt_emu::counters) c = 0;
  Work g{s};
  const RT_NS::Trav W{stack.data(), 1, nullptr};  // the emulator reads every node from memory
  int ov = run_variant(*s->P, s->variant, g, W);
  if (ov) s->overflow = 1;
  for (int i = 0; i < 4; ++i) s->cnt[i] += rt_emu::counters[i];
  return nullptr;
}

// one render of the host scene in this precision; out: tile_rows x width x 3 reals
int render(const HostScene& H, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex, RT_NS::real* out,
           int nthreads, int chunk, long long* counters, std::string& err) {
  using real = RT_NS::real;
  const HostArraysT<real>& A = H.arrays<real>();
  RT_NS::KernelParams P = {};
  int rc = rt_host_make_params(cs, seed, ex, P, err);
  if (rc) return rc;
  P.nodes = H.nodes.data();
  P.prims = A.prims.data();
  P.prim_shade = A.prim_shade.data();
  P.prim_uv = A.prim_uv.data();
  P.mats = A.mats.data();
  P.texs = A.texs.data();
  P.motions = A.motions.data();
  P.uvframes = A.uvframes.data();
  P.texels = A.texels.data();
  P.perlin_perm = H.perlin_perm.data();
  P.perlin_grad = A.perlin_grad.data();
  P.flat_recs = A.flat_recs.data();
  P.boxes = A.boxes.data();
  P.instances = A.instances.data();
  P.out = out;
  P.surface_root = H.surface_root;
  P.leaf_exit_pct = RT_F64 ? H.leaf_exit_pct64 : H.leaf_exit_pct;
  P.surface_prefix = H.flat ? 0 : 1;
  P.n_media = H.n_media;
  for (int k = 0; k < H.n_media; ++k) P.media[k] = A.media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) P.flat_sets[k] = H.flat_sets[k];
  P.stack_depth = H.max_depth > 1 ? H.max_depth : 1;
  P.n_prims = H.n_prims;
  const int variant = rt_host_variant(H.flat, H.n_media, H.noise, H.full_mats, H.uv_tex, H.n_instances > 0, H.leaf_kind,
                                      rt_host_media_late(H), H.max_depth > 1 ? H.max_depth : 1);
  rt_host_plan_work(P, 4096, (variant & RT_VAR_BASE) == RT_VAR_FLAT);
  P.trav_exit_pct = RT_F64 ? H.trav_exit_pct64 : H.trav_exit_pct;
  if (chunk > 0) {
    P.chunk = chunk;
    P.n_chunks = (P.cam.spp + chunk - 1) / chunk;
    P.n_big_chunks = 0;
    P.big_items = 0;
    P.small_start = 0;
    P.div_small = rt_host_fastdiv((uint32_t)P.n_chunks);
    P.n_items = P.n_chunks * P.tile_rows * P.cam.width;
  }
  const size_t tile_pixels = (size_t)P.tile_rows * P.cam.width;
  const size_t w = RT_ACC_WORDS(real);
  std::vector<std::atomic<long long>> accum(tile_pixels * w);
  std::vector<std::atomic<unsigned>> flags(tile_pixels);
  for (auto& a : accum) a = 0;
  for (auto& f : flags) f = 0;
  Shared s;
  s.P = &P;
  s.variant = variant;
  s.accum = &accum;
  s.flags = &flags;
  for (auto& c : s.cnt) c = 0;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pthread_t th[64];
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], nullptr, worker, &s);
  worker(&s);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], nullptr);
  for (size_t i = 0; i < tile_pixels; ++i)
    for (int c = 0; c < 3; ++c) {
      const long long hi = accum[w * i + c].load();
#if RT_F64
      // as rt_render_kernel.h rt_resolve_kernel
      const double lo = (double)(unsigned long long)accum[w * i + 3 + c].load();
      const double sum = ((double)hi + lo * (1.0 / RT_FIX_SCALE)) * (1.0 / RT_FIX_SCALE);
      out[3 * i + c] = flags[i] ? NAN : sum / (double)P.cam.spp;
#else
      out[3 * i + c] = flags[i] ? NAN : (float)((double)hi * (1.0 / (RT_FIX_SCALE * (double)P.cam.spp)));
#endif
    }
  if (counters) {
    for (int i = 0; i < 3; ++i) counters[i] = s.cnt[i];
    counters[3] = (long long)tile_pixels * P.cam.spp;
  }
  if (s.overflow) {
    err = "BVH traversal stack overflow";
    return RT_E_STACK;
  }
  return RT_OK;
}
