// rt_render_kernel.h — the persistent path-tracing megakernel, the fixed-point resolve and
// their launchers for ONE precision: included by rt_kernel.hip (RT_F64 0, float) and
// rt_kernel64.hip (RT_F64 1, binary64), each its own translation unit (built in parallel).
// The per-lane logic lives in rt_trace.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rt_trace.h"

// Where the lanes' item sums live (rt_trace.h Acc / AccLds).  Same-box A/B against registers
// (profiles/r3/slim): in LDS they free the VGPRs that let the FP32 BVH kernel without media run 6
// waves per SIMD (bunny-Cornell 107.2 -> 100.6 ms) and trim the binary64 BVH kernels (bunny 162.7
// -> 157.6, pawn+fog 643 -> 631); the flat kernels, which read their scene with scalar loads that
// share the LDS return counter, lose 2-3.5 % (Cornell f64 6.12 -> 6.33) and the FP32 media kernel
// 2.8 %, so those keep registers.  -DRT_ACC_IN_LDS=0 keeps registers everywhere.
#ifndef RT_ACC_IN_LDS
#define RT_ACC_IN_LDS 1
#endif
#define RT_ACC_LDS_OF(kVar, kMedia) (RT_ACC_IN_LDS && (kVar) != RT_VAR_FLAT && (RT_F64 || !(kMedia)))

namespace RT_NS {

// Diagnostic build only (make exp DEFS=-DRT_WAVE_STAMPS, tools/wave_stamps.py): per wave the
// wall clock (s_memrealtime, 100 MHz) at its start, when its grab first finds every queue spent
// (the queue has drained: from then on the wave only finishes the items it holds) and at its end,
// and its hardware id — the ramp and the tail of one launch, wave by wave.
#if defined(RT_WAVE_STAMPS)
#define RT_STAMP_WAVES 16384
static __device__ unsigned long long rt_stamp_buf[4 * RT_STAMP_WAVES];  // (one per translation unit)
#endif

namespace {

// Item claims.  A wave keeps a pool of consecutive item ids in SGPRs (wave-uniform state) and
// refills it with ONE returning atomicAdd of RT_POOL ids, so the global head word sees one
// atomic per RT_POOL claims instead of one per refilling wave-iteration (a single word saturates at
// ~88 returning atomics per microsecond, MI355X_MICROARCH.md "dequeue").  Lanes that need work
// take ids in lane order; ids are never dropped (a pool is contiguous and increasing, so once a
// lane draws an id >= n_items every later id is out of range too).
static_assert(RT_POOL >= 64, "a refill must cover every lane of a wave");
// The dynamic ids [offset, n_items) are split into RT_QUEUES contiguous ranges, each with its own
// head word (256 B apart): a wave starts on queue (wave % RT_QUEUES) and moves to the next one
// when its queue is spent, so each word sees 1 / RT_QUEUES of the refills.  Measured (kernel ms,
// 1 / 2 / 4 / 8 queues): README 0.315 / 0.282 / 0.285 / 0.29 (its cheap samples ran the single
// word near its returning-atomic rate), README on 2 GPUs 0.191 / 0.189 / 0.177 / 0.180, Cornell
// 3.455 / 3.42 / 3.42 / 3.43, Cornell's 8-GPU share 0.520 / 0.517 / 0.517 / 0.519.
#ifndef RT_QUEUES
#define RT_QUEUES 4
#endif
// How the queues split the dynamic ids.  Contiguous quarters (0, rounds 3-4) put the big items
// (the first ids) in the first queues and the small tail items in the last: the waves of a spent
// queue move on to the next, so the frame ENDED on the big items of the last queue to drain — the
// per-wave stamps of one binary64 Cornell launch (tools/wave_stamps.py, profiles/r5/) showed the
// queue drained at 4.78 ms and the last wave ending 1.30 ms later.  Interleaved pools (1): queue q
// serves pools q, q + RT_QUEUES, ... of RT_POOL ids, so every queue walks the ids in order and the
// tail items come last, as rt_host_plan_work intends.
#ifndef RT_QUEUE_INTERLEAVE
#define RT_QUEUE_INTERLEAVE 1
#endif
static_assert((RT_QUEUES & (RT_QUEUES - 1)) == 0 && RT_QUEUES <= 8, "RT_QUEUES: a power of two, at most 8 (workspace)");
// Per-wave commit aggregation.  Ids are pixel-major (rt_trace.h open_item), so the RT_POOL
// consecutive ids of one pool cover a few pixels: when a pool is opened the wave gives it one of
// its kSlots LDS slots (kPix pixels x RT_ACC_WORDS words, pixel-major like `accum`, plus a header:
// ids still open, first tile pixel; the item carries slot + 1, rt_trace.h ItemCtx).  A finished
// item adds its words to the slot with LDS atomics instead of 64-bit atomics to HBM and counts
// its id off; once a pool's ids are all committed the wave adds the slot's words to `accum` —
// consecutive addresses, one atomic per nonzero word per (pixel, pool) instead of per item — and
// frees the slot (lazily: when a new pool finds no free slot, and at the end).  A slot belongs to one wave
// (so no synchronisation beyond the wave's own LDS order); the ids of a pool are claimed by that
// wave only.  Pools the host did not qualify (a phase with few chunks per pixel, the pool that
// straddles the two item sizes) or that find every slot busy commit directly, as before.  Integer
// sums: the image is bit-identical either way.
// (keeping the item's pixel offset within the slot in its code, resolved at the item's start
// instead of one LDS read at its commit, measured no faster: Cornell f64 5.77 vs 5.74 ms)
static_assert(RT_AGG_SLOTS_FLAT < 255 && RT_AGG_SLOTS_FLAT_F64 < 255 && RT_AGG_SLOTS_BVH < 255,
              "slot + 1 must fit the 8 bits of rt_trace.h ItemCtx::tp");

// LDS of the aggregation slots per wave: kSlots x kPix x RT_ACC_WORDS words + 2 kSlots header ints
template <int kSlots, int kPix>
struct AggGeom {
  static constexpr int kWords = kPix * RT_ACC_WORDS(real);  // 64-bit words per slot
  static constexpr int kWaveBytes = kSlots * kWords * 8 + 2 * kSlots * 4;
};

// The work queue of the flat kernels re-reads its kernel-argument fields at each use; the BVH
// kernels' does in FP32 only (binary64 demo1 / pawn+fog -0.7 % with them held, Cornell's flat
// binary64 kernel +0.7 %: profiles/r4/kargs_phase_ab, r4/pp_ab)
#ifndef RT_KARGS_WORK_BVH
#define RT_KARGS_WORK_BVH (!RT_F64)
#endif
// kReread: the queue's kernel-argument fields re-read at each use (rt_trace.h RT_KARGS) or held
template <int kSlots, int kPix, bool kReread>
struct WaveWork {
  const KernelParams& P;
  // item claims: a pool of consecutive ids in SGPRs (wave-uniform state), refilled with ONE
  // returning atomicAdd of RT_POOL ids, so the head word sees one atomic per RT_POOL claims (a
  // single word saturates at ~88 returning atomics per microsecond, MI355X_MICROARCH.md
  // "dequeue").  Lanes that need work take ids in lane order; ids are never dropped (a pool is
  // contiguous and increasing, so once a lane draws an id >= n_items every later id is too).
  int pool;    // ids per pool: 1 << kp().pool_shift (the host's choice per launch, RT_POOL by default)
  int pool_base;
  int pool_left;
  int offset;  // ids [0, offset) are the waves' initial pools, handed out without atomics
  int queue;   // the queue this wave refills from
  int spent;   // queues found spent (RT_QUEUES: every id is claimed)
  int pool_slot;  // the current pool's slot (-1: direct commits)
  // aggregation: this wave's slots [kSlots][kWords] and header [open ids x kSlots, tplo x kSlots]
  unsigned long long* slots;
  int* hdr;
  unsigned free_mask;  // wave-uniform
#if defined(RT_WAVE_STAMPS)
  unsigned long long t_drain = 0;  // wall clock when every queue was first found spent
#endif
  // the kernel arguments re-read where used (rt_trace.h RT_KARGS): not held across the lane loop
  __device__ __forceinline__ const KernelParams& kp() const { return RT_KARGS_IF(kReread, P); }

  __device__ __forceinline__ WaveWork(const KernelParams& P_, int wave, int waves, unsigned long long* slots_)
      : P(P_), pool(1 << P_.pool_shift), pool_base(wave * pool), pool_left(pool), offset(waves * pool),
        queue(wave & (RT_QUEUES - 1)),
        spent(0), pool_slot(-1), slots(slots_),
        hdr(reinterpret_cast<int*>(slots_ + kSlots * AggGeom<kSlots, kPix>::kWords)),
        free_mask(kSlots > 0 ? (1u << kSlots) - 1u : 0u) {
#if defined(RT_NO_STATIC_POOLS)
    // (experiment: every pool from the queues, none by wave index)
    pool_left = 0;
    offset = 0;
#else
    // every wave starts with a static pool (its wave index x pool): at launch all resident
    // waves would otherwise queue up on the counter at once (~80 us at ~88 returning atomics per us)
    pool_slot = open_pool(pool_base, min(pool, P.n_items - pool_base));
#endif
  }

  // a slot for the pool of ids [b0, b0 + cnt) (wave-uniform), or -1: commit its items directly.
  // Slots are reclaimed here, lazily: when none is free, every slot whose ids are all committed
  // is flushed (so the commit path itself never waits on an LDS return or branches to a flush)
  __device__ __forceinline__ int open_pool(int b0, int cnt) {
    if (kSlots == 0 || cnt <= 0) return -1;
    const bool big = b0 < kp().big_items;
    if (big ? (!kp().agg_big || b0 + cnt > kp().big_items) : !kp().agg_small) return -1;
    if (free_mask == 0u) reclaim();
    if (free_mask == 0u) return -1;
    const int tplo = (int)fast_div((uint32_t)(big ? b0 : b0 - kp().big_items), big ? kp().div_big : kp().div_small);
    const int s = __builtin_ctz(free_mask);
    free_mask &= free_mask - 1u;
    hdr[s] = cnt;  // every active lane stores the same words
    hdr[kSlots + s] = tplo;
    return s;
  }
  __device__ __forceinline__ void reclaim() {
#pragma unroll 1
    for (int s = 0; s < kSlots; ++s)
      if (__builtin_amdgcn_readfirstlane(hdr[s]) == 0) flush(s);
  }
  // after the lane loop (every lane of the wave back): flush the slots still held
  __device__ __forceinline__ void finish() {
#pragma unroll 1
    for (int s = 0; s < kSlots; ++s)
      if (!((free_mask >> s) & 1u)) flush(s);
  }

  // wave-collective: a fresh item for lanes with need (n_items once every id is claimed), with
  // its pool's slot
  __device__ __forceinline__ int grab(bool need, int& slot) {
    slot = pool_slot;
    const unsigned long long m = __ballot(need);
    if (m == 0ull) return 0;
    const int lane = (int)__lane_id();
    const int cnt = (int)__popcll(m);
    const int rank = (int)__popcll(m & ((1ull << lane) - 1ull));
    if (pool_left >= cnt) {
      const int item = pool_base + rank;
      pool_base += cnt;
      pool_left -= cnt;
      return item;
    }
    // ranks [0, pool_left) drain the pool; the others are served by refills, in rank order
    const int n_items = kp().n_items;
    int item = rank < pool_left ? pool_base + rank : n_items;
    int first = pool_left, rest = cnt - pool_left;
    pool_left = 0;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int dyn = n_items - offset;
#if RT_QUEUE_INTERLEAVE
    const int n_pools = dyn > 0 ? (dyn + pool - 1) / pool : 0;
#else
    const int len = dyn > 0 ? (dyn + RT_QUEUES - 1) / RT_QUEUES : 0;
#endif
    while (rest > 0 && spent < RT_QUEUES) {
#if RT_QUEUE_INTERLEAVE
      // queue q hands out the dynamic pools q, q + RT_QUEUES, q + 2 RT_QUEUES, ... (one counter
      // increment per pool): the ids are claimed in (nearly) global order whatever queue a wave
      // draws from, so the frame ends with the last, smallest items
      int pk = 0;
      if (lane == leader) pk = atomicAdd(kp().counter + 64 * queue, 1);
      pk = __builtin_amdgcn_readfirstlane(__shfl(pk, leader));
      const int qs = offset, qlen = dyn;
      if (pk * RT_QUEUES + queue >= n_pools) {  // spent: the queue's next pool is past the last one
#else
      const int qs = offset + queue * len;
      const int qlen = min(len, n_items - qs);  // <= 0 for an empty last queue
      int base = 0;
      if (lane == leader) base = atomicAdd(kp().counter + 64 * queue, pool);
      base = __builtin_amdgcn_readfirstlane(__shfl(base, leader));
      if (base >= qlen) {  // spent: ids are only ever handed out below qlen
#endif
        queue = (queue + 1) & (RT_QUEUES - 1);
        ++spent;
#if defined(RT_WAVE_STAMPS)
        if (spent == RT_QUEUES && t_drain == 0) t_drain = wall_clock64();
#endif
        continue;
      }
#if RT_QUEUE_INTERLEAVE
      const int base = (pk * RT_QUEUES + queue) * pool;
#endif
      const int avail = min(pool, qlen - base);
      const int take = min(rest, avail);
      pool_slot = open_pool(qs + base, avail);
      if (rank >= first && rank < first + take) {
        item = qs + base + (rank - first);
        slot = pool_slot;
      }
      first += take;
      rest -= take;
      pool_base = qs + base + take;
      pool_left = avail - take;
      if (rest > 0) {  // the pool ended at the queue's end (interleaved: the last, short pool)
        queue = (queue + 1) & (RT_QUEUES - 1);
        ++spent;
      }
    }
    return item;
  }

  // wave-collective: lanes with c add their finished item's fixed-point sums (rt_trace.h Acc:
  // [hi.xyz] or [hi.xyz, lo.xyz]; zero words are skipped) to its pool's slot, or to `accum`
  __device__ __forceinline__ void direct(int tp, const Acc& A) const {
    unsigned long long* a = kp().accum + RT_ACC_WORDS(real) * (size_t)tp;
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (A.hi[c]) atomicAdd(a + c, (unsigned long long)A.hi[c]);
#if RT_F64
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (A.lo[c]) atomicAdd(a + 3 + c, A.lo[c]);
#endif
  }
  // an item's tile pixel tagged with its slot code in bits 24-31 (rt_trace.h ItemCtx::tp): slot +
  // 1, or 0 for direct commits.  The code exists only in launches that aggregate (kp().agg_big |
  // kp().agg_small, set by the host for tiles below 2^24 pixels); elsewhere the word is the plain tile
  // pixel, whose bits 24-30 may be set (tiles up to 2^31 pixels), and commit must not decode it
  __device__ __forceinline__ bool aggregating() const { return kSlots > 0 && (kp().agg_big | kp().agg_small) != 0; }
  // an item's plain tile pixel (its slot code cleared; rt_trace.h steal_sample)
  __device__ __forceinline__ int untag(int tpk) const { return aggregating() ? (tpk & 0xffffff) : tpk; }
  __device__ __forceinline__ int tag(int tp, int slot) const {
    if (slot < 0) return tp;
    return tp | ((slot + 1) << 24);
  }
  template <class AccT>
  __device__ __forceinline__ void commit(bool c, int tpk, const AccT& acc, bool bad) {
    if (!c) return;
    const int code = aggregating() ? (int)((uint32_t)tpk >> 24) : 0;
    const int tp = code ? tpk & 0xffffff : tpk;
    const Acc A = acc_words(acc);
    if (code == 0) {
      direct(tp, A);
    } else {
      const int s = code - 1;
      unsigned long long* w = slots + s * AggGeom<kSlots, kPix>::kWords + (tp - hdr[kSlots + s]) * RT_ACC_WORDS(real);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (A.hi[k]) lds_add(w + k, (unsigned long long)A.hi[k]);
#if RT_F64
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (A.lo[k]) lds_add(w + 3 + k, A.lo[k]);
#endif
      __hip_atomic_fetch_add(hdr + s, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // no return
    }
    if (bad) atomicOr(kp().nanflag + tp, 1u);
  }
  // add a closed slot's words to `accum` (consecutive pixels: consecutive addresses) and free it
  __device__ __forceinline__ void flush(int s) {
    constexpr int kW = AggGeom<kSlots, kPix>::kWords;
    const unsigned long long act = __ballot(true);
    const int k = (int)__popcll(act);
    const int r = (int)__popcll(act & ((1ull << __lane_id()) - 1ull));
    const int tplo = __builtin_amdgcn_readfirstlane(hdr[kSlots + s]);
    const long long g0 = (long long)tplo * RT_ACC_WORDS(real);
    const long long g_end = (long long)kp().tile_rows * kp().cam.width * RT_ACC_WORDS(real);
    unsigned long long* w = slots + s * kW;
    for (int j = r; j < kW; j += k) {
      const unsigned long long v = w[j];
      if (v != 0ull) {
        w[j] = 0ull;
        if (g0 + j < g_end) atomicAdd(kp().accum + g0 + j, v);
      }
    }
    free_mask |= 1u << s;
  }
};

}  // namespace

// Variants (rt_internal.h RT_VAR_*), chosen per scene by the host:
//  RT_VAR_FLAT: every primitive set is one flat leaf; no LDS: the records are read with
//    wave-uniform addresses (scalar loads into SGPRs, scalar-cache resident); lockstep loop.
//  RT_VAR_BVH / RT_VAR_BVH_LOCKSTEP: BVH scenes; dynamic LDS = the lanes' traversal stacks
//    [depth][lane] followed by the top P.lds_nodes nodes.  The default decouples traversal
//    from shading per lane (rt_trace.h lane_loop_bvh); the lockstep loop runs every query of a
//    segment with the whole wave (kept for experiments; images are bit-identical).
// Register budget: occupancy floor (waves per SIMD), per kernel class and precision — the table
// below (RT_WAVES_OF), each entry measured against its neighbours (DESIGN_HISTORY §1a,
// §4).  Since round 6 every entry also keeps its class free of VGPR spills (tools/spill_gate.py
// fails the build otherwise): the binary64 full-material BVH classes, the binary64 instanced
// full-material class, the FP32 full-material generic-leaf class and the FP32 instanced media-chain
// classes each run one wave less than their round-5 entries.
#ifndef RT_WAVES_FLAT
#define RT_WAVES_FLAT 7
#endif
#ifndef RT_WAVES_FLAT_NOISE
#define RT_WAVES_FLAT_NOISE 5
#endif
#ifndef RT_WAVES_BVH
#define RT_WAVES_BVH 5
#endif
// knobs for the lightest instantiations (constant textures; BVH: no media).  The flat kernel with
// constant textures runs 8 waves since round 4: with the kernel arguments re-read per iteration
// (rt_trace.h RT_KARGS) and shade's unconditional ray update it needs 64 VGPRs without spills
// (Cornell FP32 3.162 -> 3.075 ms against 7 waves, profiles/r4/unc_ab); round 3's 8-wave build
// spilled 6 VGPRs and gained nothing
#ifndef RT_WAVES_FLAT_TEX0
#define RT_WAVES_FLAT_TEX0 8
#endif
#ifndef RT_WAVES_BVH_LITE
#define RT_WAVES_BVH_LITE 6  // 80 VGPRs once the item sums moved to LDS: bunny-Cornell 107.2 -> 100.6 ms at 6 (profiles/r3/slim)
#endif
// binary64: every real is a register pair, so the same code needs about twice the VGPRs; the
// lightest instantiations (constant textures, no media, no materials beyond the diffuse ones)
// keep more waves
#ifndef RT_WAVES64_FLAT_LITE
#define RT_WAVES64_FLAT_LITE 5  // 96 VGPRs, no spills (round 4): Cornell binary64 5.442 -> 5.315 ms against 4
#endif
#ifndef RT_WAVES64_FLAT
#define RT_WAVES64_FLAT 4  // 100 VGPRs without MachineLICM (round 4: 2, with it 195 VGPRs; readme 0.65 -> 0.46 ms)
#endif
#ifndef RT_WAVES64_BVH_LITE
#define RT_WAVES64_BVH_LITE 4  // 163 ms bunny-Cornell vs 180 at 3 once the BVH nodes were tested in FP32 (profiles/r2/waves64)
#endif
#ifndef RT_WAVES64_BVH
#define RT_WAVES64_BVH 4  // demo1 69.9 ms vs 76.6 at 3 (profiles/r2/waves64); textured scenes, instances
#endif
#ifndef RT_WAVES64_BVH_MATS
// constant textures, the full material set (demo1).  Round 5 ran it at 5 (57.0 -> 56.4 ms), where
// every leaf class of it spilled 4-14 VGPRs; round 6 keeps every dispatchable kernel spill-free
// (tools/spill_gate.py), so 4
#define RT_WAVES64_BVH_MATS 4
#endif
#ifndef RT_WAVES64_BVH_MEDIA
#define RT_WAVES64_BVH_MEDIA 3  // the media chain kernels (pawn+fog 641 ms at 3, 883 at 4), instanced with textures / media
#endif
#ifndef RT_WAVES64_BVH_INST_MATS
#define RT_WAVES64_BVH_INST_MATS 3  // instances with the full material set: 1 VGPR spilled at 4
#endif
#ifndef RT_WAVES64_BVH_MEDIA_LATE
#define RT_WAVES64_BVH_MEDIA_LATE 4  // media events in the shading phase (kMedia 2): pawn+fog 508 -> 476 ms
#endif
#ifndef RT_WAVES_BVH_MEDIA_LATE
// FP32 pawn+fog: 310.7 -> 302 ms at 7 against 5 (profiles/r5/licm); 6, in two 768-lane workgroups
// per CU, stages 520 of its 631 surface nodes per copy against 120 at 7: 302.7 -> 276.1 ms (4:
// 318, 8: 297; profiles/r5/occ)
#define RT_WAVES_BVH_MEDIA_LATE 6
#endif
#ifndef RT_WAVES_BVH_MATS
#define RT_WAVES_BVH_MATS 8  // FP32 BVH, constant textures, the full material set, no media (demo1 39.7 -> 39.25 ms)
#endif
#ifndef RT_WAVES_BVH_MATS_GENERIC
#define RT_WAVES_BVH_MATS_GENERIC 7  // ... with generic leaves: 4 VGPRs spilled at 8
#endif
#ifndef RT_WAVES_BVH_INST_CHAIN
#define RT_WAVES_BVH_INST_CHAIN 4  // FP32 instances with the media query chain: 2-25 VGPRs spilled at 5
#endif
// kLeaf: the leaf class of the instantiation (0 generic, 1 triangles, 2 spheres; rt_trace.h trav_round)
#if RT_F64
#define RT_WAVES_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf)                                        \
  ((kVar) == RT_VAR_FLAT ? ((kTex) == 0 && !(kMedia) && !(kMats) ? RT_WAVES64_FLAT_LITE : RT_WAVES64_FLAT) \
                         : (kInst) && ((kTex) != 0 || (kMedia) != 0) ? RT_WAVES64_BVH_MEDIA          \
                         : (kInst) && (kMats) ? RT_WAVES64_BVH_INST_MATS                            \
                         : (kMedia) == 2 ? RT_WAVES64_BVH_MEDIA_LATE                                \
                         : (kMedia) ? RT_WAVES64_BVH_MEDIA                                          \
                         : (kTex) == 0 && !(kMats) ? RT_WAVES64_BVH_LITE                            \
                         : (kTex) == 0 && !(kInst) ? RT_WAVES64_BVH_MATS : RT_WAVES64_BVH)
#else
#define RT_WAVES_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf)                                              \
  ((kVar) == RT_VAR_FLAT ? ((kTex) == 2 ? RT_WAVES_FLAT_NOISE : (kTex) == 0 ? RT_WAVES_FLAT_TEX0 : RT_WAVES_FLAT) \
                         : (kMedia) == 2 ? ((kInst) ? RT_WAVES_BVH : RT_WAVES_BVH_MEDIA_LATE)             \
                         : (kMedia) == 1 && (kInst) ? RT_WAVES_BVH_INST_CHAIN                             \
                         : (kTex) == 0 && !(kMedia) && (kMats) && !(kInst)                                \
                             ? ((kLeaf) == 0 ? RT_WAVES_BVH_MATS_GENERIC : RT_WAVES_BVH_MATS)               \
                         : ((kTex) == 0 && !(kMedia) ? RT_WAVES_BVH_LITE : RT_WAVES_BVH))
#endif
// Kernels built without MachineLICM (rt_kernel_nl.hip / rt_kernel64_nl.hip, compiled with
// -mllvm -disable-machine-licm): the pass hoists the loop's binary64 constants (log, sincos and
// texture polynomial coefficients, ...) out of the persistent lane loop into ~20-90 VGPRs, so the
// heavier kernels sat at 2-3 waves or spilled (readme binary64 195 VGPRs -> 100: 0.65 -> 0.46 ms;
// pawn+fog binary64 107 instead of 128 + spills).  The lightest kernels keep it: the Cornell box
// (flat, constant textures, the diffuse materials) is 1.3 % slower without it and the bunny even
// (profiles/r5/licm).  Every instantiation lives in exactly one of the two translation units.
#ifndef RT_NOLICM_FLAT_LITE
#define RT_NOLICM_FLAT_LITE 0  // (experiments: the binary64 Cornell kernel without MachineLICM too)
#endif
#ifndef RT_NOLICM_BVH_LITE
#define RT_NOLICM_BVH_LITE 0  // (experiments: the bunny class without MachineLICM too)
#endif
#define RT_NOLICM_OF(kVar, kTex, kMedia, kMats, kInst)                                  \
  ((kVar) == RT_VAR_FLAT ? (RT_F64 && (RT_NOLICM_FLAT_LITE || (kTex) != 0 || (kMedia) != 0 || (kMats))) \
                         : (RT_NOLICM_BVH_LITE || (kTex) != 0 || (kMedia) != 0 || (kMats) || (kInst)))
#ifndef RT_TU_NOLICM
#define RT_TU_NOLICM 0
#endif
// kMedia of a variant code (rt_render_kernel's template parameter)
#define RT_MEDIA_OF(variant) \
  (((variant) & RT_VAR_MEDIA) == 0 ? 0 : ((variant) & RT_VAR_MEDIA_LATE) && ((variant) & RT_VAR_BASE) == RT_VAR_BVH ? 2 : 1)
// BVH workgroup size of a kernel class: each workgroup stages its own LDS copy of the top BVH
// nodes, so the fewer workgroups share a CU the more nodes each copy holds (pawn+fog and demo1
// gain 6-13 % from staging).  The largest workgroup whose waves split evenly over the
// CU's 4 SIMDs at the kernel's occupancy W (waves per SIMD): W = 3 -> 768 threads (one per CU),
// 4 -> 1024 (one), 6 -> 768 (two), 8 -> 1024 (two); W = 5 / 7 keep 256.  Round 5 (profiles/r5/
// bigwg): W = 4 at 1024 instead of 512 stages all of pawn+fog's surface nodes (binary64 476.5 ->
// 428.1 ms; bunny even); W = 8 at 1024 instead of 256, FP32 demo1 39.35 -> 37.7 ms; 640 / 896
// threads at W = 5 / 7 do not split evenly (10 / 14 waves per workgroup over 4 SIMDs): demo1
// binary64 +36 %, pawn+fog FP32 +22 %, one workgroup per CU fits.  RT_BIG_WG=0: 256 everywhere.
#ifndef RT_BIG_WG
#define RT_BIG_WG 1
#endif
#ifndef RT_BLOCK_BVH_OF
#define RT_BLOCK_BVH_OF(w) \
  (RT_BIG_WG && ((w) == 3 || (w) == 6) ? 768 : RT_BIG_WG && ((w) == 4 || (w) == 8) ? 1024 : RT_BLOCK_BVH)
#endif
#define RT_BLOCK_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf) \
  ((kVar) == RT_VAR_FLAT ? RT_BLOCK : RT_BLOCK_BVH_OF(RT_WAVES_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf)))
// commit-aggregation slots per wave and pixels per slot of a kernel class (rt_internal.h)
// (the wide slots: every binary64 flat class, and the FP32 flat classes without media —
// rt_internal.h RT_AGG_*_FLAT_F64; rt_build.cpp rt_host_plan_work mirrors the choice)
#define RT_AGG_WIDE_OF(kMedia) (RT_F64 || (kMedia) == 0)
#define RT_AGG_SLOTS_FLAT_R(kMedia) (RT_AGG_WIDE_OF(kMedia) ? RT_AGG_SLOTS_FLAT_F64 : RT_AGG_SLOTS_FLAT)
#define RT_AGG_PIX_FLAT_R(kMedia) (RT_AGG_WIDE_OF(kMedia) ? RT_AGG_PIX_FLAT_F64 : RT_AGG_PIX_FLAT)
#define RT_AGG_SLOTS_OF(kVar, kMedia) ((kVar) == RT_VAR_FLAT ? RT_AGG_SLOTS_FLAT_R(kMedia) : RT_AGG_SLOTS_BVH)
#define RT_AGG_PIX_OF(kVar, kMedia) ((kVar) == RT_VAR_FLAT ? RT_AGG_PIX_FLAT_R(kMedia) : RT_AGG_PIX_BVH)
// kMedia: 0 none; 1 the media queries chained in the traversal loop; 2 the media events in the
// shading phase (RT_VAR_MEDIA_LATE; rt_trace.h media_events_late)
// kNarrow: the 1024-lane class at 512 lanes, for a scene whose stacks do not fit one 1024-lane
// workgroup's LDS (RT_VAR_NARROW)
#define RT_BLOCK_N(kVar, kTex, kMedia, kMats, kInst, kLeaf, kNarrow)                       \
  ((kNarrow) && RT_BLOCK_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf) == 1024 ? 512 \
                                                                               : RT_BLOCK_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf))
template <int kVar, int kTex, int kMedia, bool kMats, bool kInst, int kLeaf, bool kNarrow = false>
__global__ __launch_bounds__(RT_BLOCK_N(kVar, kTex, kMedia, kMats, kInst, kLeaf, kNarrow))
__attribute__((amdgpu_waves_per_eu(RT_WAVES_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf))))
void rt_render_kernel(KernelParams P) {
  extern __shared__ int smem[];
#if defined(RT_WAVE_STAMPS)
  const unsigned long long t_start = wall_clock64();
#endif
  constexpr int kSlots = RT_AGG_SLOTS_OF(kVar, kMedia), kPix = RT_AGG_PIX_OF(kVar, kMedia);
  // (the launch bound; a deep BVH's render may launch fewer lanes: host render_block)
#if defined(RT_BLOCK_RUNTIME)  // (experiment: the stack stride from blockDim; profiles/r5/bigwg, r6/nondet)
  const int block = (int)blockDim.x;
#else
  constexpr int block = RT_BLOCK_N(kVar, kTex, kMedia, kMats, kInst, kLeaf, kNarrow);
#endif
  // (experiments, profiles/r6/nondet: one use of the launch-time workgroup size at a time)
#if defined(RT_BLOCK_RUNTIME_STACK)
  const int block_stack = (int)blockDim.x;
#else
  const int block_stack = block;
#endif
#if defined(RT_BLOCK_RUNTIME_NODES)
  const int block_nodes = (int)blockDim.x;
#else
  const int block_nodes = block;
#endif
#if defined(RT_BLOCK_RUNTIME_COPY)
  const int block_copy = (int)blockDim.x;
#else
  const int block_copy = block;
#endif
  constexpr int kAggBytes = AggGeom<kSlots, kPix>::kWaveBytes;
  const int waves = (int)(gridDim.x * (blockDim.x / 64));
  // wave-uniform (readfirstlane: the compiler cannot tell that threadIdx.x / 64 is), so the work
  // state and the slot pointers below live in SGPRs
  const int wave_in_block = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const int wave = (int)blockIdx.x * (int)(blockDim.x / 64) + wave_in_block;
  int overflow;
  // LDS: the lanes' item sums [RT_ACC_WORDS][block] (rt_trace.h AccLds; BVH kernels), the waves'
  // commit-aggregation slots (kAggBytes each), then (BVH kernels) [stack_depth + 1][block]
  // stack words (the last row a spare write target) and the top P.lds_nodes BVH nodes (64 B each)
  using AccT = typename std::conditional<RT_ACC_LDS_OF(kVar, kMedia), AccLds, Acc>::type;
  AccT acc;
  int* smem_rest = smem;
  if constexpr (RT_ACC_LDS_OF(kVar, kMedia)) {
    acc = AccLds{reinterpret_cast<unsigned long long*>(smem) + threadIdx.x, (int)blockDim.x};
    smem_rest = smem + 2 * RT_ACC_WORDS(real) * (int)blockDim.x;
  }
  // this wave's slots, zeroed by the wave itself (nothing else touches them: no barrier)
  unsigned long long* agg = reinterpret_cast<unsigned long long*>(smem_rest) + kAggBytes / 8 * wave_in_block;
  smem_rest += kAggBytes / 4 * (int)(blockDim.x / 64);
  for (int i = (int)__lane_id(); i < kAggBytes / 8; i += 64) agg[i] = 0ull;
#if defined(RT_WAVE_STAMPS)
  // (vector stores from lane 0; waves beyond the buffer are not recorded)
#define RT_STAMP_END(work)                                                                        \
  if (__lane_id() == 0 && wave < RT_STAMP_WAVES) {                                                \
    rt_stamp_buf[4 * wave] = t_start;                                                             \
    rt_stamp_buf[4 * wave + 1] = work.t_drain;                                                    \
    rt_stamp_buf[4 * wave + 2] = wall_clock64();                                                  \
    rt_stamp_buf[4 * wave + 3] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (31 << 11)) << 32 | \
                                 (unsigned)__builtin_amdgcn_s_getreg((20 << 0) | (3 << 11));      \
  }
#else
#define RT_STAMP_END(work)
#endif
  if constexpr (kVar == RT_VAR_FLAT) {
    WaveWork<kSlots, kPix, true> work(P, wave, waves, agg);
    overflow = lane_loop_lockstep<true, kTex, kMedia != 0, kMats>(P, work, Trav{nullptr, 0, nullptr}, P.prims, acc);
    work.finish();
    RT_STAMP_END(work)
  } else {
    v4f* lds_nodes = reinterpret_cast<v4f*>(smem_rest + (P.stack_depth + 1) * block_nodes);
    const float4* src = reinterpret_cast<const float4*>(P.nodes);
    for (int i = threadIdx.x; i < 4 * P.lds_nodes; i += block_copy) {
      const float4 q = src[i];
      lds_nodes[i] = v4f{q.x, q.y, q.z, q.w};
    }
    __syncthreads();
    WaveWork<kSlots, kPix, RT_KARGS_WORK_BVH> work(P, wave, waves, agg);
    const Trav W{smem_rest + threadIdx.x, block_stack, lds_nodes};
    if constexpr (kVar == RT_VAR_BVH_LOCKSTEP)
      overflow = lane_loop_lockstep<false, kTex, kMedia != 0, kMats>(P, work, W, P.prims, acc);
    else
      overflow = lane_loop_bvh<kTex, kMedia, kMats, kInst, kLeaf>(P, work, W, P.prims, acc);
    work.finish();
    RT_STAMP_END(work)
  }
  if (overflow) atomicOr(P.status, 1);
}

#ifndef RT_KERNEL_ONLY  // (register probes of one instantiation: tools/reg_probe.sh)
#if !RT_TU_NOLICM  // (the main translation unit)
// mean over spp (Ray.hs:232) from the fixed-point sums; NaN where a sample was non-finite.  One
// thread per output word (blockIdx.y = the channel) and the FP32 scale from the host: the kernel
// needs at most 8 VGPRs, so with two streams it fits beside the next frame's 7-wave FP32 render
// grid (69 VGPRs, 8 left per SIMD lane) instead of waiting for that grid to drain.  frame_rows > 0:
// `out` is the whole frame and tile row t goes to its global row (the rt_exec row interleave; rows
// past the image are padding and are skipped) — a multi-device scene's shards resolve straight into
// the first device's frame over xGMI instead of being gathered by copies afterwards
__global__ __launch_bounds__(256) void rt_resolve_kernel(const long long* __restrict__ accum,
                                                         const unsigned int* __restrict__ nanflag,
                                                         real* __restrict__ out, int n_pixels, int spp, double scale,
                                                         int width, int frame_rows, int n_shards, int shard,
                                                         int row_block) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_pixels) return;
  size_t w = 3 * (size_t)i + blockIdx.y;
  if (frame_rows > 0) {
    const int t = i / width, px = i - t * width;
    const int g = ((t / row_block) * n_shards + shard) * row_block + t % row_block;
    if (g >= frame_rows) return;
    w = 3 * ((size_t)g * width + px) + blockIdx.y;
  }
  const bool bad = nanflag[i] != 0u;
#if RT_F64
  // (hi + lo 2^-32) 2^-32 / spp: the integer words are exact in binary64 (< 2^53), one rounding
  // for the sum, one for the mean
  (void)scale;
  const long long* a = accum + 6 * (size_t)i + blockIdx.y;
  const double sum = ((double)a[0] + (double)(unsigned long long)a[3] * (1.0 / RT_FIX_SCALE)) * (1.0 / RT_FIX_SCALE);
  out[w] = bad ? __builtin_nan("") : sum / (double)spp;
#else
  (void)spp;
  out[w] = bad ? __builtin_nanf("") : (float)((double)accum[3 * (size_t)i + blockIdx.y] * scale);  // scale = 2^-32 / spp
#endif
}
#endif

#ifndef RT_LEAF_MEDIA
#define RT_LEAF_MEDIA 1
#endif
// the leaf class (kLeaf) of the instantiation render_kernel_of selects for a variant: one-class
// leaves only where render_kernel_media compiles them (the decoupled kernel without instances;
// with media, triangle leaves and constant textures only)
static int leaf_of(int variant) {
  if ((variant & RT_VAR_BASE) != RT_VAR_BVH || (variant & RT_VAR_INST)) return 0;
  if (variant & RT_VAR_MEDIA)
    return RT_LEAF_MEDIA && !(variant & (RT_VAR_TEX | RT_VAR_NOISE)) && (variant & RT_VAR_LEAF_TRI) ? 1 : 0;
  return (variant & RT_VAR_LEAF_TRI) ? 1 : (variant & RT_VAR_LEAF_SPHERE) ? 2 : 0;
}
// the workgroup of a variant's kernel (RT_BLOCK_OF of its class; RT_VAR_NARROW: half the
// 1024-lane workgroup, rt_build.cpp rt_host_variant)
static int render_block(int variant) {
  const bool flat = (variant & RT_VAR_BASE) == RT_VAR_FLAT;
  const int tex = (variant & RT_VAR_NOISE) ? 2 : (variant & RT_VAR_TEX) ? 1 : 0;
  const int media = RT_MEDIA_OF(variant);
  const bool mats = (variant & RT_VAR_MATS) != 0, inst = (variant & RT_VAR_INST) != 0;
  const int b = RT_BLOCK_OF(flat ? RT_VAR_FLAT : RT_VAR_BVH, tex, media, mats, inst, leaf_of(variant));
  return b == 1024 && (variant & RT_VAR_NARROW) ? 512 : b;
}
static bool acc_in_lds(int variant) {
  return RT_ACC_LDS_OF((variant & RT_VAR_BASE) == RT_VAR_FLAT ? RT_VAR_FLAT : RT_VAR_BVH, (variant & RT_VAR_MEDIA) != 0);
}
// LDS besides the stacks and the staged nodes: the lanes' item sums and the aggregation slots
static size_t render_fixed_lds(int variant) {
  const bool flat = (variant & RT_VAR_BASE) == RT_VAR_FLAT;
  const size_t acc = acc_in_lds(variant) ? (size_t)RT_ACC_WORDS(real) * 8 * render_block(variant) : 0;
  const bool wide = RT_F64 || (variant & RT_VAR_MEDIA) == 0;
  const size_t agg = (size_t)(!flat ? AggGeom<RT_AGG_SLOTS_BVH, RT_AGG_PIX_BVH>::kWaveBytes
                              : wide ? AggGeom<RT_AGG_SLOTS_FLAT_F64, RT_AGG_PIX_FLAT_F64>::kWaveBytes
                                     : AggGeom<RT_AGG_SLOTS_FLAT, RT_AGG_PIX_FLAT>::kWaveBytes) *
                     (render_block(variant) / 64);
  return acc + agg;
}
static size_t render_lds_bytes(int stack_depth, int variant, int lds_nodes) {
  return render_fixed_lds(variant) + ((variant & RT_VAR_BASE) == RT_VAR_FLAT
                    ? 0
                    : (size_t)(stack_depth + 1) * render_block(variant) * sizeof(int) + (size_t)lds_nodes * 64);
}

// the kernel instantiation of a variant code (base variant | RT_VAR_TEX | RT_VAR_NOISE |
// RT_VAR_MEDIA | RT_VAR_MATS): non-constant textures, noise textures, media and the materials
// beyond lightSource / pitchBlack / lambertian are compiled only into the instantiations of
// scenes that use them
// (inlined everywhere it raises the register allocation of every scene's kernel: the Cornell
// box is 4.8 % faster without the unused media code)
typedef void (*render_fn)(KernelParams);
// this translation unit's instantiation, or null when the other one holds it (RT_NOLICM_OF)
template <int kVar, int kTex, int kMedia, bool kMats, bool kInst, int kLeaf>
static render_fn kernel_here(int variant) {
  if constexpr ((bool)(RT_NOLICM_OF(kVar, kTex, kMedia, kMats, kInst)) == (bool)RT_TU_NOLICM) {
    if constexpr (RT_BLOCK_OF(kVar, kTex, kMedia, kMats, kInst, kLeaf) == 1024)  // (the narrow twin)
      if (variant & RT_VAR_NARROW) return rt_render_kernel<kVar, kTex, kMedia, kMats, kInst, kLeaf, true>;
    return rt_render_kernel<kVar, kTex, kMedia, kMats, kInst, kLeaf, false>;
  } else {
    (void)variant;
    return nullptr;
  }
}
template <int kVar, int kTex, int kMedia, bool kInst, int kLeaf>
static render_fn render_kernel_mats(int variant) {
  return (variant & RT_VAR_MATS) ? kernel_here<kVar, kTex, kMedia, true, kInst, kLeaf>(variant)
                                 : kernel_here<kVar, kTex, kMedia, false, kInst, kLeaf>(variant);
}
template <int kVar, int kTex, bool kInst>
static render_fn render_kernel_media(int variant) {
  // one-class BVH leaves (RT_VAR_LEAF_*): the decoupled kernel without instances; with media,
  // triangle leaves and constant textures only (pawn+fog)
  if (variant & RT_VAR_MEDIA) {
    // the decoupled kernel's media events: the traversal loop's query chain, or the shading phase
    // (RT_VAR_MEDIA_LATE)
    if constexpr (kVar == RT_VAR_BVH) {
      if (variant & RT_VAR_MEDIA_LATE) {
        if constexpr (!kInst && kTex == 0 && RT_LEAF_MEDIA)
          if (variant & RT_VAR_LEAF_TRI) return render_kernel_mats<kVar, kTex, 2, kInst, 1>(variant);
        return render_kernel_mats<kVar, kTex, 2, kInst, 0>(variant);
      }
    }
    if constexpr (kVar == RT_VAR_BVH && !kInst && kTex == 0 && RT_LEAF_MEDIA)
      if (variant & RT_VAR_LEAF_TRI) return render_kernel_mats<kVar, kTex, 1, kInst, 1>(variant);
    return render_kernel_mats<kVar, kTex, 1, kInst, 0>(variant);
  }
  if constexpr (kVar == RT_VAR_BVH && !kInst) {
    if (variant & RT_VAR_LEAF_TRI) return render_kernel_mats<kVar, kTex, 0, kInst, 1>(variant);
    if (variant & RT_VAR_LEAF_SPHERE) return render_kernel_mats<kVar, kTex, 0, kInst, 2>(variant);
  }
  return render_kernel_mats<kVar, kTex, 0, kInst, 0>(variant);
}
template <int kVar, bool kInst>
static render_fn render_kernel_flags(int variant) {
  if (variant & RT_VAR_NOISE) return render_kernel_media<kVar, 2, kInst>(variant);
  if (variant & RT_VAR_TEX) return render_kernel_media<kVar, 1, kInst>(variant);
  return render_kernel_media<kVar, 0, kInst>(variant);
}
// two-level instancing (RT_VAR_INST) is compiled into the decoupled BVH kernel only
static render_fn render_kernel_this_tu(int variant) {
  if (variant & RT_VAR_INST) return render_kernel_flags<RT_VAR_BVH, true>(variant);
  switch (variant & RT_VAR_BASE) {
    case RT_VAR_FLAT: return render_kernel_flags<RT_VAR_FLAT, false>(variant);
#if RT_LOCKSTEP_KERNELS
    case RT_VAR_BVH_LOCKSTEP: return render_kernel_flags<RT_VAR_BVH_LOCKSTEP, false>(variant);
#endif
    default: return render_kernel_flags<RT_VAR_BVH, false>(variant);
  }
}
// the kernels of the translation unit without MachineLICM (defined there)
render_fn render_kernel_nolicm(int variant);
// diagnostic builds: each translation unit's kernels count into that unit's own buffers; the
// main unit's readers add the other's (a wave's stamps come from one launch: the other is zero)
template <class T, size_t N>
static int diag_read(T (&buf)[N], unsigned long long* out, size_t n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(buf), n * sizeof(T)) != hipSuccess) return -1;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(buf)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(buf)) == hipSuccess ? 0 : -1;
}
int diag_read_nolicm(int which, unsigned long long* out, size_t n);  // 0: phase counters, 1: stamps
static int diag_read_this_tu(int which, unsigned long long* out, size_t n) {
  (void)which, (void)out, (void)n;
#if defined(RT_PHASE_PROF)
  if (which == 0) return diag_read(rt_prof_buf, out, n);
#endif
#if defined(RT_WAVE_STAMPS)
  if (which == 1) return diag_read(rt_stamp_buf, out, n);
#endif
  return -1;
}
#if RT_TU_NOLICM
int diag_read_nolicm(int which, unsigned long long* out, size_t n) { return diag_read_this_tu(which, out, n); }
#endif
static int diag_read_both(int which, unsigned long long* out, size_t n) {
  if (hipDeviceSynchronize() != hipSuccess || diag_read_this_tu(which, out, n)) return -1;
  unsigned long long* other = new unsigned long long[n];
  const int rc = diag_read_nolicm(which, other, n);
  for (size_t k = 0; k < n && rc == 0; ++k) out[k] += other[k];
  delete[] other;
  return rc;
}
#if RT_TU_NOLICM
render_fn render_kernel_nolicm(int variant) { return render_kernel_this_tu(variant); }
#else
static render_fn render_kernel_of(int variant) {
  const render_fn f = render_kernel_this_tu(variant);
  return f ? f : render_kernel_nolicm(variant);
}
#endif

#endif  // RT_KERNEL_ONLY
}  // namespace RT_NS
#if !defined(RT_KERNEL_ONLY) && !RT_TU_NOLICM  // (the launchers: in the main translation unit)

int rt_render_resident_blocks(const KernelParamsT<RT_NS::real>*, int device, int stack_depth, int variant,
                              int lds_nodes) {
  using namespace RT_NS;
  int per_cu = 0, cus = 0;
  size_t lds = render_lds_bytes(stack_depth, variant, lds_nodes);
  if (lds > 65536 && hipFuncSetAttribute((const void*)render_kernel_of(variant),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, render_kernel_of(variant), render_block(variant), lds);
  if (e != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return -1;
  if (per_cu < 1) per_cu = 1;
  return per_cu * cus;
}

// the render kernel's occupancy target (waves per SIMD) for a variant, and the LDS the lanes'
// item sums take per workgroup: the host sizes the LDS node staging to what is left of the
// workgroup's share of a CU's LDS at that occupancy (rt_api.hip ensure_precision)
int rt_render_waves(const KernelParamsT<RT_NS::real>*, int variant) {
  const bool flat = (variant & RT_VAR_BASE) == RT_VAR_FLAT;
  const int tex = (variant & RT_VAR_NOISE) ? 2 : (variant & RT_VAR_TEX) ? 1 : 0;
  const int media = RT_MEDIA_OF(variant);
  const bool mats = (variant & RT_VAR_MATS) != 0, inst = (variant & RT_VAR_INST) != 0;
  return RT_WAVES_OF(flat ? RT_VAR_FLAT : RT_VAR_BVH, tex, media, mats, inst, RT_NS::leaf_of(variant));
}
int rt_render_block(const KernelParamsT<RT_NS::real>*, int variant) { return RT_NS::render_block(variant); }
int rt_render_acc_lds(const KernelParamsT<RT_NS::real>*, int variant) {
  return (int)RT_NS::render_fixed_lds(variant);
}

int rt_launch_render(const KernelParamsT<RT_NS::real>& p, int grid_blocks, int variant, void* stream) {
  using namespace RT_NS;
  if (p.n_items <= 0 || grid_blocks <= 0) return 0;
  const int block = render_block(variant);
  long long need = ((long long)p.n_items + block - 1) / block;
  int grid = need < grid_blocks ? (int)need : grid_blocks;
  size_t lds = render_lds_bytes(p.stack_depth, variant, p.lds_nodes);
  hipLaunchKernelGGL(render_kernel_of(variant), dim3(grid), dim3(block), lds, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

#if defined(RT_PHASE_PROF)
// diagnostic build: read (and zero) the phase counters of this precision's BVH kernel
int rt_prof_read_kernel(const KernelParamsT<RT_NS::real>*, unsigned long long* out, int n) {
  using namespace RT_NS;
  if (n > PF_N) n = PF_N;
  return diag_read_both(0, out, (size_t)n) == 0 ? n : -1;
}
#endif

#if defined(RT_WAVE_STAMPS)
// diagnostic build: read (and zero) this precision's per-wave stamps, 4 words per wave
int rt_stamps_read_kernel(const KernelParamsT<RT_NS::real>*, unsigned long long* out, int n_waves) {
  using namespace RT_NS;
  if (n_waves > RT_STAMP_WAVES) n_waves = RT_STAMP_WAVES;
  return diag_read_both(1, out, 4 * (size_t)n_waves) == 0 ? n_waves : -1;
}
#endif

int rt_launch_resolve(const KernelParamsT<RT_NS::real>& p, void* stream) {
  using namespace RT_NS;
  int n = p.tile_rows * p.cam.width;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rt_resolve_kernel, dim3((n + 255) / 256, 3), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)p.accum, p.nanflag, p.out, n, p.cam.spp, 1.0 / (RT_FIX_SCALE * (double)p.cam.spp),
                     p.cam.width, p.out_frame_rows, p.n_shards, p.shard, p.row_block);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif  // RT_KERNEL_ONLY
