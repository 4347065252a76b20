// rt_internal.h — device-side layout shared by the host scene builder (rt_build.cpp), the
// C-ABI (rt_api.hip) and the render kernel (rt_kernel.hip / rt_trace.h).  Not part of the
// public ABI (include/rt.h).  Plain C++ (no HIP types) so the builder compiles anywhere.
//
// HBM layout (16-B records, read with one dwordx4 load per lane):
//   nodes   : 4 x float4 per BVH2 node, both children's boxes in the parent
//               [0] = (L.lo.x, L.hi.x, L.lo.y, L.hi.y)
//               [1] = (R.lo.x, R.hi.x, R.lo.y, R.hi.y)
//               [2] = (L.lo.z, L.hi.z, R.lo.z, R.hi.z)
//               [3] = (left child, right child, -, -) as int bits; child >= 0 is a node,
//                     child < 0 is a leaf ~(first * 64 + count - 1)
//   prims   : 4 x float4 per primitive (reordered into BVH leaf order, set after set)
//               plane : [0] = (n.xyz, kindflags) [1] = (q.xyz, gid) [2] = (wa.xyz, order)
//                       [3] = (wb.xyz, motion)   with a = (p-q).wa, b = (p-q).wb (Geometry.hs:130-131)
//               sphere: [0] = (c.xyz, kindflags) [1] = (radius, radius^2, uvframe, gid)
//                       [2] = (-, -, -, order)   [3] = (-, -, -, motion)
//   prim_shade: DevMaterial per primitive (its material, constant textures folded in)
//   prim_uv : 6 floats per primitive (plane shapes' uv0/uv1/uv2)
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#ifndef RT_BLOCK
// flat kernel workgroup: one wave.  Every wave has its own item pool and aggregation slots (nothing
// is shared across a workgroup), so a finished wave frees its slot at once and the next launch's
// waves (the other stream's frame) fill it; with 4-wave workgroups a slot waited for the
// workgroup's slowest wave: Cornell binary64 5.161 -> 5.070 ms, one rank's share of 8 GPUs 0.747 ->
// 0.728 ms, README's share of 8 -6 % (profiles/r4/wg_ab; round 3 measured 64 vs 256 within noise
// at 1 GPU, before the kernels fit 5 / 8 waves per SIMD)
#define RT_BLOCK 64
#endif
#ifndef RT_BLOCK_BVH
#define RT_BLOCK_BVH 256      // BVH kernel workgroup at 5 waves/SIMD (others: rt_render_kernel.h RT_BLOCK_OF)
#endif
// BVH nodes of a scene at most: the FP32 kernels address a node as a 32-bit byte offset
// node * 64 from the nodes' base (rt_trace.h RT_NODE_SADDR)
#define RT_MAX_NODES (1 << 26)
#define RT_STACK_DEPTH 64     // deepest BVH accepted: the LDS stack is sized by the scene's actual depth (deep
                              // trees lower occupancy instead of failing)
#define RT_MAX_MEDIA 8
#define RT_MAX_TARGETS 8
#ifndef RT_LEAF_MAX
#define RT_LEAF_MAX 8
#endif
// Work-item claims: a wave takes RT_POOL consecutive ids per queue atomic (rt_render_kernel.h
// WaveWork).  64 -> 128: Cornell 4.13 -> 4.04 ms (at 32 the head word saturates: 7.2 ms)
#ifndef RT_POOL
#define RT_POOL 128  // (a power of two >= 64; KernelParams::pool_shift)
#endif
// Commit aggregation (rt_render_kernel.h WaveWork): per wave, RT_AGG_SLOTS_* LDS slots of
// RT_AGG_PIX_* pixels' fixed-point words; a pool of RT_POOL ids is aggregated when it lies in one
// phase whose chunks per pixel n keep its pixel span ceil((RT_POOL - 1) / n) + 1 within a slot
#ifndef RT_AGG_SLOTS_FLAT
#define RT_AGG_SLOTS_FLAT 8
#endif
#ifndef RT_AGG_PIX_FLAT
#define RT_AGG_PIX_FLAT 17  // n >= 8
#endif
// the wide flat slots, binary64 flat kernels and FP32 flat kernels without media: 7 slots of 22
// pixels (binary64: 7.4 KB of LDS per wave, 20 waves per CU), so that the overlapped-frame plan's
// ~60-sample big items (3 per pixel, 64-id pools: a 22-pixel span) aggregate too: Cornell
// 4.728 -> 4.696 ms (profiles/r6/sweeps/agg).  The FP32 flat media classes keep 8 x 17: they
// spill 12 VGPRs with any other geometry
#ifndef RT_AGG_SLOTS_FLAT_F64
#define RT_AGG_SLOTS_FLAT_F64 7
#endif
#ifndef RT_AGG_PIX_FLAT_F64
#define RT_AGG_PIX_FLAT_F64 22
#endif
#ifndef RT_AGG_SLOTS_BVH
#define RT_AGG_SLOTS_BVH 4
#endif
#ifndef RT_AGG_PIX_BVH
#define RT_AGG_PIX_BVH 5  // n >= 32 (the BVH kernels' LDS is node staging too)
#endif
#ifndef RT_BIG_CHUNK_MAX
#define RT_BIG_CHUNK_MAX 16  // samples per big work item at most, synchronous calls (rt_build.cpp rt_host_plan_work)
#endif
#ifndef RT_BIG_CHUNK_MAX_ASYNC
#define RT_BIG_CHUNK_MAX_ASYNC 64  // ... renders whose frames overlap (rt_render_async)
#endif
// small items per resident lane kept for the queue tail (rt_build.cpp rt_host_plan_work; 0: one
// item size).  Cornell 600x600x200, same box (profiles/r2/items/): binary64 6.77 -> 6.63 ms at
// 16 (8: 6.69, 32: 6.64, 64: 6.78); FP32 3.50 -> 3.46 at 32 (16: 3.49); 8-GPU shares unchanged
#ifndef RT_TAIL_ITEMS_F64
#define RT_TAIL_ITEMS_F64 16
#endif
#ifndef RT_TAIL_ITEMS_F32
#define RT_TAIL_ITEMS_F32 32
#endif
#ifndef RT_TAIL_ITEMS_ASYNC  // (both precisions, renders whose frames overlap)
#define RT_TAIL_ITEMS_ASYNC 8
#endif
#define RT_LEAF_SHIFT 6       // leaf encoding ~(first << 6 | count - 1), count <= 64
#define RT_FLAT_MAX 32        // a set of at most this many leaves is one flat leaf (no traversal)
#define RT_LDS_PRIMS_MAX 256  // flat kernel: scenes of at most this many primitives
#define RT_PREFIX_MAX 16      // BVH scenes: at most this many large surface primitives tested first
#ifndef RT_PREFIX_AREA
#define RT_PREFIX_AREA 0.1    // ... those whose box area is >= this fraction of the surface set's box
#endif
#ifndef RT_PREFIX_SHRINK
#define RT_PREFIX_SHRINK 0.25 // ... and outliers whose removal shrinks the remaining box's area by this much
#endif
#define RT_EMPTY_ROOT ((int)0x80000000)
#ifndef RT_GRID_RESERVE
#define RT_GRID_RESERVE 0  // render-grid workgroup slots left free for the resolve (rt_api.hip render_async; 8 measured no help)
#endif
// Two-level instancing: a BVH child RT_INST_FLAG | k enters instance k (the ray goes to object
// space, the object's BVH is traversed); RT_INST_EXIT, pushed on entry, returns to world space.
// Node indices stay below RT_INST_FLAG.
#define RT_INST_FLAG 0x40000000
#define RT_INST_EXIT 0x7FFFFFFF

// render-kernel variants (rt_kernel.hip)
#define RT_VAR_FLAT 0          // every set one flat leaf, lockstep lane loop
#define RT_VAR_BVH_LOCKSTEP 1  // BVH, lockstep lane loop (reference schedule; experiments and tests)
// The lockstep BVH kernels are compiled only into experiment builds (make exp DEFS=
// -DRT_LOCKSTEP_KERNELS=1) and the host emulator: the product library's RT_AMD_VARIANT=1 runs the
// decoupled kernel
#ifndef RT_LOCKSTEP_KERNELS
#define RT_LOCKSTEP_KERNELS 0
#endif
#define RT_VAR_BVH 2           // BVH, traversal decoupled from shading (default for BVH scenes)
#define RT_VAR_BASE 3
#define RT_VAR_NOISE 4         // flag: the scene has noise / marble textures (their code compiled in)
#define RT_VAR_MEDIA 8         // flag: the scene has constantMedium volumes (their code compiled in)
#define RT_VAR_MATS 16         // flag: materials beyond lightSource / pitchBlack / lambertian
#define RT_VAR_TEX 32          // flag: some material reads a non-constant texture
#define RT_VAR_INST 64         // flag: the scene has instances (two-level traversal; RT_VAR_BVH only)
#define RT_VAR_LEAF_TRI 128    // flag: every BVH leaf below a BVH node is a static triangle (RT_VAR_BVH, no instances)
#define RT_VAR_LEAF_SPHERE 256 // flag: ... a static sphere (idem; kernels without media only)
#define RT_VAR_MEDIA_LATE 512  // flag (with RT_VAR_MEDIA, RT_VAR_BVH): the media events in the shading phase
#define RT_VAR_NARROW 1024     // flag: a 1024-lane kernel class launches its 512-lane twin (a deep BVH's stacks)
// The deepest stack (rows) one 1024-lane workgroup holds beside its lanes' item sums and slots
// (binary64: 48 + 16 B per lane; the FP32 classes take the same rule): deeper BVHs run RT_VAR_NARROW
#define RT_WIDE_STACK_ROWS 23
// Experiment knobs (rt_build.cpp): the library reads its RT_AMD_* tuning variables (variant,
// chunking, aggregation, prefix, box groups, LDS staging, ...) only when RT_AMD_EXPERIMENTS is set
// to a nonzero value — A/B sessions and the tests that compare code paths set it.  Otherwise
// rt_knob returns null and every caller (a Haskell program with a stray variable in its
// environment included) gets the measured defaults.
const char* rt_knob(const char* name);
// host choice of variant (rt_build.cpp); knob RT_AMD_VARIANT overrides the base for experiments.
// media_late: every medium's boundary is the surface set or a single leaf (rt_host_media_late)
int rt_host_variant(bool flat, int n_media, bool noise, bool mats, bool tex, bool inst = false, int leaf_kind = 0,
                    bool media_late = false, int stack_depth = 1);

#define RT_KIND_MASK 3
#define RT_FLAG_MOTION 4

// Philox event ids (the oracle uses the same: oracle/rt_oracle.c EV_*)
#define RT_EV_CAMERA0 0u
#define RT_EV_CAMERA1 1u
#define RT_EV_SCATTER 2u
#define RT_EV_MEDIA 3u

// Precision.  The reference computes in binary64 (`V3 Double`, Core.hs:29-31); the kernel is
// compiled for R = double (the default: rt_exec.flags without RT_EXEC_F32) and for R = float
// (the opt-in fast path).  Every record that holds scene values is a template over R; BVH
// nodes stay float in both (their boxes are rounded outward and padded, rt_bvh.cpp, so they
// are conservative for the binary64 primitives too).  Integer fields stored inside an R array
// (kind, gid, order, motion) keep their 32-bit pattern in the low word: rt_trace.h RT_R2I.

// Material record (32 B for float).  A constant texture's colour is folded in (tex_const = 1), so the
// common case needs no texture-table read; prim_shade holds one copy per primitive, so a surface
// hit reaches its material in one load (not primitive -> material index -> material -> texture).
template <class R>
struct DevMaterialT {
  int kind;
  int tex;
  R param;
  int tex_const;
  R c0[3];
  R pad;
};

template <class R>
struct DevTextureT {
  int kind, nu, nv, off;  // RT_TEX_*; checker dims | image width, height, first texel | noise layers
  R c0[3];
  R c1[3];
  R prm[8];               // noise: freq, shift.xyz | marble: dir.xyz, freq, shift.xyz
  R pad[2];
};

template <class R>
struct DevMediumT {
  R neg_inv_density;      // -(1 / density)  (Geometry.hs:303)
  int material;
  int root;               // BVH root of the boundary set
  int alias_surface;      // 1: the boundary set is geometrically the surface set (see below)
};
// alias_surface: the classic volume idiom `dielectric shape` + `constantMedium d shape` (the
// reference's pawnTest, test/Main.hs:323-344) has a boundary identical to the visible surfaces,
// leaf for leaf in the same depth-first order.  Then the boundary's first hit on (tmin, inf) IS
// the surface query's hit (same t, same winning leaf), and the entering case never needs the
// second query: t1 equals the surface t, so `t1 < tmax` fails (Geometry.hs:313).  The kernel
// reuses the surface result instead of traversing the boundary again; results are identical.

// Flat scenes (every set one leaf): a set's primitives are grouped by class so the kernel runs
// one specialised, branch-free loop per class: [first, end_quad) static parallelograms,
// [end_quad, end_tri) static triangles, [end_tri, end_sphere) static spheres,
// [end_sphere, end) moving primitives of any kind.  Each record's order word holds its SLOT:
// set first + rank of its depth-first `order` within the set, so the closest-hit key
// (t, slot) keeps the reference's tie-break whatever the test order, and the winner's index is
// its slot: flat scenes store `prims` in slot order and test class-grouped copies (flat_recs), so
// the loop tracks only the key and the winner's primitive index IS its slot.
#define RT_PRIM_CLASS_QUAD 1
#define RT_PRIM_CLASS_TRI 2
#define RT_PRIM_CLASS_SPHERE 0
struct DevFlatSet {
  int first, end_quad, end_tri, end_sphere, end;
  int box_first, box_end;  // its box groups: KernelParams::boxes[box_first, box_end)
  int pad;
};

// Box groups.  Parallelograms of one flat set (or of the BVH scenes' surface prefix) that are
// full faces of one rectangular box — `cuboid` (Geometry.hs:154-166) under a rigid transform, or
// the walls of the Cornell box — are tested together: the ray meets the box's surface at most
// twice (entry and exit, Kay-Kajiya slabs in the box frame), so one slab test plus a table
// lookup of the face replaces one parallelogram test per face.  Faces are numbered
// f = 2 * axis + side (side 1 = the s_axis = 1 end); each face's key order, gid and primitive
// are base + a 5-bit offset packed at bit 5 f of the codes (31: the box has no such face).
// The face primitives stay in the primitive array (shading reads them) after the set's tested
// range.  The closest hit is the reference's up to rounding at the boxes' edges.
#define RT_BOX_NO_FACE 31
template <class R>
struct DevBoxT {
  R sc[3];         // a_k . c for the corner c (s = 0 on every axis): s_k = a_k . p - sc[k]
  int ord_base;    // key order (flat: slot; prefix: depth-first order) of the faces
  R a0[3];         // axis_0 / L_0: s_0 = a0 . (p - c) in [0, 1] inside
  int ord_code;
  R a1[3];
  int gid_base;
  R a2[3];
  int gid_code;
  int prim_base;   // primitive index of the faces
  int prim_code;
  int pad[2];
};

template <class R>
struct DevTargetT {
  R q[3], u[3], v[3];
  R n[3];     // unit normal of u x v
  R wa[3];    // v x nS
  R wb[3];    // nS x u
  R cr[3];    // u x v (pdf denominator, Ray.hs:202)
  R prob;
  R thresh;   // cumulative probability (scanl1 (+) probs)
  R prob_icr; // prob / |u x v|: the pdf term p t^2 / |(u x v) . dir| = prob_icr t^2 / |n . dir|
};

// One placement of an instanced object (rt.h rt_instance): object -> world rigid transform,
// the object's BVH root, the placement's material (or -1) and the depth-first order of its first
// leaf (added to the object-space leaves' orders in the closest-hit key).
template <class R>
struct DevInstanceT {
  R m[12];       // row-major 3 x 4: rotation | translation
  int root;
  int material;
  int order;
  int pad;
};

template <class R>
struct DevCameraT {
  R center[3], top_left[3], pixel_u[3], pixel_v[3], disk_u[3], disk_v[3];
  R bg0[3], bg1[3];
  int width, height, spp, max_depth, bg_kind;
  int pad;
};

// Exact unsigned 32-bit division by a launch-constant divisor (Granlund-Montgomery, round-up
// multiplier with the add-and-shift fix-up): q = (t + ((n - t) >> 1)) >> s, t = umulhi(n, m).
// The host computes m, s (rt_build.cpp rt_host_fastdiv); d == 1 is the identity.
struct FastDiv {
  uint32_t m;
  int s;
  uint32_t d;
  int pad;
};

template <class R>
struct KernelParamsT {
  const float* nodes;      // 16 floats per node (both precisions)
  const R* prims;          // 16 R per primitive
  const DevMaterialT<R>* prim_shade;  // per primitive: its material record (DevMaterial)
  const R* prim_uv;        // 6 R per primitive
  const DevMaterialT<R>* mats;
  const DevTextureT<R>* texs;
  const R* motions;        // 8 R per motion: v0.xyz, -, v1.xyz, -
  const R* uvframes;       // 12 R per frame: rows of R (xyz, -)
  const R* texels;         // image textures: 4 R per texel (linear RGB, -)
  const int* perlin_perm;  // 3 x 256 permutation entries (Noise.hs permX / permY / permZ)
  const R* perlin_grad;    // 256 gradients, 4 R each (xyz, -)
  const R* flat_recs;      // flat scenes: the test records, class-grouped (DevFlatSet ranges)
  const DevBoxT<R>* boxes; // box groups of the flat sets / the surface prefix (DevBox)
  const DevInstanceT<R>* instances;  // two-level instancing (RT_VAR_INST)
  R* out;                  // linear RGB of the tile, R per channel
  int* status;             // device word: nonzero on stack overflow
  // persistent-lane work queue (rt_trace.h lane_loop): items = n_chunks x tile pixels
  unsigned long long* accum;  // fixed-point radiance sums per tile pixel: RT_ACC_WORDS(R) x int64
  unsigned int* nanflag;      // per tile pixel: a sample produced a non-finite radiance
  int* counter;               // next unclaimed item
  // two item sizes: the first big_items = n_big_chunks x tile pixels ids are big items (samples
  // [0, n_big_chunks * big_chunk) of their pixel in big_chunk-sample chunks: fewer commits), the
  // rest cover the remaining samples in chunk-sample chunks (a short queue tail).  Within each
  // phase the ids are PIXEL-major (id = phase start + tile pixel x chunks per pixel + chunk), so
  // a wave's pool of consecutive ids covers a few pixels (rt_render_kernel.h commit aggregation)
  int chunk;                  // samples per (small) item
  int n_chunks;               // small chunks per pixel
  int n_items;                // all items
  int big_chunk;              // samples per big item
  int n_big_chunks;           // big chunks per pixel (0: one item size)
  int big_items;              // n_big_chunks x tile pixels: the first small item's id
  int small_start;            // n_big_chunks x big_chunk: small chunk k covers [small_start + k chunk, ...)
  FastDiv div_big, div_small; // by n_big_chunks, by n_chunks (item id -> tile pixel)
  // commit aggregation (rt_render_kernel.h WaveWork): a phase's items are summed per pixel in the
  // wave's LDS slots when agg_big / agg_small (its chunks per pixel >= RT_AGG_MIN_N of the kernel
  // class); 0: every item adds to `accum` directly
  int agg_big, agg_small;
  // ids per work-queue pool, 1 << pool_shift (rt_render_kernel.h WaveWork): RT_POOL for renders
  // whose frames overlap (rt_render_async), 64 for the flat kernels' synchronous calls (rt_api.hip
  // render_async `lone`), whose one launch ends on the pools still held when the queue drains
  int pool_shift;
  int stack_depth;            // LDS stack entries per lane (>= the scene's BVH depth)
  int lds_nodes;              // BVH nodes [0, lds_nodes) are read from the workgroup's LDS copy
  int trav_exit_pct;          // BVH kernel: leave traversal when <= this % of live lanes trace
  int leaf_exit_pct;          // BVH traversal: test leaves once this % of the node loop's lanes hold one
  int n_prims;                // all leaves (every set)
  int surface_root;
  int surface_prefix;         // BVH scenes: flat_sets[0] is the surface set's prefix (rt_trace.h prefix_hits)
  int n_media;
  int n_targets;
  R rem_prob;
  DevMediumT<R> media[RT_MAX_MEDIA];
  DevFlatSet flat_sets[1 + RT_MAX_MEDIA];  // flat kernel: set 0 = surfaces, set m + 1 = medium m
  DevTargetT<R> targets[RT_MAX_TARGETS];
  DevCameraT<R> cam;
  uint32_t key0, key1;
  int n_shards, shard, row_block, tile_rows;
  // resolve target: 0 = `out` holds the shard's tile (tile_rows x width, shard-compact); otherwise
  // `out` is the WHOLE frame of out_frame_rows rows (a multi-device scene's gather buffer on the
  // first device, written across xGMI by peer devices) and the resolve puts each tile row at its
  // global row, so no separate gather copy is needed (rt_api.hip multi_render)
  int out_frame_rows;
  FastDiv div_width, div_block;  // image width, row block
};
using DevMaterial = DevMaterialT<float>;
using DevTexture = DevTextureT<float>;
using DevMedium = DevMediumT<float>;
using DevBox = DevBoxT<float>;
using DevTarget = DevTargetT<float>;
using DevCamera = DevCameraT<float>;
using DevInstance = DevInstanceT<float>;
using KernelParams = KernelParamsT<float>;
using KernelParams64 = KernelParamsT<double>;

#define RT_FIX_SCALE 4294967296.0  // 2^32: per-sample radiance is accumulated as int64 * 2^-32
// Fixed-point words per pixel: float kernels add trunc(x 2^32) per channel (3 words); binary64
// kernels add trunc(x 2^32) and the next 32 bits of x 2^64 as a second word per channel (6
// words: x to 2^-64, every bit of a binary64 radiance >= 2^-11).  Integer sums commute, so the
// mean is bit-for-bit independent of the schedule and of the shard layout in both precisions.
#define RT_ACC_WORDS(R) (sizeof(R) == 8 ? 6 : 3)

// Host-side scene image, ready for upload (rt_build.cpp): the records of one precision
template <class R>
struct HostArraysT {
  std::vector<R> prims, prim_uv, motions, uvframes, texels, perlin_grad;
  std::vector<R> flat_recs;  // flat scenes: class-grouped copies of the records (prims is in slot order)
  std::vector<DevMaterialT<R>> prim_shade, mats;
  std::vector<DevTextureT<R>> texs;
  std::vector<DevBoxT<R>> boxes;  // box groups (DevBox)
  std::vector<DevInstanceT<R>> instances;
  DevMediumT<R> media[RT_MAX_MEDIA];
};
struct HostScene {
  std::vector<float> nodes;  // BVH nodes (float in both precisions)
  std::vector<int> perlin_perm;
  std::vector<int> prim_mat;        // material index per primitive (-1: medium boundary)
  HostArraysT<float> f32;           // records of the float kernels
  HostArraysT<double> f64;          // records of the binary64 kernels
  int surface_root = RT_EMPTY_ROOT;
  int n_media = 0;
  DevFlatSet flat_sets[1 + RT_MAX_MEDIA] = {};
  int n_nodes = 0, n_prims = 0, max_depth = 0, n_boxes = 0;
  int surface_nodes = 0;  // nodes of the surface BVH: [0, surface_nodes), breadth-first
  bool flat = false;  // every set is a single flat leaf (no BVH nodes)
  bool noise = false;  // some texture is a noise / marble texture
  bool uv_tex = false;     // some material reads a non-constant texture (RT_VAR_TEX)
  int leaf_exit_pct = 100;  // BVH traversal policy for this scene (KernelParams::leaf_exit_pct)
  int leaf_exit_pct64 = 100;  // ... for the binary64 kernels
  int trav_exit_pct = 50;   // and its lane-loop exit (KernelParams::trav_exit_pct)
  int trav_exit_pct64 = 50;  // ... for the binary64 kernels
  bool full_mats = false;  // some material is not lightSource / pitchBlack / lambertian (RT_VAR_MATS)
  int n_instances = 0;     // two-level instancing (RT_VAR_INST)
  int leaf_kind = 0;       // BVH leaves (after the prefix): 1 all static triangles, 2 all static spheres, 0 mixed
  template <class R>
  const HostArraysT<R>& arrays() const;
};
template <>
inline const HostArraysT<float>& HostScene::arrays<float>() const { return f32; }
template <>
inline const HostArraysT<double>& HostScene::arrays<double>() const { return f64; }

struct rt_scene;
struct rt_camera_settings;
struct rt_exec;

// rt_build.cpp (host only; return RT_OK or RT_E_*, message in err)
int rt_host_build_scene(const rt_scene* sc, HostScene& out, std::string& err);
int rt_host_image_height(const rt_camera_settings* cs);
int rt_host_shard_rows(int height, const rt_exec* ex);
// every medium's boundary is the surface set (alias_surface) or a single leaf, whose records are
// the same for every lane: the BVH kernels can run the media events in the shading phase
// (RT_VAR_MEDIA_LATE; rt_trace.h media_events_late)
bool rt_host_media_late(const HostScene& H);
// fills camera / targets / tiling / key of P (pointers are left to the caller); R = float, double
template <class R>
int rt_host_make_params(const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex, KernelParamsT<R>& P,
                        std::string& err);
// work decomposition (rt_build.cpp): chunk so that items >= ~8 x resident lanes
template <class R>
void rt_host_plan_work(KernelParamsT<R>& P, long long resident_lanes, bool two_sizes, bool lone = false);  // two_sizes: flat kernel
FastDiv rt_host_fastdiv(uint32_t d);
// the 8-bit code thresholds of the output epilogue (rt_build.cpp): thr[k] = the smallest binary64
// x in [0, 1] whose code min(255, floor(256 transfer(x))) is >= k (k = 1..255; thr[0] = 0)
void rt_host_encode8_thresholds(int encoding, double* thr);

// rt_kernel.hip / rt_kernel64.hip (device launchers)
// resident workgroups of the render kernel for a given LDS stack depth (occupancy query)
int rt_render_resident_blocks(const KernelParams*, int device, int stack_depth, int variant, int lds_nodes);
int rt_render_resident_blocks(const KernelParams64*, int device, int stack_depth, int variant, int lds_nodes);
int rt_render_waves(const KernelParams*, int variant);
int rt_render_waves(const KernelParams64*, int variant);
int rt_render_block(const KernelParams*, int variant);  // the workgroup size of a variant's kernel
int rt_render_block(const KernelParams64*, int variant);
int rt_render_acc_lds(const KernelParams*, int variant);
int rt_render_acc_lds(const KernelParams64*, int variant);
int rt_launch_render(const KernelParams& p, int grid_blocks, int variant, void* stream);
int rt_launch_render(const KernelParams64& p, int grid_blocks, int variant, void* stream);
// accum / nanflag -> out (mean over spp, NaN where flagged)
int rt_launch_resolve(const KernelParams& p, void* stream);
int rt_launch_resolve(const KernelParams64& p, void* stream);
#if defined(RT_PHASE_PROF)
int rt_prof_read_kernel(const KernelParams*, unsigned long long* out, int n);
int rt_prof_read_kernel(const KernelParams64*, unsigned long long* out, int n);
#endif
#if defined(RT_WAVE_STAMPS)
int rt_stamps_read_kernel(const KernelParams*, unsigned long long* out, int n_waves);
int rt_stamps_read_kernel(const KernelParams64*, unsigned long long* out, int n_waves);
#endif
// 8-bit epilogue over float (in_f64 = 0) or binary64 (1) values; thr: 256 host thresholds
int rt_launch_encode8(const void* in, int in_f64, uint8_t* out, int64_t n, const double* thr, int encoding,
                      void* stream);
