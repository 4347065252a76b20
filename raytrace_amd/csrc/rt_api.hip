// rt_api.hip — the C-ABI entry points of include/rt.h: scene build (rt_build.cpp, once per
// call however many devices render), upload to HBM (a precision's records on its first render),
// kernel launch (rt_kernel.hip / rt_kernel64.hip), multi-device scenes (one process, many GPUs:
// concurrent uploads, shard renders on per-device streams, a device-side gather by peer copies
// into the first device's framebuffer and ONE device-to-host copy), the 8-bit output epilogue,
// error reporting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt.h"
#include "rt_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(RT_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
int upload(T** dst, const std::vector<T>& src) {
  size_t bytes = src.size() * sizeof(T);
  HIP_TRY(hipMalloc((void**)dst, bytes ? bytes : 16));
  if (bytes) HIP_TRY(hipMemcpy(*dst, src.data(), bytes, hipMemcpyHostToDevice));
  return RT_OK;
}

// the device copies of one precision's records (rt_internal.h HostArraysT)
template <class R>
struct DevArrays {
  R* prims = nullptr;
  DevMaterialT<R>* prim_shade = nullptr;
  R* prim_uv = nullptr;
  DevMaterialT<R>* mats = nullptr;
  DevTextureT<R>* texs = nullptr;
  R* motions = nullptr;
  R* uvframes = nullptr;
  R* texels = nullptr;
  R* perlin_grad = nullptr;
  R* flat_recs = nullptr;
  DevBoxT<R>* boxes = nullptr;
  DevInstanceT<R>* instances = nullptr;
  DevMediumT<R> media[RT_MAX_MEDIA];
  int resident_blocks = 0;  // render-kernel workgroups resident on the device (occupancy query)
  int lds_nodes = 0;        // top surface-BVH nodes this precision's kernel stages in LDS per workgroup
  int upload(const HostArraysT<R>& H) {
    int rc;
    if ((rc = ::upload(&prims, H.prims)) || (rc = ::upload(&prim_shade, H.prim_shade)) ||
        (rc = ::upload(&prim_uv, H.prim_uv)) || (rc = ::upload(&mats, H.mats)) || (rc = ::upload(&texs, H.texs)) ||
        (rc = ::upload(&motions, H.motions)) || (rc = ::upload(&uvframes, H.uvframes)) ||
        (rc = ::upload(&flat_recs, H.flat_recs)) || (rc = ::upload(&boxes, H.boxes)) ||
        (rc = ::upload(&texels, H.texels)) || (rc = ::upload(&perlin_grad, H.perlin_grad)) ||
        (rc = ::upload(&instances, H.instances)))
      return rc;
    for (int k = 0; k < RT_MAX_MEDIA; ++k) media[k] = H.media[k];
    return RT_OK;
  }
  void release() {
    for (void* p : {(void*)prims, (void*)prim_shade, (void*)prim_uv, (void*)mats, (void*)texs, (void*)motions,
                    (void*)uvframes, (void*)texels, (void*)perlin_grad, (void*)flat_recs, (void*)boxes,
                    (void*)instances})
      (void)hipFree(p);
  }
};

}  // namespace

struct rt_device_scene {
  int device = 0;
  float* nodes = nullptr;
  int* perlin_perm = nullptr;
  int* status = nullptr;
  // a precision's records are uploaded (and its kernel's occupancy queried) on its first render:
  // a caller that renders one precision never pays for the other's copy in HBM or its upload
  std::shared_ptr<const HostScene> host;
  mutable std::mutex mu;
  mutable DevArrays<float> f32;
  mutable DevArrays<double> f64;
  mutable bool have_f32 = false, have_f64 = false;
  int leaf_exit_pct = 100, leaf_exit_pct64 = 100;
  int trav_exit_pct = 50, trav_exit_pct64 = 50;
  int surface_root = RT_EMPTY_ROOT;
  int n_media = 0;
  DevFlatSet flat_sets[1 + RT_MAX_MEDIA];
  int n_nodes = 0, n_prims = 0, max_depth = 0;
  int stack_depth = 1;       // LDS stack entries per lane
  int variant = RT_VAR_FLAT;  // render-kernel variant (rt_internal.h RT_VAR_*)
  double build_ms = 0;       // host scene build (shared by every device of a multi-device scene)
  mutable double upload_ms = 0;  // host -> device copies of this device (common + precisions so far)
  template <class R>
  DevArrays<R>& arrays() const;
  template <class R>
  bool& have() const;
};
template <>
DevArrays<float>& rt_device_scene::arrays<float>() const { return f32; }
template <>
DevArrays<double>& rt_device_scene::arrays<double>() const { return f64; }
template <>
bool& rt_device_scene::have<float>() const { return have_f32; }
template <>
bool& rt_device_scene::have<double>() const { return have_f64; }

// The resident per-shard buffers of a multi-device scene: shard k's tile, its render workspace
// (fixed-point sums, NaN flags, queue heads), its stream and timing events on devices[k]
struct MultiPart {
  int device = 0;
  void* d_tile = nullptr;
  size_t tile_cap = 0;
  char* ws = nullptr;
  size_t ws_cap = 0;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};
struct rt_multi_scene {
  std::vector<int> devices;                // shard k renders on devices[k]
  std::vector<rt_device_scene*> scenes;    // one per DISTINCT device, in first-use order
  std::vector<int> scene_of;               // devices[k] -> scenes index
  double build_ms = 0, upload_ms = 0;      // one host build; the uploads' wall time (concurrent)
  // kept across renders (grown when a frame needs more): no allocation after the first render
  std::mutex mu;                           // one render at a time: the buffers below are shared
  std::vector<MultiPart> parts;            // per devices[k]
  std::vector<char> peer_ok;               // per distinct device: may write the first device's memory
  void* d_gather = nullptr;                // first device: the n tiles in global row order
  size_t gather_cap = 0;
  uint8_t* d_codes = nullptr;              // first device: the 8-bit epilogue's output
  size_t codes_cap = 0;
  hipStream_t st0 = nullptr;               // first device: epilogue and device-to-host copy
  int* h_status = nullptr;                 // pinned host word: the one-device render's status read-back
};

namespace {

// one render of the scene's records of precision R, enqueued on `stream`
// the records of precision R on the scene's device (uploaded on first use) and their kernel's
// resident workgroups; thread-safe
template <class R>
int ensure_precision(const rt_device_scene* s) {
  std::lock_guard<std::mutex> lock(s->mu);
  if (s->have<R>()) return RT_OK;
  auto t0 = std::chrono::steady_clock::now();
  HIP_TRY(hipSetDevice(s->device));
  DevArrays<R>& A = s->arrays<R>();
  int rc = A.upload(s->host->arrays<R>());
  if (rc) {
    A.release();
    A = DevArrays<R>();
    return rc;
  }
  A.lds_nodes = 0;
  if ((s->variant & RT_VAR_BASE) != RT_VAR_FLAT) {
    // stage as many top (breadth-first) surface nodes as fit beside the lanes' item sums and
    // stacks in the workgroup's share of the CU's 160 KB LDS at the kernel's occupancy (1 KB
    // granules; 4 x waves-per-SIMD waves per CU, `block` threads per workgroup); env
    // RT_AMD_LDS_NODES caps it (0 disables, for experiments)
    const int waves = std::max(1, rt_render_waves((const KernelParamsT<R>*)nullptr, s->variant));
    const int block = rt_render_block((const KernelParamsT<R>*)nullptr, s->variant);
    const int per_cu = std::max(1, 4 * waves * 64 / block);
    const int budget = (163840 / per_cu / 1024) * 1024 - 1024;
    const int used = rt_render_acc_lds((const KernelParamsT<R>*)nullptr, s->variant) +
                     (s->stack_depth + 1) * block * (int)sizeof(int);
    A.lds_nodes = std::max(0, std::min(s->host->surface_nodes, (budget - used) / 64));
    if (const char* e = rt_knob("RT_AMD_LDS_NODES")) A.lds_nodes = std::min(A.lds_nodes, std::max(0, atoi(e)));
  }
  A.resident_blocks = rt_render_resident_blocks((const KernelParamsT<R>*)nullptr, s->device, s->stack_depth,
                                                s->variant, A.lds_nodes);
  if (A.resident_blocks <= 0) {
    A.release();
    A = DevArrays<R>();
    return fail(RT_E_HIP, "occupancy query failed");
  }
  s->have<R>() = true;
  s->upload_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}

// the stream-ordered workspace of one render: fixed-point sums, NaN flags, queue head words
size_t workspace_bytes(size_t tile_pixels, int acc_words, size_t* off_flag, size_t* off_ctr) {
  const size_t of = tile_pixels * acc_words * sizeof(long long);
  const size_t oc = of + ((tile_pixels * sizeof(unsigned) + 255) & ~(size_t)255);
  if (off_flag) *off_flag = of;
  if (off_ctr) *off_ctr = oc;
  return oc + 256 * 8;  // up to 8 queue head words (rt_render_kernel.h RT_QUEUES)
}


// ws / ws_cap: a caller-held workspace (a multi-device scene's resident one), or null: the render
// takes one from the stream-ordered pool (hipMallocAsync / hipFreeAsync).  lone: a synchronous
// call's launch (rt_render, rt_multi_render), whose time includes the end of its queue: the flat
// kernels take 64-id pools there, so no wave holds a second round of items when the queue drains
// (one binary64 Cornell launch 5.385 -> 5.164 ms; with frames overlapped on two streams, as
// rt_render_async callers run them, 128 is as fast and the README scene 2 % faster:
// profiles/r5/pool).  Env RT_AMD_POOL_SHIFT overrides (experiments).
template <class R>
int render_async(const rt_device_scene* s, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex, R* d_out,
                 void* hip_stream, char* ws_given = nullptr, size_t ws_cap = 0, int frame_rows = 0, bool lone = false) {
  if (int rc = ensure_precision<R>(s)) return rc;
  lone = lone || (ex && (ex->flags & RT_EXEC_SOLO));  // (the caller says this render runs alone)
  const DevArrays<R>& A = s->arrays<R>();
  KernelParamsT<R> P;
  std::memset(&P, 0, sizeof P);
  if (lone && (s->variant & RT_VAR_BASE) == RT_VAR_FLAT) P.pool_shift = 6;
  if (const char* e = rt_knob("RT_AMD_POOL_SHIFT")) P.pool_shift = std::max(4, std::min(10, atoi(e)));
  std::string err;
  int rc = rt_host_make_params(cs, seed, ex, P, err);
  if (rc) return fail(rc, "%s", err.c_str());
  P.nodes = s->nodes;
  P.prims = A.prims;
  P.prim_shade = A.prim_shade;
  P.prim_uv = A.prim_uv;
  P.mats = A.mats;
  P.texs = A.texs;
  P.motions = A.motions;
  P.uvframes = A.uvframes;
  P.texels = A.texels;
  P.perlin_perm = s->perlin_perm;
  P.perlin_grad = A.perlin_grad;
  P.flat_recs = A.flat_recs;
  P.boxes = A.boxes;
  P.instances = A.instances;
  P.status = s->status;
  P.out = d_out;
  P.surface_root = s->surface_root;
  P.leaf_exit_pct = sizeof(R) == 8 ? s->leaf_exit_pct64 : s->leaf_exit_pct;
  P.surface_prefix = (s->variant & RT_VAR_BASE) != RT_VAR_FLAT && s->n_nodes > 0 ? 1 : 0;
  P.n_media = s->n_media;
  for (int k = 0; k < s->n_media; ++k) P.media[k] = A.media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) P.flat_sets[k] = s->flat_sets[k];
  P.stack_depth = s->stack_depth;
  P.lds_nodes = A.lds_nodes;
  P.n_prims = s->n_prims;
  rt_host_plan_work(P, (long long)A.resident_blocks * rt_render_block((const KernelParamsT<R>*)nullptr, s->variant),
                    (s->variant & RT_VAR_BASE) == RT_VAR_FLAT, lone);
  P.trav_exit_pct = sizeof(R) == 8 ? s->trav_exit_pct64 : s->trav_exit_pct;
  P.out_frame_rows = frame_rows;
  HIP_TRY(hipSetDevice(s->device));
  // stream-ordered workspace: fixed-point sums, NaN flags, queue counter (graph-capturable)
  const size_t tile_pixels = (size_t)P.tile_rows * P.cam.width;
  size_t off_flag = 0, off_ctr = 0;
  const size_t bytes = workspace_bytes(tile_pixels, RT_ACC_WORDS(R), &off_flag, &off_ctr);
  hipStream_t st = (hipStream_t)hip_stream;
  char* ws = ws_given && ws_cap >= bytes ? ws_given : nullptr;
  const bool own = ws == nullptr;
  if (own) HIP_TRY(hipMallocAsync((void**)&ws, bytes, st));
  HIP_TRY(hipMemsetAsync(ws, 0, bytes, st));
  P.accum = (unsigned long long*)ws;
  P.nanflag = (unsigned int*)(ws + off_flag);
  P.counter = (int*)(ws + off_ctr);
  rc = RT_OK;
  // The persistent grid can leave RT_GRID_RESERVE workgroup slots free, so that with frames
  // overlapped on two streams this frame's resolve starts as soon as its render ends.  Measured
  // (profiles/r3/iso): with 8 free slots the FP32 resolve still takes 3.1 ms, starved by the next
  // frame's grid; binary64's runs in 23 us either way (its kernel leaves VGPRs free) — so 0.
  int reserve = A.resident_blocks > 16 * RT_GRID_RESERVE ? RT_GRID_RESERVE : 0;
  if (const char* e = rt_knob("RT_AMD_GRID_RESERVE")) reserve = std::max(0, std::min(A.resident_blocks - 1, atoi(e)));
  if (rt_launch_render(P, A.resident_blocks - reserve, s->variant, hip_stream) || rt_launch_resolve(P, hip_stream))
    rc = fail(RT_E_HIP, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (own) HIP_TRY(hipFreeAsync(ws, st));
  return rc;
}

bool exec_f32(const rt_exec* ex) { return ex && (ex->flags & RT_EXEC_F32) != 0; }

// rt_exec.flags: known bits only, at most one 8-bit encoding
int check_flags(const rt_exec* ex) {
  const int known = RT_EXEC_F32 | RT_EXEC_ENCODE8_SRGB | RT_EXEC_ENCODE8_SQRT | RT_EXEC_SOLO;
  if (ex->flags & ~known) return fail(RT_E_INVALID, "unknown rt_exec.flags bits 0x%x", ex->flags & ~known);
  if ((ex->flags & RT_EXEC_ENCODE8_SRGB) && (ex->flags & RT_EXEC_ENCODE8_SQRT))
    return fail(RT_E_INVALID, "rt_exec.flags: RT_EXEC_ENCODE8_SRGB and RT_EXEC_ENCODE8_SQRT are exclusive");
  return RT_OK;
}

// rt_exec.flags -> the 8-bit epilogue's encoding (0 sRGB, 1 sqrt) or -1 (linear output)
int exec_encoding(const rt_exec* ex) {
  if (!ex) return -1;
  if (ex->flags & RT_EXEC_ENCODE8_SRGB) return 0;
  if (ex->flags & RT_EXEC_ENCODE8_SQRT) return 1;
  return -1;
}

const double* encode8_table(int encoding) {
  static double thr[2][256];
  static std::once_flag once[2];
  std::call_once(once[encoding], [&] { rt_host_encode8_thresholds(encoding, thr[encoding]); });
  return thr[encoding];
}

void destroy_scene(rt_device_scene* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  (void)hipFree(s->nodes);
  (void)hipFree(s->perlin_perm);
  (void)hipFree(s->status);
  s->f32.release();
  s->f64.release();
  delete s;
}

// the precision-independent part of a device scene: BVH nodes, Perlin permutations, status word,
// the kernel variant and the LDS plan; precisions follow on first render (ensure_precision)
int upload_common(const std::shared_ptr<const HostScene>& Hp, int device, rt_device_scene** out) {
  auto t0 = std::chrono::steady_clock::now();
  const HostScene& H = *Hp;
  *out = nullptr;
  HIP_TRY(hipSetDevice(device));
  auto* s = new rt_device_scene();
  s->device = device;
  s->host = Hp;
  std::vector<int> status(4, 0);
  int rc;
  if ((rc = upload(&s->nodes, H.nodes)) || (rc = upload(&s->perlin_perm, H.perlin_perm)) ||
      (rc = upload(&s->status, status))) {
    destroy_scene(s);
    return rc;
  }
  s->surface_root = H.surface_root;
  s->leaf_exit_pct = H.leaf_exit_pct;
  s->leaf_exit_pct64 = H.leaf_exit_pct64;
  s->trav_exit_pct = H.trav_exit_pct;
  s->trav_exit_pct64 = H.trav_exit_pct64;
  s->n_media = H.n_media;
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) s->flat_sets[k] = H.flat_sets[k];
  s->n_nodes = H.n_nodes;
  s->n_prims = H.n_prims;
  s->max_depth = H.max_depth;
  s->stack_depth = H.max_depth > 1 ? H.max_depth : 1;
  s->variant = rt_host_variant(H.flat, H.n_media, H.noise, H.full_mats, H.uv_tex, H.n_instances > 0, H.leaf_kind,
                               rt_host_media_late(H), s->stack_depth);
  s->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = s;
  return RT_OK;
}

int ensure_precisions(const rt_device_scene* s, int prec_mask) {  // bit 0: FP32, bit 1: binary64
  int rc = RT_OK;
  if ((prec_mask & 1) && (rc = ensure_precision<float>(s))) return rc;
  if ((prec_mask & 2) && (rc = ensure_precision<double>(s))) return rc;
  return RT_OK;
}

int check_device(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_E_HIP, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RT_E_INVALID, "device %d out of range (%d devices)", device, ndev);
  return RT_OK;
}

void multi_destroy(rt_multi_scene* M);

// A multi-device scene from one host build: the distinct devices upload CONCURRENTLY (one host
// thread each; the host build is shared, never repeated per device).  prec_mask: precisions to
// upload now (the rest on first render).
int multi_create(const std::shared_ptr<const HostScene>& H, const int32_t* devices, int n, int prec_mask,
                 rt_multi_scene** out) {
  *out = nullptr;
  if (n < 1 || n > RT_MAX_DEVICES || !devices) return fail(RT_E_INVALID, "invalid device list (%d devices)", n);
  for (int k = 0; k < n; ++k)
    if (int rc = check_device(devices[k])) return rc;
  auto* M = new rt_multi_scene();
  M->devices.assign(devices, devices + n);
  std::vector<int> distinct;
  for (int k = 0; k < n; ++k) {
    int j = (int)(std::find(distinct.begin(), distinct.end(), devices[k]) - distinct.begin());
    if (j == (int)distinct.size()) distinct.push_back(devices[k]);
    M->scene_of.push_back(j);
  }
  M->scenes.assign(distinct.size(), nullptr);
  std::vector<int> rcs(distinct.size(), RT_OK);
  std::vector<std::string> errs(distinct.size());
  auto t0 = std::chrono::steady_clock::now();
  {
    std::vector<std::thread> th;
    for (size_t j = 0; j < distinct.size(); ++j)
      th.emplace_back([&, j] {
        int rc = upload_common(H, distinct[j], &M->scenes[j]);
        if (!rc) rc = ensure_precisions(M->scenes[j], prec_mask);
        rcs[j] = rc;
        if (rc) errs[j] = g_err;
      });
    for (auto& t : th) t.join();
  }
  M->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  for (size_t j = 0; j < distinct.size(); ++j)
    if (rcs[j]) {
      for (rt_device_scene* s : M->scenes) destroy_scene(s);
      delete M;
      return fail(rcs[j], "device %d: %s", distinct[j], errs[j].c_str());
    }
  // per shard: its stream and timing events (its tile and workspace come with the first render)
  M->parts.resize(n);
  for (int k = 0; k < n; ++k) {
    MultiPart& q = M->parts[k];
    q.device = devices[k];
    if (hipSetDevice(q.device) != hipSuccess || hipStreamCreateWithFlags(&q.st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&q.e0) != hipSuccess || hipEventCreate(&q.e1) != hipSuccess) {
      multi_destroy(M);
      return fail(RT_E_HIP, "stream / events on device %d", devices[k]);
    }
  }
  if (hipSetDevice(devices[0]) != hipSuccess || hipStreamCreateWithFlags(&M->st0, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void**)&M->h_status, 64, hipHostMallocDefault) != hipSuccess) {
    multi_destroy(M);
    return fail(RT_E_HIP, "stream on device %d", devices[0]);
  }
  // the first device holds the frame: every other device's resolve writes its rows there over
  // xGMI (peer access); a device without peer access renders into its own tile, which is then
  // copied over (HIP stages such copies itself)
  M->peer_ok.assign(distinct.size(), 1);
  for (size_t j = 1; j < distinct.size(); ++j) {
    int can = 0;
    M->peer_ok[j] = 0;
    if (hipDeviceCanAccessPeer(&can, distinct[j], distinct[0]) == hipSuccess && can) {
      (void)hipSetDevice(distinct[j]);
      const hipError_t e = hipDeviceEnablePeerAccess(distinct[0], 0);
      M->peer_ok[j] = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
      (void)hipGetLastError();
    }
  }
  *out = M;
  return RT_OK;
}

void multi_destroy(rt_multi_scene* M) {
  if (!M) return;
  for (MultiPart& q : M->parts) {
    (void)hipSetDevice(q.device);
    if (q.st) (void)hipStreamSynchronize(q.st);
    if (q.e0) (void)hipEventDestroy(q.e0);
    if (q.e1) (void)hipEventDestroy(q.e1);
    if (q.st) (void)hipStreamDestroy(q.st);
    (void)hipFree(q.d_tile);
    (void)hipFree(q.ws);
  }
  if (!M->devices.empty()) {
    (void)hipSetDevice(M->devices[0]);
    if (M->st0) (void)hipStreamDestroy(M->st0);
    if (M->h_status) (void)hipHostFree(M->h_status);
    (void)hipFree(M->d_gather);
    (void)hipFree(M->d_codes);
  }
  for (rt_device_scene* s : M->scenes) destroy_scene(s);
  delete M;
}

// grow a resident device buffer to `need` bytes (on the current device); counts the allocation
int grow(void** p, size_t* cap, size_t need, int* allocs) {
  if (*cap >= need && *p) return RT_OK;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, need ? need : 16));
  *cap = need;
  ++*allocs;
  return RT_OK;
}

// One device (the drop-in's plain rt_render / a one-device scene): everything on the part's
// stream with ONE host synchronisation — status reset, workspace memset, render, resolve, the 8-bit
// epilogue, the image's device-to-host copy and the status word's into pinned memory — instead of a
// thread per shard and a synchronising call for each step (the multi-device path below)
int render_one(rt_multi_scene* M, const rt_camera_settings* cs, uint64_t seed, const rt_exec& ex, int encoding,
               void* out_host, rt_stats* stats, double build_ms, int allocs,
               std::chrono::steady_clock::time_point t0) {
  MultiPart& q = M->parts[0];
  const rt_device_scene* s = M->scenes[0];
  const bool f32 = exec_f32(&ex);
  const int h = rt_host_image_height(cs);
  const int rows = rt_host_shard_rows(h, &ex);
  const size_t esize = f32 ? sizeof(float) : sizeof(double);
  const size_t tile_pixels = (size_t)rows * cs->image_width;
  HIP_TRY(hipSetDevice(s->device));
  auto tp = std::chrono::steady_clock::now();
  if (int r = ensure_precisions(s, f32 ? 1 : 2)) return r;
  const double prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
  if (int r = grow(&q.d_tile, &q.tile_cap, tile_pixels * 3 * esize, &allocs)) return r;
  const size_t wsb = workspace_bytes(tile_pixels, f32 ? RT_ACC_WORDS(float) : RT_ACC_WORDS(double), nullptr, nullptr);
  if (int r = grow((void**)&q.ws, &q.ws_cap, wsb, &allocs)) return r;
  // everything below is enqueued on q.st; a failure after the first enqueue synchronises the
  // stream before returning, so no copy into out_host is still in flight when the call returns
  auto enqueue = [&]() -> int {
    HIP_TRY(hipMemsetAsync(s->status, 0, 4 * sizeof(int), q.st));
    HIP_TRY(hipEventRecord(q.e0, q.st));
    const int r = f32 ? render_async<float>(s, cs, seed, &ex, (float*)q.d_tile, q.st, q.ws, q.ws_cap, 0, true)
                      : render_async<double>(s, cs, seed, &ex, (double*)q.d_tile, q.st, q.ws, q.ws_cap, 0, true);
    if (r) return r;
    HIP_TRY(hipEventRecord(q.e1, q.st));
    const void* src = q.d_tile;
    size_t bytes = tile_pixels * 3 * esize;
    if (encoding >= 0) {
      const int64_t nv = (int64_t)tile_pixels * 3;
      if (rt_launch_encode8(q.d_tile, f32 ? 0 : 1, M->d_codes, nv, encode8_table(encoding), encoding, q.st))
        return fail(RT_E_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
      src = M->d_codes;
      bytes = (size_t)nv;
    }
    // (the image is copied before the status word is read, in the same synchronisation: on
    // RT_E_STACK out_host holds the partial image, include/rt.h)
    HIP_TRY(hipMemcpyAsync(out_host, src, bytes, hipMemcpyDeviceToHost, q.st));
    HIP_TRY(hipMemcpyAsync(M->h_status, s->status, sizeof(int), hipMemcpyDeviceToHost, q.st));
    return RT_OK;
  };
  if (const int r = enqueue()) {
    (void)hipStreamSynchronize(q.st);
    return r;
  }
  HIP_TRY(hipStreamSynchronize(q.st));
  if (*M->h_status) return fail(RT_E_STACK, "BVH traversal stack overflow");
  if (stats) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, q.e0, q.e1));
    std::memset(stats, 0, sizeof *stats);
    stats->upload_ms = build_ms + M->upload_ms + prep_ms;
    stats->kernel_ms = ms;
    stats->samples = (int64_t)rows * cs->image_width * cs->samples_per_pixel;
    stats->bvh_nodes = s->n_nodes;
    stats->max_stack = s->max_depth;
    stats->device_allocs = allocs;
    stats->kernel_block = f32 ? rt_render_block((const KernelParamsT<float>*)nullptr, s->variant)
                              : rt_render_block((const KernelParamsT<double>*)nullptr, s->variant);
    stats->total_ms = build_ms + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return RT_OK;
}

// Render the image (device list: shard k of n on devices[k]) or, with one device, the rt_exec
// shard; gather on the first device; optional 8-bit epilogue there; ONE copy to the host buffer.
// Every buffer, stream and event is the scene's own (rt_multi_scene), kept across renders.
int multi_render(rt_multi_scene* M, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                 void* out_host, rt_stats* stats, double build_ms) {
  auto t0 = std::chrono::steady_clock::now();
  if (int rc = check_flags(ex)) return rc;
  const int h = rt_host_image_height(cs);
  if (h <= 0 || cs->image_width <= 0) return fail(RT_E_INVALID, "image %dx%d must be non-empty", cs->image_width, h);
  const int n = (int)M->devices.size();
  if (n > 1 && ex->n_shards != 1) return fail(RT_E_INVALID, "a device list renders the whole image (n_shards must be 1)");
  const int rows_out = rt_host_shard_rows(h, ex);  // == h for a device list / a single shard
  if (rows_out < 0) return fail(RT_E_INVALID, "invalid rt_exec");
  {  // validate the camera before touching a device
    KernelParams P;
    std::string err;
    int rc = rt_host_make_params(cs, seed, ex, P, err);
    if (rc) return fail(rc, "%s", err.c_str());
  }
  std::lock_guard<std::mutex> lock(M->mu);
  const bool f32 = exec_f32(ex);
  const int encoding = exec_encoding(ex);
  const size_t esize = f32 ? sizeof(float) : sizeof(double);
  const size_t row_bytes = (size_t)cs->image_width * 3 * esize;
  struct Job {
    rt_exec ex{};
    int rows = 0;
    float ms = 0;
    int rc = RT_OK;
    std::string err;
    double prep_ms = 0;
    int allocs = 0;
  };
  std::vector<Job> jobs(n);
  // experiments and tests: shards forced onto the tile + strided-copy path a device without peer
  // access takes (RT_AMD_COPY_SHARDS: bit k for shard k, -1 every shard), so one GPU exercises it
  unsigned long long copy_mask = 0;
  if (const char* e = rt_knob("RT_AMD_COPY_SHARDS")) copy_mask = (unsigned long long)strtoll(e, nullptr, 0);
  for (int k = 0; k < n; ++k) {
    Job& p = jobs[k];
    p.ex = *ex;
    p.ex.n_devices = 0;
    p.ex.devices = nullptr;
    p.ex.device = M->devices[k];
    p.ex.flags &= ~(RT_EXEC_ENCODE8_SRGB | RT_EXEC_ENCODE8_SQRT);  // the tiles are linear; encoded after the gather
    if (n > 1) {
      p.ex.n_shards = n;
      p.ex.shard = k;
    }
    p.rows = rt_host_shard_rows(h, &p.ex);
  }
  // the first device's framebuffer: n shard tiles in global row order (n > 1; padded to equal
  // tiles), or the single shard's tile itself
  const int dev0 = M->devices[0];
  const int rb = ex->row_block;
  const size_t gather_rows = n > 1 ? (size_t)n * jobs[0].rows : (size_t)rows_out;
  int allocs = 0;
  int rc = RT_OK;
  if (hipSetDevice(dev0) != hipSuccess) rc = fail(RT_E_HIP, "device %d", dev0);
  if (!rc && n > 1) rc = grow(&M->d_gather, &M->gather_cap, gather_rows * row_bytes, &allocs);
  if (!rc && encoding >= 0)
    rc = grow((void**)&M->d_codes, &M->codes_cap, std::max<size_t>(16, gather_rows * cs->image_width * 3), &allocs);
  if (!rc && n == 1) return render_one(M, cs, seed, jobs[0].ex, encoding, out_host, stats, build_ms, allocs, t0);
  // a stack overflow of an earlier render must not fail this one: clear each device's status word
  for (size_t j = 0; j < M->scenes.size() && !rc; ++j) {
    const rt_device_scene* s = M->scenes[j];
    const MultiPart& q = M->parts[std::find(M->scene_of.begin(), M->scene_of.end(), (int)j) - M->scene_of.begin()];
    if (hipSetDevice(s->device) != hipSuccess || hipMemsetAsync(s->status, 0, 4 * sizeof(int), q.st) != hipSuccess ||
        hipStreamSynchronize(q.st) != hipSuccess)
      rc = fail(RT_E_HIP, "status reset on device %d", s->device);
  }
  if (!rc) {
    std::vector<std::thread> th;
    for (int k = 0; k < n; ++k)
      th.emplace_back([&, k] {
        Job& p = jobs[k];
        MultiPart& q = M->parts[k];
        const rt_device_scene* s = M->scenes[M->scene_of[k]];
        auto run = [&]() -> int {
          HIP_TRY(hipSetDevice(s->device));
          auto tp = std::chrono::steady_clock::now();
          if (int r = ensure_precisions(s, f32 ? 1 : 2)) return r;
          p.prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
          const size_t tile_pixels = (size_t)p.rows * cs->image_width;
          // n > 1: the resolve writes the shard's rows straight into the frame on the first device
          // (over xGMI from a peer); without peer access, a tile and a strided copy
          const bool direct = n > 1 && M->peer_ok[M->scene_of[k]] && !((copy_mask >> k) & 1ull);
          if (!direct)
            if (int r = grow(&q.d_tile, &q.tile_cap, tile_pixels * 3 * esize, &p.allocs)) return r;
          const size_t wsb = workspace_bytes(tile_pixels, f32 ? RT_ACC_WORDS(float) : RT_ACC_WORDS(double), nullptr, nullptr);
          if (int r = grow((void**)&q.ws, &q.ws_cap, wsb, &p.allocs)) return r;
          void* dst = direct ? M->d_gather : q.d_tile;
          const int frame_rows = direct ? h : 0;
          HIP_TRY(hipEventRecord(q.e0, q.st));
          const int r = f32 ? render_async<float>(s, cs, seed, &p.ex, (float*)dst, q.st, q.ws, q.ws_cap, frame_rows, true)
                            : render_async<double>(s, cs, seed, &p.ex, (double*)dst, q.st, q.ws, q.ws_cap, frame_rows, true);
          if (r) return r;
          HIP_TRY(hipEventRecord(q.e1, q.st));
          if (n > 1 && !direct) {
            // shard-local row block b is global block b n + k: one strided copy into the first
            // device's framebuffer (peer-to-peer over xGMI for another device)
            const size_t w = (size_t)rb * row_bytes;
            HIP_TRY(hipMemcpy2DAsync((char*)M->d_gather + (size_t)k * w, (size_t)n * w, q.d_tile, w, w,
                                     (size_t)p.rows / rb, hipMemcpyDeviceToDevice, q.st));
          }
          HIP_TRY(hipStreamSynchronize(q.st));
          HIP_TRY(hipEventElapsedTime(&p.ms, q.e0, q.e1));
          return RT_OK;
        };
        p.rc = run();
        if (p.rc) p.err = g_err;
      });
    for (auto& t : th) t.join();
    for (int k = 0; k < n && !rc; ++k)
      if (jobs[k].rc) rc = fail(jobs[k].rc, "device %d: %s", M->devices[k], jobs[k].err.c_str());
  }
  for (const Job& p : jobs) allocs += p.allocs;
  int status = 0;
  for (size_t j = 0; j < M->scenes.size() && !rc; ++j) {
    int ps = 0;
    (void)hipSetDevice(M->scenes[j]->device);
    if (hipMemcpy(&ps, M->scenes[j]->status, 4, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RT_E_HIP, "status");
    status |= ps;
  }
  if (!rc && status) rc = fail(RT_E_STACK, "BVH traversal stack overflow");
  const void* d_img = n > 1 ? M->d_gather : M->parts[0].d_tile;
  const size_t out_rows = n > 1 ? (size_t)h : (size_t)rows_out;
  if (!rc) {
    (void)hipSetDevice(dev0);
    const void* src = d_img;
    size_t bytes = out_rows * row_bytes;
    if (encoding >= 0) {
      const int64_t nv = (int64_t)out_rows * cs->image_width * 3;
      if (rt_launch_encode8(d_img, f32 ? 0 : 1, M->d_codes, nv, encode8_table(encoding), encoding, M->st0))
        rc = fail(RT_E_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
      src = M->d_codes;
      bytes = (size_t)nv;
    }
    if (!rc && (hipMemcpyAsync(out_host, src, bytes, hipMemcpyDeviceToHost, M->st0) != hipSuccess ||
                hipStreamSynchronize(M->st0) != hipSuccess))
      rc = fail(RT_E_HIP, "copy back: %s", hipGetErrorString(hipGetLastError()));
  }
  if (stats && !rc) {
    std::memset(stats, 0, sizeof *stats);
    double prep = 0;
    float ms = 0;
    for (const Job& p : jobs) {
      prep = std::max(prep, p.prep_ms);
      ms = std::max(ms, p.ms);
    }
    stats->upload_ms = build_ms + M->upload_ms + prep;
    stats->kernel_ms = ms;
    stats->samples = (int64_t)rows_out * cs->image_width * cs->samples_per_pixel;
    stats->bvh_nodes = M->scenes[0]->n_nodes;
    stats->max_stack = M->scenes[0]->max_depth;
    stats->device_allocs = allocs;
    stats->kernel_block = f32 ? rt_render_block((const KernelParamsT<float>*)nullptr, M->scenes[0]->variant)
                              : rt_render_block((const KernelParamsT<double>*)nullptr, M->scenes[0]->variant);
    stats->total_ms = build_ms + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return rc;
}

int build_host(const rt_scene* sc, std::shared_ptr<const HostScene>& out, double& ms) {
  auto t0 = std::chrono::steady_clock::now();
  auto H = std::make_shared<HostScene>();
  std::string err;
  int rc = rt_host_build_scene(sc, *H, err);
  if (rc) return fail(rc, "%s", err.c_str());
  out = H;
  ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}


}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_E_HIP, "no HIP device");
  return n;
}

int rt_image_height(const rt_camera_settings* cs) {
  if (!cs) return fail(RT_E_INVALID, "null camera settings");
  int h = rt_host_image_height(cs);
  if (h < 0) return fail(RT_E_INVALID, "image height is not finite");
  return h;
}

int rt_shard_rows(int32_t height, const rt_exec* ex) {
  int r = rt_host_shard_rows(height, ex);
  if (r < 0) return fail(RT_E_INVALID, "invalid rt_exec");
  return r;
}

int rt_shard_row(int32_t t, const rt_exec* ex) {
  if (!ex || ex->n_shards < 1 || ex->row_block < 1) return fail(RT_E_INVALID, "invalid rt_exec");
  return ((t / ex->row_block) * ex->n_shards + ex->shard) * ex->row_block + (t % ex->row_block);
}

int rt_scene_destroy(rt_device_scene* s) {
  destroy_scene(s);
  return RT_OK;
}

int rt_scene_create(const rt_scene* sc, int32_t device, rt_device_scene** out) {
  if (!sc || !out) return fail(RT_E_INVALID, "null argument");
  *out = nullptr;
  std::shared_ptr<const HostScene> H;
  double build_ms = 0;
  if (int rc = build_host(sc, H, build_ms)) return rc;
  if (int rc = check_device(device)) return rc;
  if (int rc = upload_common(H, device, out)) return rc;
  (*out)->build_ms = build_ms;
  return RT_OK;
}

int rt_scene_stats(const rt_device_scene* s, rt_stats* st) {
  if (!s || !st) return fail(RT_E_INVALID, "null argument");
  std::memset(st, 0, sizeof *st);
  st->upload_ms = s->build_ms + s->upload_ms;
  st->bvh_nodes = s->n_nodes;
  st->max_stack = s->stack_depth;
  return RT_OK;
}

int rt_render_async(const rt_device_scene* s, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                    void* d_out_rgb, void* hip_stream) {
  if (!s || !d_out_rgb || !ex || !cs) return fail(RT_E_INVALID, "null argument");
  if (ex->n_devices != 0) return fail(RT_E_INVALID, "rt_render_async renders on the scene's device (n_devices = 0)");
  if (int rc = check_flags(ex)) return rc;
  if (exec_encoding(ex) >= 0) return fail(RT_E_INVALID, "rt_render_async writes linear RGB (use rt_encode8_async)");
  if (exec_f32(ex)) return render_async<float>(s, cs, seed, ex, (float*)d_out_rgb, hip_stream);
  return render_async<double>(s, cs, seed, ex, (double*)d_out_rgb, hip_stream);
}

int rt_multi_scene_create(const rt_scene* sc, const int32_t* devices, int32_t n_devices, rt_multi_scene** out) {
  if (!sc || !out) return fail(RT_E_INVALID, "null argument");
  *out = nullptr;
  std::shared_ptr<const HostScene> H;
  double build_ms = 0;
  if (int rc = build_host(sc, H, build_ms)) return rc;
  if (int rc = multi_create(H, devices, n_devices, 0, out)) return rc;
  (*out)->build_ms = build_ms;
  return RT_OK;
}

int rt_multi_scene_destroy(rt_multi_scene* m) {
  multi_destroy(m);
  return RT_OK;
}

int rt_multi_render(const rt_multi_scene* m, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                    void* out, rt_stats* stats) {
  if (!m || !cs || !ex || !out) return fail(RT_E_INVALID, "null argument");
  if (ex->n_devices != 0) return fail(RT_E_INVALID, "rt_multi_render renders on the scene's devices (n_devices = 0)");
  // the scene's resident buffers are its internal state (the caller's handle stays const)
  const int rc = multi_render(const_cast<rt_multi_scene*>(m), cs, seed, ex, out, stats, 0.0);
  if (!rc && stats) stats->upload_ms += m->build_ms;  // the scene's one-time cost, as rt_render reports it
  return rc;
}

int rt_render(const rt_camera_settings* cs, const rt_scene* scene, uint64_t seed, const rt_exec* ex, void* out_rgb,
              rt_stats* stats) {
  if (!cs || !scene || !ex || !out_rgb) return fail(RT_E_INVALID, "null argument");
  int h = rt_host_image_height(cs);
  if (h <= 0 || cs->image_width <= 0) return fail(RT_E_INVALID, "image %dx%d must be non-empty", cs->image_width, h);
  if (rt_host_shard_rows(h, ex) < 0) return fail(RT_E_INVALID, "invalid rt_exec");
  if (int rc = check_flags(ex)) return rc;
  if (ex->n_devices < 0 || ex->n_devices > RT_MAX_DEVICES || (ex->n_devices > 0 && !ex->devices))
    return fail(RT_E_INVALID, "invalid device list (%d devices)", ex->n_devices);
  if (ex->n_devices > 0 && ex->n_shards != 1)
    return fail(RT_E_INVALID, "a device list renders the whole image (n_shards must be 1)");
  {  // validate the camera before building or touching a device
    KernelParams P;
    std::string err;
    int rc = rt_host_make_params(cs, seed, ex, P, err);
    if (rc) return fail(rc, "%s", err.c_str());
  }
  std::shared_ptr<const HostScene> H;
  double build_ms = 0;
  if (int rc = build_host(scene, H, build_ms)) return rc;  // ONE host build, whatever the device count
  const int32_t one = ex->device;
  const int32_t* devs = ex->n_devices > 0 ? ex->devices : &one;
  const int n = ex->n_devices > 0 ? ex->n_devices : 1;
  rt_multi_scene* M = nullptr;
  if (int rc = multi_create(H, devs, n, exec_f32(ex) ? 1 : 2, &M)) return rc;  // only this call's precision
  rt_exec e = *ex;
  e.n_devices = 0;
  e.devices = nullptr;
  const int rc = multi_render(M, cs, seed, &e, out_rgb, stats, build_ms);
  multi_destroy(M);
  return rc;
}

int rt_encode8_async(const void* d_rgb, int32_t in_f64, uint8_t* d_out, int64_t n_values, int32_t encoding,
                     void* hip_stream) {
  if (!d_rgb || !d_out || n_values < 0) return fail(RT_E_INVALID, "invalid encode arguments");
  if (encoding != 0 && encoding != 1) return fail(RT_E_INVALID, "encoding must be 0 (sRGB) or 1 (sqrt)");
  if (rt_launch_encode8(d_rgb, in_f64 ? 1 : 0, d_out, n_values, encode8_table(encoding), encoding, hip_stream))
    return fail(RT_E_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
  return RT_OK;
}

#if defined(RT_PHASE_PROF)
// diagnostic build only: the BVH kernel's phase counters (rt_trace.h RT_PHASE_PROF), read and zeroed
int rt_prof_read(int f64, unsigned long long* out, int n) {
  return f64 ? rt_prof_read_kernel((const KernelParams64*)nullptr, out, n) : rt_prof_read_kernel((const KernelParams*)nullptr, out, n);
}
#endif
#if defined(RT_WAVE_STAMPS)
// diagnostic build only: per-wave (start, queue drained, end, hw id) stamps of the last renders
// (rt_render_kernel.h RT_WAVE_STAMPS), read and zeroed; returns the waves read
int rt_stamps_read(int f64, unsigned long long* out, int n_waves) {
  return f64 ? rt_stamps_read_kernel((const KernelParams64*)nullptr, out, n_waves)
             : rt_stamps_read_kernel((const KernelParams*)nullptr, out, n_waves);
}
#endif

}  // extern "C"
