// rt_api.hip — the C-ABI entry points of include/rt.h: scene build (rt_build.cpp), upload to
// HBM (both precisions' records), kernel launch (rt_kernel.hip / rt_kernel64.hip), the device
// list of rt_render (one process, many GPUs), error reporting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
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
  DevArrays<float> f32;
  DevArrays<double> f64;
  int leaf_exit_pct = 100;
  int trav_exit_pct = 50;
  int surface_root = RT_EMPTY_ROOT;
  int n_media = 0;
  DevFlatSet flat_sets[1 + RT_MAX_MEDIA];
  int n_nodes = 0, n_prims = 0, max_depth = 0;
  int stack_depth = 1;       // LDS stack entries per lane
  int lds_nodes = 0;         // top surface-BVH nodes staged in LDS per workgroup
  int variant = RT_VAR_FLAT;  // render-kernel variant (rt_internal.h RT_VAR_*)
  double upload_ms = 0;
  template <class R>
  const DevArrays<R>& arrays() const;
};
template <>
const DevArrays<float>& rt_device_scene::arrays<float>() const { return f32; }
template <>
const DevArrays<double>& rt_device_scene::arrays<double>() const { return f64; }

namespace {

// one render of the scene's records of precision R, enqueued on `stream`
template <class R>
int render_async(const rt_device_scene* s, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex, R* d_out,
                 void* hip_stream) {
  const DevArrays<R>& A = s->arrays<R>();
  KernelParamsT<R> P;
  std::memset(&P, 0, sizeof P);
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
  P.leaf_exit_pct = s->leaf_exit_pct;
  P.surface_prefix = (s->variant & RT_VAR_BASE) != RT_VAR_FLAT && s->n_nodes > 0 ? 1 : 0;
  P.n_media = s->n_media;
  for (int k = 0; k < s->n_media; ++k) P.media[k] = A.media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) P.flat_sets[k] = s->flat_sets[k];
  P.stack_depth = s->stack_depth;
  P.lds_nodes = s->lds_nodes;
  P.n_prims = s->n_prims;
  rt_host_plan_work(P, (long long)A.resident_blocks * rt_block_of(s->variant), (s->variant & RT_VAR_BASE) == RT_VAR_FLAT);
  P.trav_exit_pct = s->trav_exit_pct;
  HIP_TRY(hipSetDevice(s->device));
  // stream-ordered workspace: fixed-point sums, NaN flags, queue counter (graph-capturable)
  const size_t tile_pixels = (size_t)P.tile_rows * P.cam.width;
  const size_t off_flag = tile_pixels * RT_ACC_WORDS(R) * sizeof(long long);
  const size_t off_ctr = off_flag + ((tile_pixels * sizeof(unsigned) + 255) & ~(size_t)255);
  const size_t bytes = off_ctr + 256 * 8;  // up to 8 queue head words (rt_render_kernel.h RT_QUEUES)
  hipStream_t st = (hipStream_t)hip_stream;
  char* ws = nullptr;
  HIP_TRY(hipMallocAsync((void**)&ws, bytes, st));
  HIP_TRY(hipMemsetAsync(ws, 0, bytes, st));
  P.accum = (unsigned long long*)ws;
  P.nanflag = (unsigned int*)(ws + off_flag);
  P.counter = (int*)(ws + off_ctr);
  rc = RT_OK;
  if (rt_launch_render(P, A.resident_blocks, s->variant, hip_stream) || rt_launch_resolve(P, hip_stream))
    rc = fail(RT_E_HIP, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
  HIP_TRY(hipFreeAsync(ws, st));
  return rc;
}

bool exec_f32(const rt_exec* ex) { return ex && (ex->flags & RT_EXEC_F32) != 0; }

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
  if (!s) return RT_OK;
  (void)hipSetDevice(s->device);
  (void)hipFree(s->nodes);
  (void)hipFree(s->perlin_perm);
  (void)hipFree(s->status);
  s->f32.release();
  s->f64.release();
  delete s;
  return RT_OK;
}

int rt_scene_create(const rt_scene* sc, int32_t device, rt_device_scene** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!sc || !out) return fail(RT_E_INVALID, "null argument");
  *out = nullptr;
  HostScene H;
  std::string err;
  int rc = rt_host_build_scene(sc, H, err);
  if (rc) return fail(rc, "%s", err.c_str());
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_E_HIP, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RT_E_INVALID, "device %d out of range (%d devices)", device, ndev);
  HIP_TRY(hipSetDevice(device));
  auto* s = new rt_device_scene();
  s->device = device;
  std::vector<int> status(4, 0);
  if ((rc = upload(&s->nodes, H.nodes)) || (rc = upload(&s->perlin_perm, H.perlin_perm)) ||
      (rc = upload(&s->status, status)) || (rc = s->f32.upload(H.f32)) || (rc = s->f64.upload(H.f64))) {
    rt_scene_destroy(s);
    return rc;
  }
  s->surface_root = H.surface_root;
  s->leaf_exit_pct = H.leaf_exit_pct;
  s->trav_exit_pct = H.trav_exit_pct;
  s->n_media = H.n_media;
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) s->flat_sets[k] = H.flat_sets[k];
  s->n_nodes = H.n_nodes;
  s->n_prims = H.n_prims;
  s->max_depth = H.max_depth;
  s->stack_depth = H.max_depth > 1 ? H.max_depth : 1;
  s->variant = rt_host_variant(H.flat, H.n_media, H.noise, H.full_mats, H.uv_tex, H.n_instances > 0);
  if ((s->variant & RT_VAR_BASE) != RT_VAR_FLAT) {
    // stage as many top (breadth-first) surface nodes as fit beside the stacks in the per-
    // workgroup budget; env RT_AMD_LDS_NODES caps it (0 disables, for experiments)
    const int room = (RT_LDS_WG_BUDGET - (s->stack_depth + 1) * RT_BLOCK_BVH * (int)sizeof(int)) / 64;
    s->lds_nodes = std::max(0, std::min(H.surface_nodes, room));
    if (const char* e = std::getenv("RT_AMD_LDS_NODES")) s->lds_nodes = std::min(s->lds_nodes, std::max(0, atoi(e)));
  }
  s->f32.resident_blocks =
      rt_render_resident_blocks((const KernelParams*)nullptr, device, s->stack_depth, s->variant, s->lds_nodes);
  s->f64.resident_blocks =
      rt_render_resident_blocks((const KernelParams64*)nullptr, device, s->stack_depth, s->variant, s->lds_nodes);
  if (s->f32.resident_blocks <= 0 || s->f64.resident_blocks <= 0) {
    rt_scene_destroy(s);
    return fail(RT_E_HIP, "occupancy query failed");
  }
  s->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = s;
  return RT_OK;
}

int rt_scene_stats(const rt_device_scene* s, rt_stats* st) {
  if (!s || !st) return fail(RT_E_INVALID, "null argument");
  std::memset(st, 0, sizeof *st);
  st->upload_ms = s->upload_ms;
  st->bvh_nodes = s->n_nodes;
  st->max_stack = s->stack_depth;
  return RT_OK;
}

int rt_render_async(const rt_device_scene* s, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                    void* d_out_rgb, void* hip_stream) {
  if (!s || !d_out_rgb || !ex) return fail(RT_E_INVALID, "null argument");
  if (ex->n_devices != 0) return fail(RT_E_INVALID, "rt_render_async renders on the scene's device (n_devices = 0)");
  if (exec_f32(ex)) return render_async<float>(s, cs, seed, ex, (float*)d_out_rgb, hip_stream);
  return render_async<double>(s, cs, seed, ex, (double*)d_out_rgb, hip_stream);
}

int rt_render(const rt_camera_settings* cs, const rt_scene* scene, uint64_t seed, const rt_exec* ex, void* out_rgb,
              rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!cs || !scene || !ex || !out_rgb) return fail(RT_E_INVALID, "null argument");
  int h = rt_host_image_height(cs);
  if (h <= 0 || cs->image_width <= 0) return fail(RT_E_INVALID, "image %dx%d must be non-empty", cs->image_width, h);
  int rows = rt_host_shard_rows(h, ex);
  if (rows < 0) return fail(RT_E_INVALID, "invalid rt_exec");
  if (ex->n_devices < 0 || ex->n_devices > RT_MAX_DEVICES || (ex->n_devices > 0 && !ex->devices))
    return fail(RT_E_INVALID, "invalid device list (%d devices)", ex->n_devices);
  if (ex->n_devices > 0 && ex->n_shards != 1)
    return fail(RT_E_INVALID, "a device list renders the whole image (n_shards must be 1)");
  {  // validate the camera before touching a device
    KernelParams P;
    std::string err;
    int rc = rt_host_make_params(cs, seed, ex, P, err);
    if (rc) return fail(rc, "%s", err.c_str());
  }
  const bool f32 = exec_f32(ex);
  const size_t esize = f32 ? sizeof(float) : sizeof(double);
  const size_t row_bytes = (size_t)cs->image_width * 3 * esize;
  // the parts of this call: one (the rt_exec shard on `device`), or shard k of n_devices on
  // devices[k]; each part renders into its own device buffer on its own stream, concurrently
  const int n_parts = ex->n_devices > 0 ? ex->n_devices : 1;
  struct Part {
    int device = 0;
    rt_exec ex{};
    int rows = 0;
    rt_device_scene* scene = nullptr;  // owned by the first part on its device
    bool owns_scene = false;
    void* d_out = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<char> host;
  };
  std::vector<Part> parts(n_parts);
  int rc = RT_OK;
  for (int k = 0; k < n_parts && !rc; ++k) {
    Part& p = parts[k];
    p.ex = *ex;
    p.ex.n_devices = 0;
    p.ex.devices = nullptr;
    if (ex->n_devices > 0) {
      p.device = ex->devices[k];
      p.ex.device = p.device;
      p.ex.n_shards = n_parts;
      p.ex.shard = k;
    } else {
      p.device = ex->device;
    }
    p.rows = rt_host_shard_rows(h, &p.ex);
    for (int j = 0; j < k; ++j)
      if (parts[j].device == p.device) p.scene = parts[j].scene;  // one upload per device
    if (!p.scene) {
      if ((rc = rt_scene_create(scene, p.device, &p.scene))) break;
      p.owns_scene = true;
    }
    if (hipSetDevice(p.device) != hipSuccess) {
      rc = fail(RT_E_HIP, "hipSetDevice(%d) failed", p.device);
      break;
    }
    const size_t bytes = (size_t)p.rows * row_bytes;
    if (hipMalloc(&p.d_out, bytes ? bytes : 16) != hipSuccess) rc = fail(RT_E_HIP, "hipMalloc(%zu) failed", bytes);
    if (!rc && hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking) != hipSuccess) rc = fail(RT_E_HIP, "stream create");
    if (!rc && (hipEventCreate(&p.e0) != hipSuccess || hipEventCreate(&p.e1) != hipSuccess)) rc = fail(RT_E_HIP, "events");
    if (!rc) {
      (void)hipEventRecord(p.e0, p.st);
      rc = rt_render_async(p.scene, cs, seed, &p.ex, p.d_out, p.st);
      (void)hipEventRecord(p.e1, p.st);
    }
  }
  float ms = 0;
  int status = 0;
  for (int k = 0; k < n_parts && !rc; ++k) {  // every part is in flight: wait, copy back
    Part& p = parts[k];
    float pm = 0;
    int ps = 0;
    (void)hipSetDevice(p.device);
    if (hipStreamSynchronize(p.st) != hipSuccess)
      rc = fail(RT_E_HIP, "render on device %d failed: %s", p.device, hipGetErrorString(hipGetLastError()));
    if (!rc) (void)hipEventElapsedTime(&pm, p.e0, p.e1);
    ms = std::max(ms, pm);
    const size_t bytes = (size_t)p.rows * row_bytes;
    void* dst = out_rgb;
    if (n_parts > 1) {
      p.host.resize(bytes);
      dst = p.host.data();
    }
    if (!rc && hipMemcpy(dst, p.d_out, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RT_E_HIP, "copy back");
    if (!rc && hipMemcpy(&ps, p.scene->status, 4, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RT_E_HIP, "status");
    status |= ps;
  }
  if (!rc && status) rc = fail(RT_E_STACK, "BVH traversal stack overflow");
  if (!rc && n_parts > 1) {  // gather: shard-local row t of part k is global row rt_shard_row(t)
    for (int k = 0; k < n_parts; ++k) {
      const Part& p = parts[k];
      for (int t = 0; t < p.rows; ++t) {
        const int y = ((t / p.ex.row_block) * p.ex.n_shards + p.ex.shard) * p.ex.row_block + (t % p.ex.row_block);
        if (y < h) std::memcpy((char*)out_rgb + (size_t)y * row_bytes, p.host.data() + (size_t)t * row_bytes, row_bytes);
      }
    }
  }
  if (stats && !rc) {
    std::memset(stats, 0, sizeof *stats);
    for (const Part& p : parts)
      if (p.owns_scene) stats->upload_ms += p.scene->upload_ms;
    stats->kernel_ms = ms;
    stats->samples = (int64_t)rows * cs->image_width * cs->samples_per_pixel;
    stats->bvh_nodes = parts[0].scene->n_nodes;
    stats->max_stack = parts[0].scene->max_depth;
    stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  for (Part& p : parts) {
    if (!p.scene) continue;
    (void)hipSetDevice(p.device);
    if (p.st) (void)hipStreamSynchronize(p.st);
    if (p.e0) (void)hipEventDestroy(p.e0);
    if (p.e1) (void)hipEventDestroy(p.e1);
    if (p.st) (void)hipStreamDestroy(p.st);
    (void)hipFree(p.d_out);
  }
  for (Part& p : parts)
    if (p.owns_scene) rt_scene_destroy(p.scene);
  return rc;
}

int rt_encode8_async(const void* d_rgb, int32_t in_f64, uint8_t* d_out, int64_t n_values, int32_t encoding,
                     void* hip_stream) {
  if (!d_rgb || !d_out || n_values < 0) return fail(RT_E_INVALID, "invalid encode arguments");
  if (encoding != 0 && encoding != 1) return fail(RT_E_INVALID, "encoding must be 0 (sRGB) or 1 (sqrt)");
  static double thr[2][256];
  static std::once_flag once[2];
  std::call_once(once[encoding], [&] { rt_host_encode8_thresholds(encoding, thr[encoding]); });
  if (rt_launch_encode8(d_rgb, in_f64 ? 1 : 0, d_out, n_values, thr[encoding], encoding, hip_stream))
    return fail(RT_E_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
  return RT_OK;
}

#if defined(RT_PHASE_PROF)
// diagnostic build only: the BVH kernel's phase counters (rt_trace.h RT_PHASE_PROF), read and zeroed
int rt_prof_read(int f64, unsigned long long* out, int n) {
  return f64 ? rt_prof_read_kernel((const KernelParams64*)nullptr, out, n) : rt_prof_read_kernel((const KernelParams*)nullptr, out, n);
}
#endif

}  // extern "C"
