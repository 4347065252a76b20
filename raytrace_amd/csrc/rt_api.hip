// rt_api.hip — the C-ABI entry points of include/rt.h: scene build (rt_build.cpp), upload to
// HBM, kernel launch (rt_kernel.hip), error reporting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

}  // namespace

struct rt_device_scene {
  int device = 0;
  float* nodes = nullptr;
  float* prims = nullptr;
  DevMaterial* prim_shade = nullptr;
  float* prim_uv = nullptr;
  DevMaterial* mats = nullptr;
  DevTexture* texs = nullptr;
  float* motions = nullptr;
  float* uvframes = nullptr;
  float* texels = nullptr;
  int* perlin_perm = nullptr;
  float* perlin_grad = nullptr;
  float* flat_recs = nullptr;
  DevBox* boxes = nullptr;
  int leaf_exit_pct = 100;
  int trav_exit_pct = 50;
  int* status = nullptr;
  int surface_root = RT_EMPTY_ROOT;
  int n_media = 0;
  DevMedium media[RT_MAX_MEDIA];
  DevFlatSet flat_sets[1 + RT_MAX_MEDIA];
  int n_nodes = 0, n_prims = 0, max_depth = 0;
  int stack_depth = 1;       // LDS stack entries per lane
  int lds_nodes = 0;         // top surface-BVH nodes staged in LDS per workgroup
  int variant = RT_VAR_FLAT;  // render-kernel variant (rt_internal.h RT_VAR_*)
  int resident_blocks = 0;   // render-kernel workgroups resident on the device at that stack depth
  double upload_ms = 0;
};

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return g_err.c_str(); }

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
  (void)hipFree(s->prims);
  (void)hipFree(s->prim_shade);
  (void)hipFree(s->prim_uv);
  (void)hipFree(s->mats);
  (void)hipFree(s->texs);
  (void)hipFree(s->motions);
  (void)hipFree(s->uvframes);
  (void)hipFree(s->texels);
  (void)hipFree(s->perlin_perm);
  (void)hipFree(s->perlin_grad);
  (void)hipFree(s->flat_recs);
  (void)hipFree(s->boxes);
  (void)hipFree(s->status);
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
  if ((rc = upload(&s->nodes, H.nodes)) || (rc = upload(&s->prims, H.prims)) ||
      (rc = upload(&s->prim_shade, H.prim_shade)) || (rc = upload(&s->prim_uv, H.prim_uv)) ||
      (rc = upload(&s->mats, H.mats)) || (rc = upload(&s->texs, H.texs)) || (rc = upload(&s->motions, H.motions)) ||
      (rc = upload(&s->uvframes, H.uvframes)) || (rc = upload(&s->flat_recs, H.flat_recs)) || (rc = upload(&s->boxes, H.boxes)) ||
      (rc = upload(&s->texels, H.texels)) || (rc = upload(&s->perlin_perm, H.perlin_perm)) ||
      (rc = upload(&s->perlin_grad, H.perlin_grad)) ||
      (rc = upload(&s->status, status))) {
    rt_scene_destroy(s);
    return rc;
  }
  s->surface_root = H.surface_root;
  s->leaf_exit_pct = H.leaf_exit_pct;
  s->trav_exit_pct = H.trav_exit_pct;
  s->n_media = H.n_media;
  for (int k = 0; k < H.n_media; ++k) s->media[k] = H.media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) s->flat_sets[k] = H.flat_sets[k];
  s->n_nodes = H.n_nodes;
  s->n_prims = H.n_prims;
  s->max_depth = H.max_depth;
  s->stack_depth = H.max_depth > 1 ? H.max_depth : 1;
  s->variant = rt_host_variant(H.flat, H.n_media, H.noise, H.full_mats, H.uv_tex);
  if ((s->variant & RT_VAR_BASE) != RT_VAR_FLAT) {
    // stage as many top (breadth-first) surface nodes as fit beside the stacks in the per-
    // workgroup budget; env RT_AMD_LDS_NODES caps it (0 disables, for experiments)
    const int room = (RT_LDS_WG_BUDGET - (s->stack_depth + 1) * RT_BLOCK_BVH * (int)sizeof(int)) / 64;
    s->lds_nodes = std::max(0, std::min(H.surface_nodes, room));
    if (const char* e = std::getenv("RT_AMD_LDS_NODES")) s->lds_nodes = std::min(s->lds_nodes, std::max(0, atoi(e)));
  }
  s->resident_blocks = rt_render_resident_blocks(device, s->stack_depth, s->variant, s->lds_nodes);
  if (s->resident_blocks <= 0) {
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
                    float* d_out_rgb, void* hip_stream) {
  if (!s || !d_out_rgb) return fail(RT_E_INVALID, "null argument");
  KernelParams P;
  std::memset(&P, 0, sizeof P);
  std::string err;
  int rc = rt_host_make_params(cs, seed, ex, P, err);
  if (rc) return fail(rc, "%s", err.c_str());
  P.nodes = s->nodes;
  P.prims = s->prims;
  P.prim_shade = s->prim_shade;
  P.prim_uv = s->prim_uv;
  P.mats = s->mats;
  P.texs = s->texs;
  P.motions = s->motions;
  P.uvframes = s->uvframes;
  P.texels = s->texels;
  P.perlin_perm = s->perlin_perm;
  P.perlin_grad = s->perlin_grad;
  P.flat_recs = s->flat_recs;
  P.boxes = s->boxes;
  P.status = s->status;
  P.out = d_out_rgb;
  P.surface_root = s->surface_root;
  P.leaf_exit_pct = s->leaf_exit_pct;
  P.surface_prefix = (s->variant & RT_VAR_BASE) != RT_VAR_FLAT && s->n_nodes > 0 ? 1 : 0;
  P.n_media = s->n_media;
  for (int k = 0; k < s->n_media; ++k) P.media[k] = s->media[k];
  for (int k = 0; k <= RT_MAX_MEDIA; ++k) P.flat_sets[k] = s->flat_sets[k];
  P.stack_depth = s->stack_depth;
  P.lds_nodes = s->lds_nodes;
  P.n_prims = s->n_prims;
  rt_host_plan_work(P, (long long)s->resident_blocks * rt_block_of(s->variant));
  P.trav_exit_pct = s->trav_exit_pct;
  HIP_TRY(hipSetDevice(s->device));
  // stream-ordered workspace: fixed-point sums, NaN flags, queue counter (graph-capturable)
  const size_t tile_pixels = (size_t)P.tile_rows * P.cam.width;
  const size_t off_flag = tile_pixels * 3 * sizeof(long long);
  const size_t off_ctr = off_flag + ((tile_pixels * sizeof(unsigned) + 255) & ~(size_t)255);
  const size_t bytes = off_ctr + 256 * 8;  // up to 8 queue head words (rt_kernel.hip RT_QUEUES)
  hipStream_t st = (hipStream_t)hip_stream;
  char* ws = nullptr;
  HIP_TRY(hipMallocAsync((void**)&ws, bytes, st));
  HIP_TRY(hipMemsetAsync(ws, 0, bytes, st));
  P.accum = (unsigned long long*)ws;
  P.nanflag = (unsigned int*)(ws + off_flag);
  P.counter = (int*)(ws + off_ctr);
  rc = RT_OK;
  if (rt_launch_render(P, s->resident_blocks, s->variant, hip_stream) || rt_launch_resolve(P, hip_stream))
    rc = fail(RT_E_HIP, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
  HIP_TRY(hipFreeAsync(ws, st));
  return rc;
}

int rt_render(const rt_camera_settings* cs, const rt_scene* scene, uint64_t seed, const rt_exec* ex, float* out_rgb,
              rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!cs || !scene || !ex || !out_rgb) return fail(RT_E_INVALID, "null argument");
  int h = rt_host_image_height(cs);
  if (h <= 0 || cs->image_width <= 0) return fail(RT_E_INVALID, "image %dx%d must be non-empty", cs->image_width, h);
  int rows = rt_host_shard_rows(h, ex);
  if (rows < 0) return fail(RT_E_INVALID, "invalid rt_exec");
  {  // validate the camera before touching the device
    KernelParams P;
    std::string err;
    int rc = rt_host_make_params(cs, seed, ex, P, err);
    if (rc) return fail(rc, "%s", err.c_str());
  }
  rt_device_scene* s = nullptr;
  int rc = rt_scene_create(scene, ex->device, &s);
  if (rc) return rc;
  size_t bytes = (size_t)rows * cs->image_width * 3 * sizeof(float);
  float* d_out = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int status = 0;
  float ms = 0;
  if (hipMalloc((void**)&d_out, bytes ? bytes : 16) != hipSuccess) rc = fail(RT_E_HIP, "hipMalloc(%zu) failed", bytes);
  if (!rc && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) rc = fail(RT_E_HIP, "stream create");
  if (!rc && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) rc = fail(RT_E_HIP, "events");
  if (!rc) {
    (void)hipEventRecord(e0, st);
    rc = rt_render_async(s, cs, seed, ex, d_out, st);
    (void)hipEventRecord(e1, st);
  }
  if (!rc && hipStreamSynchronize(st) != hipSuccess)
    rc = fail(RT_E_HIP, "render failed: %s", hipGetErrorString(hipGetLastError()));
  if (!rc) (void)hipEventElapsedTime(&ms, e0, e1);
  if (!rc && hipMemcpy(out_rgb, d_out, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RT_E_HIP, "copy back");
  if (!rc && hipMemcpy(&status, s->status, 4, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RT_E_HIP, "status");
  if (!rc && status) rc = fail(RT_E_STACK, "BVH traversal stack overflow");
  if (stats && !rc) {
    std::memset(stats, 0, sizeof *stats);
    stats->upload_ms = s->upload_ms;
    stats->kernel_ms = ms;
    stats->samples = (int64_t)rows * cs->image_width * cs->samples_per_pixel;
    stats->bvh_nodes = s->n_nodes;
    stats->max_stack = s->max_depth;
    stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  (void)hipFree(d_out);
  rt_scene_destroy(s);
  return rc;
}

int rt_encode8_async(const float* d_rgb, uint8_t* d_out, int64_t n_values, int32_t encoding, void* hip_stream) {
  if (!d_rgb || !d_out || n_values < 0) return fail(RT_E_INVALID, "invalid encode arguments");
  if (encoding != 0 && encoding != 1) return fail(RT_E_INVALID, "encoding must be 0 (sRGB) or 1 (sqrt)");
  if (rt_launch_encode8(d_rgb, d_out, n_values, encoding, hip_stream))
    return fail(RT_E_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
  return RT_OK;
}

}  // extern "C"
