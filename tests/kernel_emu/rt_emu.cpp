// rt_emu.cpp — TEST TOOLING: the device logic of raytrace_amd/csrc/rt_trace.h compiled for
// the host, so the kernel's algorithm can be checked against the FP64 oracle without a GPU
// and kernel faults can be reproduced on the CPU.  Never linked into librt_amd.so.
#define RT_HOST_EMU 1
#include <pthread.h>

#include <atomic>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../raytrace_amd/csrc/rt_internal.h"
#include "../../raytrace_amd/csrc/rt_trace.h"

namespace {
thread_local std::string g_err;

struct Job {
  const KernelParams* P;
  int n;
  std::atomic<int> next{0};
  std::atomic<int> overflow{0};
};

void* worker(void* arg) {
  Job* j = (Job*)arg;
  int stack[RT_STACK_DEPTH];
  for (;;) {
    int k = j->next.fetch_add(1);
    if (k >= j->n) break;
    if (rtk::render_pixel(*j->P, k, stack, 1)) j->overflow = 1;
  }
  return nullptr;
}
}  // namespace

extern "C" {
const char* rt_emu_last_error(void) { return g_err.c_str(); }

int rt_emu_render(const rt_camera_settings* cs, const rt_scene* sc, uint64_t seed, const rt_exec* ex, float* out,
                  int nthreads) {
  HostScene H;
  int rc = rt_host_build_scene(sc, H, g_err);
  if (rc) return rc;
  KernelParams P = {};
  rc = rt_host_make_params(cs, seed, ex, P, g_err);
  if (rc) return rc;
  P.nodes = H.nodes.data();
  P.prims = H.prims.data();
  P.prim_mat = H.prim_mat.data();
  P.prim_uv = H.prim_uv.data();
  P.mats = H.mats.data();
  P.texs = H.texs.data();
  P.motions = H.motions.data();
  P.uvframes = H.uvframes.data();
  P.out = out;
  P.surface_root = H.surface_root;
  P.n_media = H.n_media;
  for (int k = 0; k < H.n_media; ++k) P.media[k] = H.media[k];
  Job j;
  j.P = &P;
  j.n = P.tile_rows * P.cam.width;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pthread_t th[64];
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], nullptr, worker, &j);
  worker(&j);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], nullptr);
  if (j.overflow) {
    g_err = "BVH traversal stack overflow";
    return RT_E_STACK;
  }
  return RT_OK;
}
}
