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
// The device's FP32 reciprocal (v_rcp_f32) is within 1 ulp of 1/x, not correctly rounded:
// rt_emu_set_rcp_ulps(k) makes the emulator's reciprocal the IEEE result moved k ulps (k < 0:
// toward -inf), so the node test's conservativeness check covers both roundings the device can
// produce (tests/test_node_test.py).
namespace rt_emu {
int rcp_ulps = 0;
}
static inline float rt_emu_rcpf(float x) {
  float r = 1.0f / x;
  for (int k = rt_emu::rcp_ulps; k > 0; --k) r = std::nextafter(r, HUGE_VALF);
  for (int k = rt_emu::rcp_ulps; k < 0; ++k) r = std::nextafter(r, -HUGE_VALF);
  return r;
}
#define RT_RCPF(x) rt_emu_rcpf(x)
#define RT_F64 0
#include "../../raytrace_amd/csrc/rt_trace.h"
namespace emu32 {
#include "emu_body.h"
}  // namespace emu32
#undef RT_F64
#define RT_F64 1
#include "../../raytrace_amd/csrc/rt_trace.h"
namespace emu64 {
#include "emu_body.h"
}  // namespace emu64

namespace rt_emu {
thread_local long long counters[4];
}

namespace {
thread_local std::string g_err;
}  // namespace

extern "C" {
const char* rt_emu_last_error(void) { return g_err.c_str(); }

// counters (optional, 4 values): BVH nodes visited, primitives tested, segments, samples.
// f64 = 1: the binary64 kernel (out: doubles), else the FP32 kernel (out: floats)
int rt_emu_render(const rt_camera_settings* cs, const rt_scene* sc, uint64_t seed, const rt_exec* ex, void* out,
                  int nthreads, int chunk, long long* counters, int f64) {
  HostScene H;
  int rc = rt_host_build_scene(sc, H, g_err);
  if (rc) return rc;
  if (f64) return emu64::render(H, cs, seed, ex, (double*)out, nthreads, chunk, counters, g_err);
  return emu32::render(H, cs, seed, ex, (float*)out, nthreads, chunk, counters, g_err);
}
}

extern "C" {
void rt_emu_set_rcp_ulps(int k) { rt_emu::rcp_ulps = k; }

// The binary64 kernel's FP32 BVH node test (rtk64::prep_ray + node_slabs_f32) for n rays, each
// against one box given as both children of a node: box = (xmin, xmax, ymin, ymax, zmin, zmax)
// floats, o / d / (tmin, tmax) doubles; accept[i] = 1 when the kernel would enter the box.
void rt_emu_node_test_f64(int n, const double* o, const double* d, const float* box, const double* tr, int* accept) {
  for (int i = 0; i < n; ++i) {
    rtk64::RayCtx R{};
    R.o = rtk64::f3{o[3 * i], o[3 * i + 1], o[3 * i + 2]};
    R.d = rtk64::f3{d[3 * i], d[3 * i + 1], d[3 * i + 2]};
    rtk64::prep_ray(R);
    const float* b = box + 6 * i;
    const rtk64::v4f n0{b[0], b[1], b[2], b[3]}, n1{b[0], b[1], b[2], b[3]}, n2{b[4], b[5], b[4], b[5]};
    float ln, lf, rn, rf;
    rtk64::node_slabs_f32(R, n0, n1, n2, (float)tr[2 * i], (float)tr[2 * i + 1], ln, lf, rn, rf);
    accept[i] = (ln <= lf ? 1 : 0) | (rn <= rf ? 2 : 0);
  }
}

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
  info[5] = H.n_boxes;
  // BVH scenes: primitives tested before the surface BVH (prefix records + box-group faces)
  int pre = 0;
  if (!H.flat) {
    const DevFlatSet& F = H.flat_sets[0];
    pre = F.end - F.first;
    for (int b = F.box_first; b < F.box_end; ++b)
      for (int f = 0; f < 6; ++f) pre += ((H.f32.boxes[b].ord_code >> (5 * f)) & 31) != RT_BOX_NO_FACE;
  }
  info[6] = pre;
  info[7] = H.leaf_kind;
  return RT_OK;
}
}
