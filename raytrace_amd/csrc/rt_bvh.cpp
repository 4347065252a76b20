// rt_bvh.cpp — binned SAH BVH builder (host): BVH2 by binned SAH, collapsed to 4-wide nodes with
// 8-bit quantised child boxes.  See rt_bvh.h.
#include "rt_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "rt_internal.h"

namespace {

struct Box {
  double lo[3], hi[3];
  void reset() {
    for (int a = 0; a < 3; ++a) {
      lo[a] = INFINITY;
      hi[a] = -INFINITY;
    }
  }
  void grow(const double* l, const double* h) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], l[a]);
      hi[a] = std::max(hi[a], h[a]);
    }
  }
  void grow(const Box& b) { grow(b.lo, b.hi); }
  double area() const {
    double d[3];
    for (int a = 0; a < 3; ++a) d[a] = std::max(0.0, hi[a] - lo[a]);
    return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
  }
};

struct Node {
  Box box;
  int left = -1, right = -1;  // indices into `tmp` nodes
  int first = 0, count = 0;   // leaf range into the prim order
};

struct Builder {
  std::vector<BuildPrim>& p;
  std::vector<Node> tmp;
  int max_depth = 0;
  int leaf_max = RT_LEAF_MAX;
  explicit Builder(std::vector<BuildPrim>& prims) : p(prims) {}

  bool has_inst(int b, int e) const {
    for (int i = b; i < e; ++i)
      if (p[i].inst >= 0) return true;
    return false;
  }

  Box bounds(int b, int e) const {
    Box bx;
    bx.reset();
    for (int i = b; i < e; ++i) bx.grow(p[i].lo, p[i].hi);
    return bx;
  }

  int build(int b, int e, int depth) {
    max_depth = std::max(max_depth, depth);
    int id = (int)tmp.size();
    tmp.emplace_back();
    tmp[id].box = bounds(b, e);
    int n = e - b;
    // instances are single-item leaves (RT_INST_CODE children), never mixed with primitives
    const bool inst = has_inst(b, e);
    if (n == 1 || (!inst && (n <= 2 || (depth == 0 && n <= RT_FLAT_MAX)))) {  // tiny sets: one flat, coherent leaf
      tmp[id].first = b;
      tmp[id].count = n;
      return id;
    }
    // centroid bounds
    double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = b; i < e; ++i)
      for (int a = 0; a < 3; ++a) {
        double c = 0.5 * (p[i].lo[a] + p[i].hi[a]);
        clo[a] = std::min(clo[a], c);
        chi[a] = std::max(chi[a], c);
      }
    const int NB = 16;
    double best_cost = INFINITY;
    int best_axis = -1, best_split = -1;
    for (int a = 0; a < 3; ++a) {
      double ext = chi[a] - clo[a];
      if (!(ext > 0)) continue;
      Box bb[NB];
      int cnt[NB] = {0};
      for (int k = 0; k < NB; ++k) bb[k].reset();
      for (int i = b; i < e; ++i) {
        double c = 0.5 * (p[i].lo[a] + p[i].hi[a]);
        int k = std::min(NB - 1, (int)((c - clo[a]) / ext * NB));
        cnt[k]++;
        bb[k].grow(p[i].lo, p[i].hi);
      }
      Box lb[NB], rb[NB];
      int lc[NB], rc[NB];
      Box acc;
      acc.reset();
      int c = 0;
      for (int k = 0; k < NB; ++k) {
        acc.grow(bb[k]);
        c += cnt[k];
        lb[k] = acc;
        lc[k] = c;
      }
      acc.reset();
      c = 0;
      for (int k = NB - 1; k >= 0; --k) {
        acc.grow(bb[k]);
        c += cnt[k];
        rb[k] = acc;
        rc[k] = c;
      }
      for (int k = 0; k < NB - 1; ++k) {
        if (lc[k] == 0 || rc[k + 1] == 0) continue;
        double cost = lb[k].area() * lc[k] + rb[k + 1].area() * rc[k + 1];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = a;
          best_split = k;
        }
      }
    }
    double leaf_cost = tmp[id].box.area() * n;
    double node_area = tmp[id].box.area();
    int mid;
    if (best_axis < 0) {
      // all centroids coincide: split in the middle of the index range
      if (n <= leaf_max && !inst) {
        tmp[id].first = b;
        tmp[id].count = n;
        return id;
      }
      mid = b + n / 2;
    } else {
      // SAH with traversal cost ~ 1 box pair ~ 1 primitive test
      if (n <= leaf_max && !inst && leaf_cost <= node_area * 1.0 + best_cost) {
        tmp[id].first = b;
        tmp[id].count = n;
        return id;
      }
      double ext = chi[best_axis] - clo[best_axis];
      BuildPrim* it = std::partition(p.data() + b, p.data() + e, [&](const BuildPrim& q) {
        double c = 0.5 * (q.lo[best_axis] + q.hi[best_axis]);
        int k = std::min(NB - 1, (int)((c - clo[best_axis]) / ext * NB));
        return k <= best_split;
      });
      mid = (int)(it - p.data());
      if (mid == b || mid == e) mid = b + n / 2;
    }
    int l = build(b, mid, depth + 1);
    int r = build(mid, e, depth + 1);
    tmp[id].left = l;
    tmp[id].right = r;
    return id;
  }
};

inline float f_down(double x, double pad) { return std::nextafter((float)(x - pad), -INFINITY); }
inline float f_up(double x, double pad) { return std::nextafter((float)(x + pad), INFINITY); }

// A child box as the device decodes it: plane = fma(q, s, origin) in FP32 with q an 8-bit code,
// s = 2^e and origin = k s for an integer k with |k| + 255 < 2^24, so every decoded plane is an
// exactly representable float (the fma is exact).  Codes round OUTWARD from the padded float box,
// so the decoded box contains it: traversal tests a superset of the leaves the float box would
// give, and the closest hit, keyed by (t, depth-first order), cannot change.
struct Quant {
  float origin[3], scale[3];
  uint8_t lo[4][3], hi[4][3];
};

inline float decode(int q, float s, float o) { return std::fma((float)q, s, o); }

// the smallest scale 2^e for which [lo, hi] fits 255 steps from an origin k 2^e with exact decode
void axis_frame(float lo, float hi, float& origin, float& scale) {
  int e = -140;
  const double ext = (double)hi - (double)lo;
  if (ext > 0) e = std::max(e, (int)std::floor(std::log2(ext / 255.0)) - 1);
  for (;; ++e) {
    const double s = std::ldexp(1.0, e);
    const double k = std::floor((double)lo / s);
    if (std::fabs(k) + 256.0 >= 16777216.0) continue;  // decode would round
    if (std::ceil(((double)hi - k * s) / s) > 255.0) continue;
    if (e < -126) continue;  // keep s and the planes normal floats
    origin = (float)(k * s);
    scale = (float)s;
    return;
  }
}

int code_down(float v, float s, float o) {  // largest q with decode(q) <= v
  int q = (int)std::floor(((double)v - (double)o) / (double)s);
  q = std::max(0, std::min(255, q));
  while (q > 0 && decode(q, s, o) > v) --q;
  return q;
}
int code_up(float v, float s, float o) {  // smallest q with decode(q) >= v
  int q = (int)std::ceil(((double)v - (double)o) / (double)s);
  q = std::max(0, std::min(255, q));
  while (q < 255 && decode(q, s, o) < v) ++q;
  return q;
}

}  // namespace

void rt_build_bvh(std::vector<BuildPrim> prims, int node_base, int prim_base, BvhOut& out, int leaf_max) {
  out.nodes.clear();
  out.order.clear();
  out.n_nodes = 0;
  out.max_depth = 0;
  if (prims.empty()) {
    out.root = RT_EMPTY_ROOT;
    return;
  }
  Builder B(prims);
  B.leaf_max = leaf_max;
  int root = B.build(0, (int)prims.size(), 0);
  // primitive slots skip the instance items (each is its own leaf, encoded as RT_INST_CODE)
  std::vector<int> slot(prims.size() + 1, 0);
  for (size_t i = 0; i < prims.size(); ++i) {
    slot[i + 1] = slot[i] + (prims[i].inst < 0 ? 1 : 0);
    if (prims[i].inst < 0) out.order.push_back(prims[i].index);
  }
  // BVH2 -> BVH4: a node's children are its two children, then repeatedly the internal child of
  // largest surface area is replaced by its two children, up to four (Wald et al. 2008's collapse)
  const int T = (int)B.tmp.size();
  std::vector<std::vector<int>> kids(T);
  auto collapse = [&](int id) {
    std::vector<int> c = {B.tmp[id].left, B.tmp[id].right};
    while (c.size() < 4) {
      int best = -1;
      double best_area = -1.0;
      for (int j = 0; j < (int)c.size(); ++j)
        if (B.tmp[c[j]].left >= 0 && B.tmp[c[j]].box.area() > best_area) {
          best_area = B.tmp[c[j]].box.area();
          best = j;
        }
      if (best < 0) break;
      const int n = c[best];
      c[best] = B.tmp[n].left;
      c.insert(c.begin() + best + 1, B.tmp[n].right);
    }
    kids[id] = c;
  };
  // number the 4-wide internal nodes breadth-first: the top levels are the first nodes of the
  // set, which is what the kernel stages in LDS (KernelParams::lds_nodes)
  std::vector<int> dev_index(T, -1);
  std::vector<int> internal;
  std::vector<int> queue = {root};
  for (size_t head = 0; head < queue.size(); ++head) {
    int id = queue[head];
    if (B.tmp[id].left < 0) continue;
    collapse(id);
    dev_index[id] = node_base + (int)internal.size();
    internal.push_back(id);
    for (int c : kids[id]) queue.push_back(c);
  }
  auto enc = [&](int id) -> int {
    const Node& nd = B.tmp[id];
    if (nd.left >= 0) return dev_index[id];
    if (nd.count == 1 && prims[nd.first].inst >= 0) return RT_INST_FLAG | prims[nd.first].inst;
    // leaf: ~(first << RT_LEAF_SHIFT | count - 1); leaves hold <= RT_FLAT_MAX primitives
    return ~(((prim_base + slot[nd.first]) << RT_LEAF_SHIFT) | (nd.count - 1));
  };
  // traversal stack a root-to-leaf walk can need: a node pushes at most (children - 1) entries
  std::vector<int> need(T, 0);
  for (int k = (int)internal.size() - 1; k >= 0; --k) {  // children come later in breadth-first order
    const int id = internal[k];
    int deepest = 0;
    for (int c : kids[id]) deepest = std::max(deepest, need[c]);
    need[id] = (int)kids[id].size() - 1 + deepest;
  }
  out.max_depth = std::max(1, need[root]);
  out.n_nodes = (int)internal.size();
  out.nodes.assign((size_t)out.n_nodes * 16, 0.0f);
  auto pad = [](const Box& b, int a) { return 1e-6 * std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a])) + 1e-7; };
  for (size_t k = 0; k < internal.size(); ++k) {
    const std::vector<int>& c = kids[internal[k]];
    // the children's float boxes, rounded outward and padded (conservative for binary64 leaves)
    float flo[4][3], fhi[4][3];
    float ulo[3] = {INFINITY, INFINITY, INFINITY}, uhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t j = 0; j < c.size(); ++j) {
      const Box& bx = B.tmp[c[j]].box;
      for (int a = 0; a < 3; ++a) {
        flo[j][a] = f_down(bx.lo[a], pad(bx, a));
        fhi[j][a] = f_up(bx.hi[a], pad(bx, a));
        ulo[a] = std::min(ulo[a], flo[j][a]);
        uhi[a] = std::max(uhi[a], fhi[j][a]);
      }
    }
    Quant Q{};
    for (int a = 0; a < 3; ++a) axis_frame(ulo[a], uhi[a], Q.origin[a], Q.scale[a]);
    uint32_t qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
    for (size_t j = 0; j < c.size(); ++j)
      for (int a = 0; a < 3; ++a) {
        const int l = code_down(flo[j][a], Q.scale[a], Q.origin[a]);
        const int h = code_up(fhi[j][a], Q.scale[a], Q.origin[a]);
        qlo[a] |= (uint32_t)l << (8 * j);
        qhi[a] |= (uint32_t)h << (8 * j);
      }
    // layout (rt_internal.h, 4 x float4): (ox, oy, oz, sx) (sy, sz, qlo.x, qhi.x)
    // (qlo.y, qhi.y, qlo.z, qhi.z) (child 0..3); byte j of a code word is child j
    float* f = out.nodes.data() + 16 * k;
    f[0] = Q.origin[0];
    f[1] = Q.origin[1];
    f[2] = Q.origin[2];
    f[3] = Q.scale[0];
    f[4] = Q.scale[1];
    f[5] = Q.scale[2];
    std::memcpy(&f[6], &qlo[0], 4);
    std::memcpy(&f[7], &qhi[0], 4);
    std::memcpy(&f[8], &qlo[1], 4);
    std::memcpy(&f[9], &qhi[1], 4);
    std::memcpy(&f[10], &qlo[2], 4);
    std::memcpy(&f[11], &qhi[2], 4);
    for (int j = 0; j < 4; ++j) {
      const int r = j < (int)c.size() ? enc(c[j]) : RT_EMPTY_ROOT;
      std::memcpy(&f[12 + j], &r, 4);
    }
  }
  out.root = enc(root);
}

// the decoded (exact float) box of child j of a 4-wide node, as the kernel computes it
void rt_bvh4_child_box(const float* node, int j, float lo[3], float hi[3]) {
  uint32_t w[6];
  std::memcpy(w, node + 6, sizeof w);
  const float o[3] = {node[0], node[1], node[2]}, s[3] = {node[3], node[4], node[5]};
  for (int a = 0; a < 3; ++a) {
    lo[a] = decode((int)((w[2 * a] >> (8 * j)) & 255u), s[a], o[a]);
    hi[a] = decode((int)((w[2 * a + 1] >> (8 * j)) & 255u), s[a], o[a]);
  }
}
