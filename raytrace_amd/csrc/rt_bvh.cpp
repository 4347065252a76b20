// rt_bvh.cpp — binned SAH BVH2 builder (host).  See rt_bvh.h.
#include "rt_bvh.h"

#include <algorithm>
#include <cmath>
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
  out.max_depth = B.max_depth;
  // primitive slots skip the instance items (each is its own leaf, encoded as RT_INST_CODE)
  std::vector<int> slot(prims.size() + 1, 0);
  for (size_t i = 0; i < prims.size(); ++i) {
    slot[i + 1] = slot[i] + (prims[i].inst < 0 ? 1 : 0);
    if (prims[i].inst < 0) out.order.push_back(prims[i].index);
  }
  // number internal nodes breadth-first: the top levels are the first nodes of the set, which
  // is what the kernel stages in LDS (KernelParams::lds_nodes)
  std::vector<int> dev_index(B.tmp.size(), -1);
  std::vector<int> internal;
  std::vector<int> queue = {root};
  for (size_t head = 0; head < queue.size(); ++head) {
    int id = queue[head];
    if (B.tmp[id].left < 0) continue;
    dev_index[id] = node_base + (int)internal.size();
    internal.push_back(id);
    queue.push_back(B.tmp[id].left);
    queue.push_back(B.tmp[id].right);
  }
  auto enc = [&](int id) -> int {
    const Node& nd = B.tmp[id];
    if (nd.left >= 0) return dev_index[id];
    if (nd.count == 1 && prims[nd.first].inst >= 0) return RT_INST_FLAG | prims[nd.first].inst;
    // leaf: ~(first << RT_LEAF_SHIFT | count - 1); leaves hold <= RT_FLAT_MAX primitives
    return ~(((prim_base + slot[nd.first]) << RT_LEAF_SHIFT) | (nd.count - 1));
  };
  out.n_nodes = (int)internal.size();
  out.nodes.assign((size_t)out.n_nodes * 16, 0.0f);
  for (size_t k = 0; k < internal.size(); ++k) {
    const Node& nd = B.tmp[internal[k]];
    const Box& L = B.tmp[nd.left].box;
    const Box& R = B.tmp[nd.right].box;
    float* f = out.nodes.data() + 16 * k;
    auto pad = [](const Box& b, int a) { return 1e-6 * std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a])) + 1e-7; };
    f[0] = f_down(L.lo[0], pad(L, 0)); f[1] = f_up(L.hi[0], pad(L, 0));
    f[2] = f_down(L.lo[1], pad(L, 1)); f[3] = f_up(L.hi[1], pad(L, 1));
    f[4] = f_down(R.lo[0], pad(R, 0)); f[5] = f_up(R.hi[0], pad(R, 0));
    f[6] = f_down(R.lo[1], pad(R, 1)); f[7] = f_up(R.hi[1], pad(R, 1));
    f[8] = f_down(L.lo[2], pad(L, 2)); f[9] = f_up(L.hi[2], pad(L, 2));
    f[10] = f_down(R.lo[2], pad(R, 2)); f[11] = f_up(R.hi[2], pad(R, 2));
    int l = enc(nd.left), r = enc(nd.right);
    std::memcpy(&f[12], &l, 4);
    std::memcpy(&f[13], &r, 4);
  }
  out.root = enc(root);
}
