// rt_bvh.h — host-side binned-SAH BVH2 builder for the device layout of rt_internal.h.
//
// The reference's own hierarchy is `bvhTree` (Geometry.hs:368-377: median split on the
// longest axis, one object per leaf) plus linear `group`s that are tested without any
// culling (Geometry.hs:335-347).  The closest hit does not depend on the hierarchy, so the
// library builds its own: binned surface-area heuristic over primitive centroids, up to
// RT_LEAF_MAX primitives per leaf, children stored in the parent (one 64-B node fetch tests
// both children's boxes).
#pragma once
#include <stdint.h>

#include <vector>

#include "rt_internal.h"

struct BuildPrim {
  double lo[3], hi[3];
  int index;      // caller's primitive index (-1 for an instance)
  int inst = -1;  // >= 0: an instance of an instanced object (a single-item leaf, RT_INST_CODE)
};

struct BvhOut {
  std::vector<float> nodes;   // 16 floats per node (4 x float4)
  std::vector<int> order;     // primitive order of the leaves (caller indices; instances excluded)
  int root = 0;               // node index, leaf encoding, or RT_EMPTY_ROOT
  int max_depth = 0;          // deepest root-to-leaf path (bounds the traversal stack)
  int n_nodes = 0;
};

// Builds a BVH over `prims`; node indices start at `node_base`, leaf primitive indices at
// `prim_base` (the position of order[0] in the final primitive array).
// leaf_max: at most this many primitives per leaf (the binned SAH decides below that)
void rt_build_bvh(std::vector<BuildPrim> prims, int node_base, int prim_base, BvhOut& out, int leaf_max = RT_LEAF_MAX);
