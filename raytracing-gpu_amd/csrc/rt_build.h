// rt_build.h -- device octree build (rt_build.hip); internal, not the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

struct rt_device_build_opts {
  int leaf_cap;    // a node with <= leaf_cap references is a leaf
  int clip_level;  // triangles bigger than a cell of this level are referenced per cell
};

struct rt_device_tree {
  float4* node;    // nnode x 2 float4 (host/rt_cull.h), hipMalloc'd, caller frees
  float4* tri;     // nref x 3 float4 records in leaf order, hipMalloc'd, caller frees
  uint32_t nref, nnode, depth, leaves, max_leaf;
};

// d_rec = ntri triangle records in prim order (host/rt_internal.h layout);
// scene_lo/hi = the scene box.  Synchronises s.
extern "C" hipError_t rt_device_build_octree(const float4* d_rec, uint32_t ntri,
                                             const float scene_lo[3], const float scene_hi[3],
                                             const rt_device_build_opts* opts, hipStream_t s,
                                             rt_device_tree* out);
