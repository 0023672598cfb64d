// rt_shadow.h -- per-node culling multipliers of the shadow walk
// (csrc/rt_shadow.hip, DESIGN.md §2 "Exact shadow rays").  Not part of the
// public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

struct ShadowParams {
  const float4* tri;   // prim-order triangle records (3 float4 each)
  uint32_t nprim;
  const float* light;  // RT_LIGHT_FLOATS (8) per light: type r g b v.xyz pad
  uint32_t nlight;
  const float4* node;  // octree nodes (2 float4 each)
  uint32_t nnode;
  const float4* rec;   // leaf-order records of the tree (q2.y = prim)
  double c[3];         // scene box centre
  double R;            // scene box half-extent (max-norm)
  double eps_rel;      // the shadow walk's slack per unit of (|o - c|_max + R) (host/rt_cull.h)
  double plane_eps;    // its constant part: RT_CULL_PLANE (|c|_max + R) + 1e-6
  double omax_assumed; // point lights: shadow origins with |o - c|_max beyond this are counted unproven
  double reach_cap;    // point lights: the largest error region the cosine bound assumes
  float2* prim_mu;     // out, per prim: (mu, nu)
  float2* node_mu;     // out, per node: max over the subtree
  uint32_t* global;    // out: prims tested by every unshadowed shadow ray
  uint32_t* nglobal;   // out: their count (zeroed by the caller)
};

// prims -> leaves -> interior nodes (depth + 1 upward passes)
extern "C" hipError_t rt_shadow_build(const ShadowParams* p, int depth, hipStream_t s);
