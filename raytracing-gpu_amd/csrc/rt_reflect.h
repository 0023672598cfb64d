// rt_reflect.h -- per-node bounds of the exact reflection walk
// (csrc/rt_reflect.hip, DESIGN.md §2 "Reflection rays: exact by proof").
// Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Largest |d| a reflection query may have for the floor bound (float accept
// => |a| >= 1e-7f - E_a, so a_lb / |d| >= 1e-7f / |d| - E_a / |d|).  Camera
// directions are normalize()d (|d| <= 1 + 2^-22) and ray_bounce never
// lengthens d beyond its rounding (|d'|^2 = |d|^2 - 4 (N.d)^2 (1 - |N|^2) with
// |N| <= 1 + a few ulps: N interpolates unit normals with barycentric weights
// in [0, 1], cpu/hit.c:38-40, cpu/ray.c:16-25); a query past it is counted
// (rt_stats.closest_unproven -> RT_EINEXACT), never assumed.
#define RT_RF_DLMAX 1.0625f

struct ReflParams {
  const float4* node;  // octree nodes (2 float4 each, host/rt_cull.h)
  uint32_t nnode;
  const float4* rec;   // leaf-order triangle records (3 float4 each)
  float4* node_rf;     // out: 3 float4 per node (rt_render.hip RfNode)
  float* node_phi;     // scratch: the normal cone's half-angle per node (radians; >= pi/2: none)
  uint32_t* unbounded; // out: leaves holding a triangle no bound covers (their ancestors are always visited)
};

// leaves, then depth + 1 upward passes
extern "C" hipError_t rt_reflect_build(const ReflParams* p, int depth, hipStream_t s);
