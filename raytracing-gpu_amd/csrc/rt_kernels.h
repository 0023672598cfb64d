// rt_kernels.h -- parameter block shared by the render kernels and their
// host-side launcher (rt_hip.cpp).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"

#define RT_ACCEL_FLAT_D 0
#define RT_ACCEL_OCTREE_D 1
#define RT_LEAF_FLAG_D 0x80000000u
#define RT_MAT_FLOATS_D 12
#define RT_LIGHT_FLOATS_D 8
#define RT_MAX_DEPTH 32
#define RT_NSTATS 8

struct WorkCount {
  unsigned long long closest, shadow, pixels, nodes, tris, overflow, zero_normal, hits;
};

struct KParams {
  const float4* tri;    // triangle records, 3 float4 each (host/rt_internal.h)
  const float* nrm;     // 9 floats per prim
  const float* mat;     // RT_MAT_FLOATS_D per object
  const float* light;   // RT_LIGHT_FLOATS_D per light
  const float4* node;   // 2 float4 per octree node (NULL for FLAT)
  uint32_t nrec, nlight;
  rt::f3 u, v, C, pos;  // camera frame (cpu/raytracer.c:82-86)
  int W, H;
  int tiles_x, ntiles_total, rank, nranks, ntiles_local;
  float* out;                   // rank's tile buffer
  uint32_t* tile_counter;       // zeroed before launch
  unsigned long long* stats;    // RT_NSTATS counters, zeroed before launch
  rt::f3 scene_c;               // scene box centre
  float scene_r;                // scene box half-diagonal (max-norm)
  float eps_rel, eps_abs;       // culling slack: eps = eps_rel*(|o-c|+r)+eps_abs
};

extern "C" hipError_t rt_launch_render(const KParams* p, int accel, int count_work, int grid,
                                       hipStream_t stream);
extern "C" hipError_t rt_launch_assemble(const float* tiles, float* rgb, int W, int H, int tiles_x,
                                         int ntiles, int nranks, int tiles_per_rank,
                                         hipStream_t stream);
