// rt_kernels.h -- parameter block shared by the render kernels and their
// host-side launcher (rt_hip.cpp).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"

#define RT_ACCEL_FLAT_D 0
#define RT_ACCEL_OCTREE_D 1
#define RT_MAT_FLOATS_D 12
#define RT_LIGHT_FLOATS_D 8
#define RT_MAX_DEPTH 32
#define RT_NSTATS 8
// per-lane global overflow area of the traversal stack (entries beyond LDS)
#define RT_SPILL_STACK 112
// tile bands and their counters in KParams::tile_counter (<= 16).  Measured
// (C5): 8 bands, one per XCD, ran 13 % slower than 1 -- one scanline-ordered
// band keeps all 8 XCDs on the same few tile rows, whose geometry then stays
// in the Infinity Cache; 8 stripes at once multiply that working set.
#ifndef RT_BANDS
#define RT_BANDS 1
#endif

// wave-total counters (wave-uniform, so they live in SGPRs; 32-bit per wave,
// widened to 64-bit by the final atomics)
struct WorkCount {
  uint32_t closest, shadow, pixels, nodes, tris, overflow, zero_normal, hits;
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
  uint2* spill;                 // grid*64 lanes x RT_SPILL_STACK stack entries
  rt::f3 scene_c;               // scene box centre
  float scene_cmag;             // max-norm of scene_c
  float scene_r;                // scene box half-extent (max-norm)
  float eps_rel;                // culling slack, rt_cull.h rt_cull_eps()
  int trav;                     // RT_TRAV_LANE / _PACKET / _HYBRID (rt_render.hip)
  int packet_min;               // hybrid: packet walk while >= this many lanes query
  int trav_shadow, packet_min_shadow;  // the same two for shadow (any-hit) queries
  int packet_max_depth;         // closest hit: packet walk only up to this bounce depth
  // camera-ray candidate lists (csrc/rt_cand.hip); cand_start == NULL: none
  const uint32_t* cand_start;   // ntiles_local + 1 offsets into cand
  const uint32_t* cand;         // prims
  const uint32_t* cand_global;  // prims every camera ray tests
  uint32_t n_cand_global;
  const float4* tri_prim;       // prim-order triangle records
  const float* cand_skip;       // per prim: lower bound of new_dist - |pos - o| (depth skip)
};

// min_waves = occupancy target per SIMD (launch bounds of the instantiation:
// 2..5); 0 = default
extern "C" hipError_t rt_launch_render(const KParams* p, int accel, int count_work, int min_waves,
                                       int grid, hipStream_t stream);
extern "C" hipError_t rt_launch_assemble(const float* tiles, float* rgb, int W, int H, int tiles_x,
                                         int ntiles, int nranks, int tiles_per_rank,
                                         hipStream_t stream);
