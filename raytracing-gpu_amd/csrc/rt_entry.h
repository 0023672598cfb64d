// rt_entry.h -- per-tile entry nodes of the camera packet walk
// (csrc/rt_entry.hip).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_ENTRY_MAX 32           // entry nodes kept per tile (more: start at the root)
#define RT_ENTRY_STACK 128        // the build's per-thread stack
#define RT_ENTRY_ROOT 0xffffffffu // entry_n value: walk from the root

struct EntryParams {
  const float4* node;  // octree nodes (2 float4 each)
  int depth;           // entry depth (root = 0)
  // camera frame (cpu/raytracer.c:82-86): eye, w = u x v, L = film distance;
  // ku = v x w, kv = w x u: a point pos + y projects to film coordinates
  // (k, l) = L (y.ku, y.kv) / (y.w)
  float pos[3], w[3], ku[3], kv[3];
  float L;
  float grow;          // box growth: 2 x the camera rays' largest culling slack
  int W, H, tiles_x, rank, nranks;
  uint32_t ntiles;     // the rank's tiles
  uint32_t* entry_n;   // out, per tile: entries, or RT_ENTRY_ROOT
  uint32_t* entry;     // out, RT_ENTRY_MAX per tile: node indices, near to far
};

extern "C" hipError_t rt_entry_build(const EntryParams* p, hipStream_t s);
