// rt_lightbuf.h -- light buffers: per-light cell grids of triangle lists for
// the shadow queries of the default walk (DESIGN.md §4 "Light buffers").
//
// A directional light's shadow rays are parallel (direction -l.v exactly,
// cpu/light.c:53) and a point light's all pass through the light
// (cpu/light.c:78); so a grid over the light's view -- the scene projected
// along the light's direction, or a cube map around the point light -- tells
// each shadow ray which triangles it can meet, without a tree walk
// (Haines & Greenberg's light buffer).  Each cell lists the triangles whose
// footprint, grown by the shadow walk's culling slack, touches it, ordered by
// how far toward the light they reach, so a query tests only the triangles
// that can lie on its ray and stops at the first any-hit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_LB_NONE 0u  // no buffer: the light's shadow queries walk the octree
#define RT_LB_DIR 1u   // directional light: a grid over the projection along -l.v
#define RT_LB_POINT 2u // point light: a cube map of n x n cells per face around l.v

// Device view of one light's buffer (the shade kernel reads it through
// KParams::lbuf, indexed by light).
struct RtLightBuf {
  uint32_t kind;
  uint32_t nx, ny;   // DIR: grid cells per axis; POINT: n = nx per face side (ny = nx)
  float u[3], v[3], w[3];  // DIR: the grid's axes u, v and w (toward the light)
  float u0, v0, inv_cs;    // DIR: grid origin and 1 / cell size
  float half_n;            // POINT: nx / 2
  const uint32_t* start;   // per cell: first entry; [ncell] = total
  // per entry: the triangle's record (3 float4, as the prim-order records)
  // with its prim slot (rec[3k+2].y) holding the entry's key; ascending
  // within a cell, a query stops at key > its limit.  One contiguous 48 B
  // load per test: no prim -> record indirection on the query's chain.
  const float4* rec;
  const uint32_t* global;  // prims every query of this light tests (footprint unbounded)
  uint32_t nglobal;
  // proven footprints (LBParams::proven) hold for shadow rays leaving this
  // box (floats inside the build's box); the shade pass counts the others
  // (rt_stats.shadow_unproven -> RT_EINEXACT)
  uint32_t proven;
  float olo[3], ohi[3];
};

// Build parameters (host -> rt_lightbuf_build).
struct LBParams {
  const float4* tri;  // prim-order records, 3 float4 each
  uint32_t nprim;
  uint32_t kind;
  double lv[3];       // the light's v (direction for DIR, position for POINT)
  double slack;       // >= the shadow walk's culling slack eps(o) for every surface origin
  double s1;          // >= |x| + |y| + |z| over the scene box (rounding of the projections)
  double dmax;        // POINT: >= the distance from the light to any scene point
  double box_lo[3], box_hi[3];  // a box holding every triangle and shadow-ray origin
  uint32_t target_cells;
  // 0: footprints grown by the walk's slack (tested exactness, like the
  // walk); 1: grown by the reference float test's proven error region for the
  // light's ray family (exact by construction, DESIGN.md §2 "Shadow rays")
  uint32_t proven;
  // test hook (rt_hip_set_lightbuf_entry_cap): fail a build of more entries
  // than this (0: only the 2^31 format limit)
  uint64_t max_entries;
};

struct LBDevice;  // device allocations of one light's buffer (rt_lightbuf.hip)

// Build one light's buffer on the stream (synchronous at the end: the entry
// count sizes the sort).  *out is filled with device pointers owned by *dev.
extern "C" int rt_lightbuf_build(const LBParams* p, RtLightBuf* out, LBDevice** dev, hipStream_t s,
                                 char* err, size_t errlen);
extern "C" void rt_lightbuf_free(LBDevice* dev);
// entries and cells of a built buffer (bench / info)
extern "C" void rt_lightbuf_sizes(const LBDevice* dev, unsigned long long* entries,
                                  unsigned long long* cells, unsigned long long* global);
// The same footprints counted on the host (in->tri = host prim-order
// records), every stride-th prim: out[0] entries, [1] never accepted, [2]
// global, [3] band prims, [4] big prims, [5] prims surveyed, [6] band-row
// entries, [7] largest per-prim count, [8] its prim.
extern "C" int rt_lightbuf_survey_host(const LBParams* in, uint32_t stride, unsigned long long out[12],
                                       char* err, size_t errlen);
// proven mode: triangles no ray of the light can make the float test accept
// (skipped), and triangles listed along a band of the cube map (point lights)
extern "C" void rt_lightbuf_proof_counts(const LBDevice* dev, unsigned long long* never,
                                         unsigned long long* band);
