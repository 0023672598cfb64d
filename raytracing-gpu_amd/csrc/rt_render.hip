// rt_render.hip -- the MI355X (gfx950) render kernels.
//
// One lane renders one pixel: the 4 supersamples of cpu/raytracer.c:55-69 in
// the reference order, each a path of closest-hit queries (cpu/raytracer.c:19-34)
// with Phong + shadow-ray shading at every hit (cpu/light.c:33-100).  A wave
// owns an 8x8 pixel tile; waves are persistent and pull tiles from an atomic
// counter, so the irregular per-tile cost balances across the 256 CUs.
//
// Bit-parity with cpu/rt:
//   * -ffp-contract=off, IEEE div/sqrt, f64 sqrt/pow where the reference uses them;
//   * closest hit = lexicographic min of (new_dist, prim) over hits with
//     new_dist > 0.01 (prim = object-major, LIFO-triangle index);
//   * shadow = any hit with new_dist > 0.01 (early exit is exact);
//   * reflection terms are buffered and summed deepest-first.
//
// Acceleration: FLAT tests every triangle record (the reference's brute
// force, cpu/hit.c:72-109) with wave-uniform scalar loads of each record;
// OCTREE walks the octree built by host/accel.c with a per-lane stack,
// front-to-back child order and conservative distance culling.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_cull.h"
#include "rt_device.h"
#include "rt_kernels.h"

namespace rt {

static constexpr float kEps = 0.0000001f;  // cpu/hit.c:7 (float)1e-7
static constexpr int kMaxDepth = RT_MAX_DEPTH;

__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }

// Moller-Trumbore, cpu/hit.c:15-33 with e1/e2 precomputed (same bits).
__device__ __forceinline__ bool mt_test(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float& t, float& u,
                                        float& v) {
  f3 h = cross(d, e2);
  float a = dot(e1, h);
  if (a > -kEps && a < kEps) return false;
  float f = 1.0f / a;
  f3 s = sub(o, v0);
  u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return false;
  f3 q = cross(s, e1);
  v = f * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  t = f * dot(e2, q);
  return t > kEps;
}

struct Ray {
  f3 o, d;     // origin, direction (as the reference holds them)
  f3 nd;       // normalize(d)
  float dlen;  // length(d)
  float eps;   // culling slack (world units) for this origin
  f3 oh, ol;   // o + eps, o - eps: the grown slab planes' offsets (rt_cull.h)
};

__device__ __forceinline__ Ray make_ray(const KParams& p, f3 o, f3 d) {
  Ray r;
  r.o = o;
  r.d = d;
  r.dlen = length(d);
  r.nd = f3{d.x / r.dlen, d.y / r.dlen, d.z / r.dlen};
  r.eps = rt_cull_eps(p.eps_rel, o.x - p.scene_c.x, o.y - p.scene_c.y, o.z - p.scene_c.z,
                      p.scene_cmag, p.scene_r);
  r.oh = f3{o.x + r.eps, o.y + r.eps, o.z + r.eps};
  r.ol = f3{o.x - r.eps, o.y - r.eps, o.z - r.eps};
  return r;
}

// new_dist = |(o + nd * (t*|d|)) - o| (cpu/hit.c:35-37,58); returns the hit point too.
__device__ __forceinline__ float hit_dist(const Ray& r, float t, f3& out) {
  out = add(r.o, scale(r.nd, t * r.dlen));
  return length(sub(out, r.o));
}

// Conservative pre-filter of the Moller-Trumbore test.  h, a, s.h, d.q, e2.q
// are the reference's own float values (same operations); only the IEEE
// division f = 1/a is replaced by v_rcp_f32 (1 ulp).  A triangle is dropped
// only when the reference's u, v, t (which differ from these by a few ulps)
// are certain to fail cpu/hit.c:20-33, or when its distance certainly exceeds
// t_cut (closest hit: it cannot beat the current winner, ties included);
// survivors are re-tested exactly.  DESIGN.md "Exact MT with a cheap reject".
__device__ __forceinline__ bool mt_candidate(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float t_cut) {
#ifdef RT_EXACT_ONLY
  return true;
#else
  // same staging as cpu/hit.c:15-33, so a wave whose lanes all fail u skips
  // the v and t work (coherent packets mostly agree)
  const float m = 1e-5f;  // >> the few-ulp gap between (u,v,t) and the reference's
  f3 h = cross(d, e2);
  float a = dot(e1, h);
  if (a > -kEps && a < kEps) return false;  // identical test, identical a
  float r = __builtin_amdgcn_rcpf(a);
  f3 s = sub(o, v0);
  float u = dot(s, h) * r;
  if (u < -1e-30f || u > 1.0f + m) return false;
  f3 q = cross(s, e1);
  float v = dot(d, q) * r;
  if (v < -1e-30f || u + v > 1.0f + m) return false;
  float t = dot(e2, q) * r;
  return !(t < kEps * (1.0f - m) || t > t_cut);
#endif
}

#ifndef RT_BEST_T
#define RT_BEST_T 0  // measured: C5 15.40/15.53 (on) vs 15.63/15.36 ms (off), C3 no better
#endif

struct Best {
  float dist;  // +inf = none
  float t_cut; // parametric bound beyond which no triangle can win (+inf = none)
  uint32_t prim, obj;
  float u, v;
#if RT_BEST_T
  float t;  // MT t of the winner; the hit point is recomputed from it (hit_pt)
#else
  f3 pt;
#endif
};

__device__ __forceinline__ void consider(const Ray& r, const float4& q0, const float4& q1,
                                         const float4& q2, Best& b) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  if (!mt_candidate(r.o, r.d, v0, e1, e2, b.t_cut)) return;
  float t, u, v;
  if (!mt_test(r.o, r.d, v0, e1, e2, t, u, v)) return;
  f3 out;
  float nd = hit_dist(r, t, out);
  if (!((double)nd > 0.01)) return;
  uint32_t prim = __float_as_uint(q2.y);
  if (nd < b.dist || (nd == b.dist && prim < b.prim)) {
    b.dist = nd;
    // a rival's new_dist is |(o + nd*(t*|d|)) - o|: t*|d| up to a few ulps of
    // |t*|d||, plus the rounding of the hit point (ulps of |o|+dist)
    float ao = fmaxf(fabsf(r.o.x), fmaxf(fabsf(r.o.y), fabsf(r.o.z)));
    b.t_cut = (nd * (1.0f + 1e-5f) + (ao + nd) * 2e-6f) / r.dlen;
    b.prim = prim;
    b.obj = __float_as_uint(q2.z);
    b.u = u;
    b.v = v;
#if RT_BEST_T
    b.t = t;
#else
    b.pt = out;
#endif
  }
}

#ifndef RT_ANY_DLEN_RECOMPUTE
#define RT_ANY_DLEN_RECOMPUTE 1  // measured: C5 15.43/15.39 (on) vs 15.66/15.39 ms (off)
#endif
#ifndef RT_ANY_ND_RECOMPUTE
#define RT_ANY_ND_RECOMPUTE 1  // measured: C5 15.37/15.39 (on) vs 15.53/15.50 ms (off)
#endif

__device__ __forceinline__ bool any_hit_rec(const Ray& r, const float4& q0, const float4& q1,
                                            const float4& q2) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  if (!mt_candidate(r.o, r.d, v0, e1, e2, __builtin_inff())) return false;
  float t, u, v;
  if (!mt_test(r.o, r.d, v0, e1, e2, t, u, v)) return false;
#if RT_ANY_ND_RECOMPUTE
  // normalize(d) recomputed here (same IEEE divisions as make_ray, same
  // bits) instead of keeping it live through the whole any-hit walk
#if RT_ANY_DLEN_RECOMPUTE
  float dlen = length(r.d);  // = make_ray's r.dlen, same operations
#else
  float dlen = r.dlen;
#endif
  f3 nd{r.d.x / dlen, r.d.y / dlen, r.d.z / dlen};
  f3 out = add(r.o, scale(nd, t * dlen));
  return (double)length(sub(out, r.o)) > 0.01;
#else
  f3 out;
  return (double)hit_dist(r, t, out) > 0.01;
#endif
}

// -------------------------------------------------------------- OCTREE
// Per-lane traversal stack: the first kLdsStack entries live in LDS, laid
// out [entry][lane] so every lane hits its own bank; deeper entries spill to
// a per-lane area in global memory (rare: typical depth is < 16).
#ifndef RT_LDS_STACK
#define RT_LDS_STACK 6
#endif
static constexpr int kLdsStack = RT_LDS_STACK;
static constexpr int kSpillStack = RT_SPILL_STACK;

struct Stack {
  uint32_t* idx;  // LDS, kLdsStack x 64
  float* tt;      // LDS, kLdsStack x 64
  uint2* spill;   // this lane's kSpillStack entries
  int lane;
  int sp;
  uint32_t occ;   // record index of this lane's last shadow occluder (~0u: none)
  uint32_t occ2;  // the same for the other light parity (RT_OCC_SLOTS 2)
  uint32_t slot;  // light parity of the current shadow query (wave-uniform)
};

// Counters of one lane's own walk (divergent code); folded into the wave's
// WorkCount after the walk (absorb).
struct LaneCount {
  uint32_t nodes, tris, overflow;
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return __builtin_amdgcn_readfirstlane(x);
}

// Number of distinct keys among the lanes executing this call (divergent
// code: the lanes of the current loop iteration), added once to lane `first`.
// Algorithmic-byte accounting of the per-lane walks (COUNT pass only): a
// record that several lanes load with the same instruction counts once, the
// same rule as the packet walk's wave-uniform fetches.
__device__ __forceinline__ uint32_t lanes_distinct(uint32_t key) {
  uint64_t m = __ballot(1);
  uint32_t n = 0;
  int me = __lane_id();
  bool first = (int)(__ffsll((unsigned long long)m) - 1) == me;
  while (m) {
    int l = __ffsll((unsigned long long)m) - 1;
    uint32_t k = __shfl(key, l);
    m &= ~__ballot(key == k);
    n++;
  }
  return first ? n : 0u;
}

template <bool COUNT>
__device__ __forceinline__ void absorb(WorkCount& wc, const LaneCount& lc) {
  if (COUNT) {
    wc.nodes += wave_sum(lc.nodes);
    wc.tris += wave_sum(lc.tris);
  }
  wc.overflow += wave_sum(lc.overflow);
}

__device__ __forceinline__ void push(Stack& s, uint32_t i, float t, LaneCount& wc) {
  if (s.sp < kLdsStack) {
    s.idx[s.sp * 64 + s.lane] = i;
    s.tt[s.sp * 64 + s.lane] = t;
  } else if (s.sp < kLdsStack + kSpillStack) {
    s.spill[s.sp - kLdsStack] = make_uint2(i, __float_as_uint(t));
  } else {
    wc.overflow++;  // reported as RT_EDEPTH by rt_hip_stats: never silent
    return;
  }
  s.sp++;
}

__device__ __forceinline__ void pop(Stack& s, uint32_t& i, float& t) {
  --s.sp;
  if (s.sp < kLdsStack) {
    i = s.idx[s.sp * 64 + s.lane];
    t = s.tt[s.sp * 64 + s.lane];
  } else {
    uint2 e = s.spill[s.sp - kLdsStack];
    i = e.x;
    t = __uint_as_float(e.y);
  }
}

__device__ __forceinline__ f3 inv_dir(f3 d) { return f3{rt_inv(d.x), rt_inv(d.y), rt_inv(d.z)}; }

// entry parameter of the eps-grown box, +inf on a miss (rt_cull.h)
__device__ __forceinline__ float box_enter(const Ray& r, f3 inv, float4 lo, float4 hi) {
  float t;
  bool hit = rt_box_hit(r.oh.x, r.oh.y, r.oh.z, r.ol.x, r.ol.y, r.ol.z, inv.x, inv.y, inv.z, lo.x,
                        lo.y, lo.z, hi.x, hi.y, hi.z, &t);
  return hit ? t : __builtin_inff();
}

__device__ __forceinline__ bool rt_prune(float t_enter, float dlen, float best, float eps) {
  return t_enter * dlen > rt_prune_limit(best, eps);
}

// octant nearest to the origin side (rt_cull.h: bit a = upper half of axis a)
__device__ __forceinline__ uint32_t near_octant(f3 d) {
  return (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
}

#ifndef RT_CHILD_PIPE
#define RT_CHILD_PIPE 1
#endif

// child-mask bit o moved to bit o ^ dm (the visiting order's index space)
__device__ __forceinline__ uint32_t mask_xor(uint32_t m, uint32_t dm) {
  if (dm & 1u) m = ((m & 0x55u) << 1) | ((m & 0xAAu) >> 1);
  if (dm & 2u) m = ((m & 0x33u) << 2) | ((m & 0xCCu) >> 2);
  if (dm & 4u) m = ((m & 0x0Fu) << 4) | ((m & 0xF0u) >> 4);
  return m;
}

// Interior node: test the children's boxes and push the hits far-to-near in
// octant order (a valid front-to-back order for the disjoint octant cells),
// so the nearest child is popped first.  CLOSEST also prunes by best.
template <bool CLOSEST, bool COUNT>
__device__ __forceinline__ void push_children(const float4* __restrict__ node, const Ray& r, f3 inv,
                                              uint32_t dm, uint32_t first, uint32_t info,
                                              float best, Stack& s, LaneCount& wc) {
  uint32_t mask = RT_NODE_MASK(info);
#if RT_CHILD_PIPE
  // same order, software-pipelined: child k+1's box is in flight while
  // child k is tested
  uint32_t mj = mask_xor(mask, dm);
  if (!mj) return;
  int j = 31 - __clz(mj);
  mj &= ~(1u << j);
  uint32_t ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
  float4 nlo = node[2 * ci], nhi = node[2 * ci + 1];
  if (COUNT) wc.nodes += lanes_distinct(ci);
  for (;;) {
    float4 clo = nlo, chi = nhi;
    uint32_t cc = ci;
    bool more = mj != 0u;
    if (more) {
      j = 31 - __clz(mj);
      mj &= ~(1u << j);
      ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
      nlo = node[2 * ci];
      nhi = node[2 * ci + 1];
      if (COUNT) wc.nodes += lanes_distinct(ci);
    }
    float t0 = box_enter(r, inv, clo, chi);
    if (t0 != __builtin_inff() &&
        !(CLOSEST && best != __builtin_inff() && rt_prune(t0, r.dlen, best, r.eps)))
      push(s, cc, t0, wc);
    if (!more) break;
  }
  return;
#endif
#pragma unroll 1
  for (int j = 7; j >= 0; --j) {
    uint32_t o = (uint32_t)j ^ dm;
    if (mask & (1u << o)) {
      uint32_t ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
      if (COUNT) wc.nodes += lanes_distinct(ci);
      float t0 = box_enter(r, inv, node[2 * ci], node[2 * ci + 1]);
      if (t0 == __builtin_inff()) continue;
      if (CLOSEST && best != __builtin_inff() && rt_prune(t0, r.dlen, best, r.eps)) continue;
      push(s, ci, t0, wc);
    }
  }
}

#ifndef RT_LEAF_PIPE
#define RT_LEAF_PIPE 1
#endif

template <bool COUNT>
__device__ void oct_closest(const KParams& p, const Ray& r, Best& b, Stack& s, LaneCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  f3 inv = inv_dir(r.d);
  uint32_t dm = near_octant(r.d);
  s.sp = 0;
  {
    float t0 = box_enter(r, inv, node[0], node[1]);
    if (t0 != __builtin_inff()) push(s, 0, t0, wc);
  }
  while (s.sp > 0) {
    uint32_t ni;
    float tn;
    pop(s, ni, tn);
    if (b.dist != __builtin_inff() && rt_prune(tn, r.dlen, b.dist, r.eps)) continue;
    float4 lo = node[2 * ni], hi = node[2 * ni + 1];
    uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
    if (COUNT) wc.nodes += lanes_distinct(ni);
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
#if RT_LEAF_PIPE
      // software-pipelined: record k+1 is in flight while record k is tested
      const float4* q = tri + 3 * (size_t)first;
      float4 n0 = q[0], n1 = q[1], n2 = q[2];
      for (uint32_t k = 0; k < cnt; k++) {
        float4 q0 = n0, q1 = n1, q2 = n2;
        if (k + 1 < cnt) {
          n0 = q[3 * (k + 1)];
          n1 = q[3 * (k + 1) + 1];
          n2 = q[3 * (k + 1) + 2];
        }
        if (COUNT) wc.tris += lanes_distinct(first + k);
        consider(r, q0, q1, q2, b);
      }
#else
      for (uint32_t k = 0; k < cnt; k++) {
        const float4* q = tri + 3 * (size_t)(first + k);
        if (COUNT) wc.tris += lanes_distinct(first + k);
        consider(r, q[0], q[1], q[2], b);
      }
#endif
    } else {
      push_children<true, COUNT>(node, r, inv, dm, first, info, b.dist, s, wc);
    }
  }
}

// Any-hit walk: a stack entry holds the node's own (first, info) words,
// taken from the child box record its parent already fetched, so a pop needs
// no node fetch -- one dependent load per step (the children's boxes or the
// leaf's triangles) instead of two.
#ifndef RT_PREFETCH
#define RT_PREFETCH 0  // measured: C5 16.8 (on) vs 15.5-15.7 ms (off); VGPR spills 40 -> 50
#endif

// first child (in visiting order) of an interior node, for the prefetch
__device__ __forceinline__ uint32_t first_child(uint32_t first, uint32_t info, uint32_t dm) {
  uint32_t mask = RT_NODE_MASK(info);
  uint32_t mj = mask_xor(mask, dm);
  int j = 31 - __clz(mj | 1u);
  return first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
}

// push_children_any with the first child's box already loaded (plo, phi);
// returns true when it pushed, with the last pushed entry (the new stack
// top) in (tf, ti).
template <bool COUNT>
__device__ __forceinline__ bool push_children_any_pf(const float4* __restrict__ node, const Ray& r,
                                                     f3 inv, uint32_t dm, uint32_t first,
                                                     uint32_t info, float4 plo, float4 phi,
                                                     Stack& s, LaneCount& wc, uint32_t& tf,
                                                     uint32_t& ti) {
  uint32_t mask = RT_NODE_MASK(info);
  uint32_t mj = mask_xor(mask, dm);
  if (!mj) return false;
  int j = 31 - __clz(mj);
  mj &= ~(1u << j);
  uint32_t ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
  float4 nlo = plo, nhi = phi;
  if (COUNT) wc.nodes += lanes_distinct(ci);
  int sp0 = s.sp;
  for (;;) {
    float4 clo = nlo, chi = nhi;
    bool more = mj != 0u;
    if (more) {
      j = 31 - __clz(mj);
      mj &= ~(1u << j);
      ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
      nlo = node[2 * ci];
      nhi = node[2 * ci + 1];
      if (COUNT) wc.nodes += lanes_distinct(ci);
    }
    if (box_enter(r, inv, clo, chi) != __builtin_inff()) {
      int sp1 = s.sp;
      push(s, __float_as_uint(clo.w), chi.w, wc);
      if (s.sp != sp1) {
        tf = __float_as_uint(clo.w);
        ti = __float_as_uint(chi.w);
      }
    }
    if (!more) break;
  }
  return s.sp != sp0;
}

template <bool COUNT>
__device__ __forceinline__ void push_children_any(const float4* __restrict__ node, const Ray& r,
                                                  f3 inv, uint32_t dm, uint32_t first,
                                                  uint32_t info, Stack& s, LaneCount& wc) {
  uint32_t mask = RT_NODE_MASK(info);
#if RT_CHILD_PIPE
  // Same far-to-near order as below (j = 7..0, octant j ^ dm), software-
  // pipelined: child k+1's box is in flight while child k is tested.
  uint32_t mj = mask_xor(mask, dm);
  if (!mj) return;
  int j = 31 - __clz(mj);
  mj &= ~(1u << j);
  uint32_t o = (uint32_t)j ^ dm;
  uint32_t ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
  float4 nlo = node[2 * ci], nhi = node[2 * ci + 1];
  if (COUNT) wc.nodes += lanes_distinct(ci);
  for (;;) {
    float4 clo = nlo, chi = nhi;
    bool more = mj != 0u;
    if (more) {
      j = 31 - __clz(mj);
      mj &= ~(1u << j);
      o = (uint32_t)j ^ dm;
      ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
      nlo = node[2 * ci];
      nhi = node[2 * ci + 1];
      if (COUNT) wc.nodes += lanes_distinct(ci);
    }
    if (box_enter(r, inv, clo, chi) != __builtin_inff()) push(s, __float_as_uint(clo.w), chi.w, wc);
    if (!more) break;
  }
  return;
#endif
#pragma unroll 1
  for (int j = 7; j >= 0; --j) {
    uint32_t o = (uint32_t)j ^ dm;
    if (mask & (1u << o)) {
      uint32_t ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
      if (COUNT) wc.nodes += lanes_distinct(ci);
      float4 clo = node[2 * ci], chi = node[2 * ci + 1];
      if (box_enter(r, inv, clo, chi) == __builtin_inff()) continue;
      push(s, __float_as_uint(clo.w), chi.w, wc);
    }
  }
}

#ifndef RT_OCC_CACHE
#define RT_OCC_CACHE 0  // measured: C5 15.37/15.56 (on) vs 15.33/15.53 ms (off): a wave waits for its slowest lane
#endif
#ifndef RT_OCC_SLOTS
#define RT_OCC_SLOTS 2  // one cached occluder per light parity
#endif
#ifndef RT_WHILE_WHILE
#define RT_WHILE_WHILE 0  // measured: C5 15.89/16.00 (on) vs 15.46/15.57 ms (off)
#endif

template <bool COUNT>
__device__ bool oct_any(const KParams& p, const Ray& r, Stack& s, LaneCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  f3 inv = inv_dir(r.d);
  uint32_t dm = near_octant(r.d);
  s.sp = 0;
#if RT_OCC_CACHE
  // Occluder cache: the triangle that blocked this lane's previous shadow ray
  // (a neighbouring supersample's, usually) is tested first.  Any record hit
  // with the walk's own exact test decides the query (cpu/light.c:24-31 is an
  // any-hit predicate), so this only reorders work.
  uint32_t oc = (RT_OCC_SLOTS == 2 && s.slot) ? s.occ2 : s.occ;
  if (oc != 0xffffffffu) {
    const float4* q = tri + 3 * (size_t)oc;
    if (COUNT) wc.tris += lanes_distinct(oc);
    if (any_hit_rec(r, q[0], q[1], q[2])) return true;
  }
#endif
  {
    float4 lo = node[0], hi = node[1];
    if (COUNT) wc.nodes += lanes_distinct(0);
    if (box_enter(r, inv, lo, hi) != __builtin_inff()) push(s, __float_as_uint(lo.w), hi.w, wc);
  }
#if RT_PREFETCH && !RT_WHILE_WHILE
  // Prefetch: when a node's children were pushed, the new stack top is known
  // (the nearest child) and its first payload -- its first child's box, or
  // its first triangle record -- is loaded at once, so the next iteration's
  // pop does not start with a dependent load.  Same visiting order and
  // results as the loop below; only the load issue moves earlier.
  {
    bool pf = false;
    float4 p0, p1, p2;
    while (s.sp > 0) {
      uint32_t first;
      float info_bits;
      pop(s, first, info_bits);
      uint32_t info = __float_as_uint(info_bits);
      bool have = pf;
      pf = false;
      if (info & RT_NODE_LEAF) {
        uint32_t cnt = RT_LEAF_COUNT(info);
        const float4* q = tri + 3 * (size_t)first;
        if (!have) {
          p0 = q[0];
          p1 = q[1];
          p2 = q[2];
        }
        float4 n0 = p0, n1 = p1, n2 = p2;
        for (uint32_t k = 0; k < cnt; k++) {
          float4 q0 = n0, q1 = n1, q2 = n2;
          if (k + 1 < cnt) {
            n0 = q[3 * (k + 1)];
            n1 = q[3 * (k + 1) + 1];
            n2 = q[3 * (k + 1) + 2];
          }
          if (COUNT) wc.tris += lanes_distinct(first + k);
          if (any_hit_rec(r, q0, q1, q2)) {
            s.sp = 0;
            return true;
          }
        }
      } else {
        if (!have) {
          uint32_t c0 = first_child(first, info, dm);
          p0 = node[2 * c0];
          p1 = node[2 * c0 + 1];
        }
        uint32_t tf = 0, ti = 0;
        if (push_children_any_pf<COUNT>(node, r, inv, dm, first, info, p0, p1, s, wc, tf, ti)) {
          pf = true;
          if (ti & RT_NODE_LEAF) {
            const float4* q = tri + 3 * (size_t)tf;
            p0 = q[0];
            p1 = q[1];
            p2 = q[2];
          } else {
            uint32_t c0 = first_child(tf, ti, dm);
            p0 = node[2 * c0];
            p1 = node[2 * c0 + 1];
          }
        }
      }
    }
    return false;
  }
#endif
#if RT_WHILE_WHILE
  // "while-while" order (Aila & Laine 2009): each lane descends interior
  // nodes until it holds a leaf (or its stack is empty); the leaf tests then
  // run with every lane that found one active at once, instead of the leaf
  // loop and the child loop alternating as divergent branches.
  for (;;) {
    uint32_t lf = 0, lcnt = 0;
    bool have = false;
    while (!have && s.sp > 0) {
      uint32_t first;
      float info_bits;
      pop(s, first, info_bits);
      uint32_t info = __float_as_uint(info_bits);
      if (info & RT_NODE_LEAF) {
        have = true;
        lf = first;
        lcnt = RT_LEAF_COUNT(info);
      } else {
        push_children_any<COUNT>(node, r, inv, dm, first, info, s, wc);
      }
    }
    if (!have) return false;
    const float4* q = tri + 3 * (size_t)lf;
    float4 n0 = q[0], n1 = q[1], n2 = q[2];
    for (uint32_t k = 0; k < lcnt; k++) {
      float4 q0 = n0, q1 = n1, q2 = n2;
      if (k + 1 < lcnt) {
        n0 = q[3 * (k + 1)];
        n1 = q[3 * (k + 1) + 1];
        n2 = q[3 * (k + 1) + 2];
      }
      if (COUNT) wc.tris += lanes_distinct(lf + k);
      if (any_hit_rec(r, q0, q1, q2)) {
        s.sp = 0;
        return true;
      }
    }
  }
#endif
  while (s.sp > 0) {
    uint32_t first;
    float info_bits;
    pop(s, first, info_bits);
    uint32_t info = __float_as_uint(info_bits);
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
#if RT_LEAF_PIPE
      // software-pipelined: record k+1 is in flight while record k is tested
      const float4* q = tri + 3 * (size_t)first;
      float4 n0 = q[0], n1 = q[1], n2 = q[2];
      for (uint32_t k = 0; k < cnt; k++) {
        float4 q0 = n0, q1 = n1, q2 = n2;
        if (k + 1 < cnt) {
          n0 = q[3 * (k + 1)];
          n1 = q[3 * (k + 1) + 1];
          n2 = q[3 * (k + 1) + 2];
        }
        if (COUNT) wc.tris += lanes_distinct(first + k);
        if (any_hit_rec(r, q0, q1, q2)) {
          s.sp = 0;
          if (RT_OCC_SLOTS == 2 && s.slot)
            s.occ2 = first + k;
          else
            s.occ = first + k;
          return true;
        }
      }
#else
      for (uint32_t k = 0; k < cnt; k++) {
        const float4* q = tri + 3 * (size_t)(first + k);
        if (COUNT) wc.tris += lanes_distinct(first + k);
        if (any_hit_rec(r, q[0], q[1], q[2])) {
          s.sp = 0;
          return true;
        }
      }
#endif
    } else {
      push_children_any<COUNT>(node, r, inv, dm, first, info, s, wc);
    }
  }
  return false;
}

// ------------------------------------------------------ PACKET (wave) walk
// The 64 lanes of a wave walk the octree together: one wave-uniform stack of
// node indices in LDS, node and triangle records fetched once per wave with
// wave-uniform addresses (broadcast to every lane), each lane testing its own
// ray, and __ballot deciding which children any lane still needs.  Camera
// rays of an 8x8 tile and shadow rays toward one light are coherent, so the
// union of the lanes' walks is barely larger than each one's.
static constexpr int kWaveStack = 192;

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float4 uni4(float4 v) {
  return make_float4(__uint_as_float(uni(__float_as_uint(v.x))),
                     __uint_as_float(uni(__float_as_uint(v.y))),
                     __uint_as_float(uni(__float_as_uint(v.z))),
                     __uint_as_float(uni(__float_as_uint(v.w))));
}
// Wave-uniform loads through the constant address space: with a uniform
// address they become scalar (SMEM) loads straight into SGPRs.  The scene
// image is read-only for the whole launch.
__device__ __forceinline__ float4 ldu(const float4* p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) float4 cfloat4;
  return ((cfloat4*)p)[i];
#else
  return p[i];  // host pass only parses device code
#endif
}
__device__ __forceinline__ void node_u(const float4* __restrict__ node, uint32_t ni, float4& lo,
                                       float4& hi) {
  lo = ldu(node, 2 * (size_t)ni);
  hi = ldu(node, 2 * (size_t)ni + 1);
}

// majority ray-direction octant of the active lanes (child push order)
__device__ __forceinline__ uint32_t wave_near_octant(bool act, f3 d, uint64_t am) {
  int na = __popcll(am);
  uint32_t dm = 0;
  if (2 * __popcll(__ballot(act && d.x < 0.0f)) > na) dm |= 1u;
  if (2 * __popcll(__ballot(act && d.y < 0.0f)) > na) dm |= 2u;
  if (2 * __popcll(__ballot(act && d.z < 0.0f)) > na) dm |= 4u;
  return dm;
}

// Must be called by all 64 lanes (converged); act = this lane has a query.
template <bool COUNT>
__device__ void packet_closest(const KParams& p, const Ray& r, bool act, Best& b, uint32_t* ws,
                               int lane, WorkCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  uint64_t am = __ballot(act);
  if (am == 0) return;
  f3 inv = inv_dir(r.d);
  uint32_t dm = wave_near_octant(act, r.d, am);
  int sp = 0;
  ws[sp++] = 0;
  while (sp > 0) {
    uint32_t ni = uni(ws[--sp]);
    float4 lo, hi;
    node_u(node, ni, lo, hi);
    float tn = box_enter(r, inv, lo, hi);
    bool want = act && tn != __builtin_inff() &&
                !(b.dist != __builtin_inff() && rt_prune(tn, r.dlen, b.dist, r.eps));
    if (__ballot(want) == 0) continue;
    uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
    if (COUNT) wc.nodes++;
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
      for (uint32_t k = 0; k < cnt; k++) {
        const float4* q = tri + 3 * (size_t)(first + k);
        float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
        if (want) consider(r, q0, q1, q2, b);
      }
      if (COUNT) wc.tris += cnt;
    } else {
      uint32_t mask = RT_NODE_MASK(info);
      for (int j = 7; j >= 0; --j) {
        uint32_t o = (uint32_t)j ^ dm;
        if (!(mask & (1u << o))) continue;
        uint32_t ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
        float4 clo, chi;
        node_u(node, ci, clo, chi);
        float t0 = box_enter(r, inv, clo, chi);
        bool w2 = want && t0 != __builtin_inff() &&
                  !(b.dist != __builtin_inff() && rt_prune(t0, r.dlen, b.dist, r.eps));
        if (__ballot(w2) != 0) {
          if (sp < kWaveStack)
            ws[sp++] = ci;
          else
            wc.overflow++;  // RT_EDEPTH, never silent
        }
      }
    }
  }
}

template <bool COUNT>
__device__ bool packet_any(const KParams& p, const Ray& r, bool act, uint32_t* ws, int lane,
                           WorkCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  bool alive = act, hit = false;
  uint64_t am = __ballot(alive);
  if (am == 0) return false;
  f3 inv = inv_dir(r.d);
  uint32_t dm = wave_near_octant(act, r.d, am);
  int sp = 0;
  ws[sp++] = 0;
  while (sp > 0) {
    uint32_t ni = uni(ws[--sp]);
    float4 lo, hi;
    node_u(node, ni, lo, hi);
    bool want = alive && box_enter(r, inv, lo, hi) != __builtin_inff();
    if (__ballot(want) == 0) continue;
    uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
    if (COUNT) wc.nodes++;
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
      for (uint32_t k = 0; k < cnt; k++) {
        const float4* q = tri + 3 * (size_t)(first + k);
        float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
        if (COUNT) wc.tris++;
        if (want && any_hit_rec(r, q0, q1, q2)) {
          hit = true;
          alive = false;
          want = false;
        }
        if (__ballot(want) == 0) break;
      }
      if (__ballot(alive) == 0) break;
    } else {
      uint32_t mask = RT_NODE_MASK(info);
      for (int j = 7; j >= 0; --j) {
        uint32_t o = (uint32_t)j ^ dm;
        if (!(mask & (1u << o))) continue;
        uint32_t ci = first + (uint32_t)__popc(mask & ((1u << o) - 1u));
        float4 clo, chi;
        node_u(node, ci, clo, chi);
        bool w2 = want && box_enter(r, inv, clo, chi) != __builtin_inff();
        if (__ballot(w2) != 0) {
          if (sp < kWaveStack)
            ws[sp++] = ci;
          else
            wc.overflow++;
        }
      }
    }
  }
  return hit;
}

// ------------------------------------------- PACKET walk, LDS-staged records
// Same wave walk, but every fetch is one coalesced vector load by the lanes
// (lane k loads float4 k of the records) staged in LDS, then read back as
// broadcasts: a leaf's triangle records (3 float4 each, 21 per chunk) or an
// interior node's child boxes (2 float4 each, <= 8 children, contiguous) cost
// one memory round trip instead of one per record.  The wave stack holds the
// pushed child's whole node record (box + first/info), so a pop needs no
// memory access before the next fetch is issued.
// float4 staging slots per wave: FLAT streams 64 triangle records at a time;
// the octree walk stages one node's payload (<= 8 children, or a leaf's
// records, RT_OCT_LEAF_CAP = 32 of them in one chunk).  LDS per one-wave
// workgroup must stay <= 10 KB for 16 workgroups per CU.
static constexpr int kStageFlat = 192;
#ifndef RT_STAGE_OCT
#define RT_STAGE_OCT 96
#endif
static constexpr int kStageOct = RT_STAGE_OCT;
#ifndef RT_STACK2
#define RT_STACK2 96
#endif
static constexpr int kStack2 = RT_STACK2;  // wave stack entries (2 float4 each)

struct WaveCtx {
  uint32_t* ws;    // kWaveStack node indices (packet walk)
  float4* stk2;    // kStack2 x 2 float4 (staged packet walk)
  uint64_t* stkm;  // kStack2 lane masks: lanes that wanted the pushed node
  float4* stage;   // kStageFlat / kStageOct float4
  int lane;
};

// A fetch in flight: the wave's lanes hold float4 k, k+64, k+128 of src[0, n)
// in registers (issued early so its latency overlaps other work), then commit
// it to the LDS stage; n <= kStageFlat.
struct Fetch {
  float4 v0, v1, v2;
  int n;
};

__device__ __forceinline__ Fetch fetch_issue(const float4* __restrict__ src, int n, int l) {
  Fetch f;
  f.n = n;
  if (l < n) f.v0 = src[l];
  if (l + 64 < n) f.v1 = src[l + 64];
  if (l + 128 < n) f.v2 = src[l + 128];
  return f;
}

// The workgroup is one wave and a wave's LDS instructions execute in issue
// order, so staging needs no s_barrier: only a compiler barrier that keeps
// the LDS reads and writes in source order.
__device__ __forceinline__ void wave_sync() { __asm__ volatile("" ::: "memory"); }

__device__ __forceinline__ void fetch_commit(const Fetch& f, WaveCtx& w) {
  const int l = w.lane;
  wave_sync();  // after the previous readers of stage
  if (l < f.n) w.stage[l] = f.v0;
  if (l + 64 < f.n) w.stage[l + 64] = f.v1;
  if (l + 128 < f.n) w.stage[l + 128] = f.v2;
  wave_sync();
}

__device__ __forceinline__ void stage_load(const float4* __restrict__ src, int n, WaveCtx& w) {
  fetch_commit(fetch_issue(src, n, w.lane), w);
}

template <int RECS>
__device__ __forceinline__ uint32_t chunk(uint32_t n, uint32_t base) {
  return n - base < (uint32_t)RECS ? n - base : (uint32_t)RECS;
}
static constexpr int kFlatRecs = kStageFlat / 3;
static constexpr int kOctRecs = kStageOct / 3;

// Brute force over every triangle record (cpu/hit.c:72-109 order-free, the
// (new_dist, prim) key makes the winner order-independent), streamed through
// LDS 64 records at a time with the next chunk's fetch in flight while the
// current one is tested; converged calls.
template <bool COUNT>
__device__ void flat_closest_w(const KParams& p, const Ray& r, bool act, Best& b, WaveCtx& w,
                               WorkCount& wc) {
  if (__ballot(act) == 0) return;
  const uint32_t n = p.nrec;
  Fetch f = fetch_issue(p.tri, 3 * (int)chunk<kFlatRecs>(n, 0), w.lane);
  for (uint32_t base = 0; base < n; base += kFlatRecs) {
    uint32_t m = chunk<kFlatRecs>(n, base);
    fetch_commit(f, w);
    uint32_t nb = base + kFlatRecs;
    if (nb < n) f = fetch_issue(p.tri + 3 * (size_t)nb, 3 * (int)chunk<kFlatRecs>(n, nb), w.lane);
    // software-pipelined: record k+1's LDS reads are in flight while k is tested
    float4 n0 = w.stage[0], n1 = w.stage[1], n2 = w.stage[2];
    for (uint32_t k = 0; k < m; k++) {
      float4 q0 = n0, q1 = n1, q2 = n2;
      uint32_t kn = k + 1 < m ? 3 * (k + 1) : 0;
      n0 = w.stage[kn];
      n1 = w.stage[kn + 1];
      n2 = w.stage[kn + 2];
      if (act) consider(r, q0, q1, q2, b);
    }
  }
  if (COUNT) wc.tris += n;
}

template <bool COUNT>
__device__ bool flat_any_w(const KParams& p, const Ray& r, bool act, WaveCtx& w, WorkCount& wc) {
  bool alive = act, hit = false;
  const uint32_t n = p.nrec;
  if (__ballot(alive) == 0 || n == 0) return false;
  Fetch f = fetch_issue(p.tri, 3 * (int)chunk<kFlatRecs>(n, 0), w.lane);
  for (uint32_t base = 0; base < n; base += kFlatRecs) {
    uint32_t m = chunk<kFlatRecs>(n, base);
    fetch_commit(f, w);
    uint32_t nb = base + kFlatRecs;
    if (nb < n) f = fetch_issue(p.tri + 3 * (size_t)nb, 3 * (int)chunk<kFlatRecs>(n, nb), w.lane);
    if (COUNT) wc.tris += m;
    float4 n0 = w.stage[0], n1 = w.stage[1], n2 = w.stage[2];
    for (uint32_t k = 0; k < m; k++) {
      float4 q0 = n0, q1 = n1, q2 = n2;
      uint32_t kn = k + 1 < m ? 3 * (k + 1) : 0;
      n0 = w.stage[kn];
      n1 = w.stage[kn + 1];
      n2 = w.stage[kn + 2];
      if (alive && any_hit_rec(r, q0, q1, q2)) {
        hit = true;
        alive = false;
      }
      if (__ballot(alive) == 0) break;
    }
    if (__ballot(alive) == 0) break;
  }
  return hit;
}

// Interior node whose child boxes are staged: test them, push the ones any
// lane wants (with the mask of the lanes that want each) far-to-near in
// octant order, so the nearest child ends on top of the stack.
template <bool ANY>
__device__ __forceinline__ void stage_push_children(const Ray& r, f3 inv, uint32_t dm,
                                                    uint32_t info, bool want, float limit,
                                                    int& sp, WaveCtx& w, WorkCount& wc) {
  uint32_t mask = RT_NODE_MASK(info), cnt = RT_NODE_COUNT(info);
  uint64_t lanes[8];
  uint32_t hitmask = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) {
    lanes[c] = 0;
    if ((uint32_t)c < cnt) {
      float4 clo = w.stage[2 * c], chi = w.stage[2 * c + 1];
      float t0 = box_enter(r, inv, clo, chi);
      bool w2 = want && t0 != __builtin_inff() && (ANY || !(t0 * r.dlen > limit));
      lanes[c] = __ballot(w2);
      if (lanes[c] != 0) hitmask |= 1u << c;
    }
  }
  for (int j = 7; j >= 0; --j) {
    uint32_t o = (uint32_t)j ^ dm;
    if (!(mask & (1u << o))) continue;
    uint32_t c = (uint32_t)__popc(mask & ((1u << o) - 1u));
    if (!(hitmask & (1u << c))) continue;
    if (sp < kStack2) {
      if (w.lane < 2) w.stk2[2 * sp + w.lane] = w.stage[2 * c + w.lane];
      uint64_t lm = 0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if ((uint32_t)k == c) lm = lanes[k];
      if (w.lane == 0) w.stkm[sp] = lm;
      sp++;
    } else {
      wc.overflow++;  // RT_EDEPTH, never silent
    }
  }
}

#ifndef RT_STAGE_PIPE
#define RT_STAGE_PIPE 0  // measured: C5 15.34 (off) vs 15.65 ms (on)
#endif

template <bool COUNT>
__device__ void staged_closest(const KParams& p, const Ray& r, bool act, Best& b, WaveCtx& w,
                               WorkCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  uint64_t am = __ballot(act);
  if (am == 0) return;
  f3 inv = inv_dir(r.d);
  uint32_t dm = wave_near_octant(act, r.d, am);
  int sp = 0;
  wave_sync();
  if (w.lane < 2) w.stk2[w.lane] = node[w.lane];
  if (w.lane == 0) w.stkm[0] = am;
  sp = 1;
  float limit = rt_prune_limit(b.dist, r.eps);
  while (sp > 0) {
    --sp;
    wave_sync();
    float4 lo = w.stk2[2 * sp], hi = w.stk2[2 * sp + 1];
    uint64_t lm = w.stkm[sp];
    uint32_t first = uni(__float_as_uint(lo.w)), info = uni(__float_as_uint(hi.w));
    bool leaf = (info & RT_NODE_LEAF) != 0;
    uint32_t cnt = leaf ? RT_LEAF_COUNT(info) : RT_NODE_COUNT(info);
    // issue the node's payload fetch now; its latency overlaps the re-test
    Fetch f = leaf ? fetch_issue(tri + 3 * (size_t)first, 3 * (int)chunk<kOctRecs>(cnt, 0), w.lane)
                   : fetch_issue(node + 2 * (size_t)first, 2 * (int)cnt, w.lane);
    // lanes that wanted it when pushed, re-tested against their best so far
    bool want = ((lm >> w.lane) & 1) != 0;
    if (want && b.dist != __builtin_inff()) {
      float tn = box_enter(r, inv, lo, hi);
      want = !(tn * r.dlen > limit);
    }
    if (__ballot(want) == 0) continue;
    if (COUNT) wc.nodes++;
    fetch_commit(f, w);
    if (leaf) {
      for (uint32_t base = 0; base < cnt; base += kOctRecs) {
        uint32_t m = chunk<kOctRecs>(cnt, base);
        if (base) stage_load(tri + 3 * (size_t)(first + base), 3 * (int)m, w);
#if RT_STAGE_PIPE
        // software-pipelined: record k+1's LDS reads are in flight while k is tested
        float4 n0 = w.stage[0], n1 = w.stage[1], n2 = w.stage[2];
        for (uint32_t k = 0; k < m; k++) {
          float4 q0 = n0, q1 = n1, q2 = n2;
          uint32_t kn = k + 1 < m ? 3 * (k + 1) : 0;
          n0 = w.stage[kn];
          n1 = w.stage[kn + 1];
          n2 = w.stage[kn + 2];
          if (want) consider(r, q0, q1, q2, b);
        }
#else
        for (uint32_t k = 0; k < m; k++) {
          float4 q0 = w.stage[3 * k], q1 = w.stage[3 * k + 1], q2 = w.stage[3 * k + 2];
          if (want) consider(r, q0, q1, q2, b);
        }
#endif
      }
      limit = rt_prune_limit(b.dist, r.eps);
      if (COUNT) wc.tris += cnt;
    } else {
      stage_push_children<false>(r, inv, dm, info, want, limit, sp, w, wc);
    }
  }
}

template <bool COUNT>
__device__ bool staged_any(const KParams& p, const Ray& r, bool act, WaveCtx& w, WorkCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ tri = p.tri;
  bool alive = act, hit = false;
  uint64_t am = __ballot(alive);
  if (am == 0) return false;
  f3 inv = inv_dir(r.d);
  uint32_t dm = wave_near_octant(act, r.d, am);
  int sp = 0;
  wave_sync();
  if (w.lane < 2) w.stk2[w.lane] = node[w.lane];
  if (w.lane == 0) w.stkm[0] = am;
  sp = 1;
  while (sp > 0) {
    --sp;
    wave_sync();
    float4 lo = w.stk2[2 * sp], hi = w.stk2[2 * sp + 1];
    uint64_t lm = w.stkm[sp];
    uint32_t first = uni(__float_as_uint(lo.w)), info = uni(__float_as_uint(hi.w));
    // any-hit has no pruning: the lanes that wanted the node when it was
    // pushed and still search want it now (no re-test)
    bool want = alive && ((lm >> w.lane) & 1) != 0;
    if (__ballot(want) == 0) continue;
    if (COUNT) wc.nodes++;
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
      for (uint32_t base = 0; base < cnt && __ballot(want) != 0; base += kOctRecs) {
        uint32_t m = chunk<kOctRecs>(cnt, base);
        stage_load(tri + 3 * (size_t)(first + base), 3 * (int)m, w);
        if (COUNT) wc.tris += m;
        for (uint32_t k = 0; k < m; k++) {
          float4 q0 = w.stage[3 * k], q1 = w.stage[3 * k + 1], q2 = w.stage[3 * k + 2];
          if (want && any_hit_rec(r, q0, q1, q2)) {
            hit = true;
            alive = false;
            want = false;
          }
          if (__ballot(want) == 0) break;
        }
      }
      if (__ballot(alive) == 0) break;
    } else {
      stage_load(node + 2 * (size_t)first, 2 * (int)RT_NODE_COUNT(info), w);
      stage_push_children<true>(r, inv, dm, info, want, 0.0f, sp, w, wc);
    }
  }
  return hit;
}

// Traversal policy: per-lane walks (each lane its own stack) or a packet
// walk; with TRAV_HYBRID the packet walk is used while at least
// p.packet_min lanes of the wave have a query.
#ifndef RT_LEAN  // 1: only the staged-hybrid closest walk and the per-lane any-hit walk
#define RT_LEAN 0
#endif
#define RT_TRAV_LANE 0
#define RT_TRAV_PACKET 1
#define RT_TRAV_HYBRID 2
#define RT_TRAV_STAGED 3         // staged packet walk always
#define RT_TRAV_STAGED_HYBRID 4  // staged packet walk while >= packet_min lanes

// Closest-hit query; converged call, act = lane has a query.
template <int ACCEL, bool COUNT>
__device__ __forceinline__ void closest_q(const KParams& p, const Ray& r, bool act, int depth, Best& b,
                                          Stack& s, WaveCtx& w, WorkCount& wc) {
  if (ACCEL == RT_ACCEL_FLAT_D) {
    flat_closest_w<COUNT>(p, r, act, b, w, wc);
    return;
  }
  // packet walk for coherent queries: enough lanes, and a bounce depth at
  // which rays are still coherent (camera rays: depth 0)
  bool many = __popcll(__ballot(act)) >= p.packet_min && depth <= p.packet_max_depth;
  if (p.trav == RT_TRAV_STAGED || (p.trav == RT_TRAV_STAGED_HYBRID && many))
    staged_closest<COUNT>(p, r, act, b, w, wc);
#if !RT_LEAN
  else if (p.trav == RT_TRAV_PACKET || (p.trav == RT_TRAV_HYBRID && many))
    packet_closest<COUNT>(p, r, act, b, w.ws, w.lane, wc);
#endif
  else {
    LaneCount lc = {0, 0, 0};
    if (act) oct_closest<COUNT>(p, r, b, s, lc);
    absorb<COUNT>(wc, lc);
  }
}

// Shadow query (collide_dist > 0.01, cpu/light.c:24-31); converged call.
template <int ACCEL, bool COUNT>
__device__ __forceinline__ bool shadow_q(const KParams& p, f3 o, f3 d, bool act, Stack& s,
                                         WaveCtx& w, WorkCount& wc) {
  uint64_t am = __ballot(act);
  wc.shadow += (uint32_t)__popcll(am);
#ifdef RT_DBG_SHADOW_SLOTS  // lane slots of shadow calls (in zero_normal; breakdown only)
  if (am) wc.zero_normal += 64u;
#endif
#ifdef RT_DBG_NO_SHADOW  // timing breakdown only (wrong images)
  return false;
#endif
  Ray r = make_ray(p, o, d);
  if (ACCEL == RT_ACCEL_FLAT_D) return flat_any_w<COUNT>(p, r, act, w, wc);
  bool many = __popcll(am) >= p.packet_min_shadow;
#if !RT_LEAN
  if (p.trav_shadow == RT_TRAV_STAGED || (p.trav_shadow == RT_TRAV_STAGED_HYBRID && many))
    return staged_any<COUNT>(p, r, act, w, wc);
  if (p.trav_shadow == RT_TRAV_PACKET || (p.trav_shadow == RT_TRAV_HYBRID && many))
    return packet_any<COUNT>(p, r, act, w.ws, w.lane, wc);
#else
  (void)many;
#endif
  LaneCount lc = {0, 0, 0};
  bool hit = act && oct_any<COUNT>(p, r, s, lc);
  absorb<COUNT>(wc, lc);
  return hit;
}

// cpu/light.c:7-22
__device__ __forceinline__ col specular(col tmp, f3 inc_o, f3 inc_d, f3 P, f3 N, const float* m) {
  col k = init_color(m[6], m[7], m[8]);
  f3 V = sub(inc_o, P);
  f3 R = sub(inc_d, scale(N, 2.0f * dot(N, inc_d)));
  R = normalize(R);
  V = normalize(V);
  float ls = (float)pow(fmax((double)dot(R, V), 0.0), (double)m[9]);
  k = color_mul(k, ls);
  return color_add(tmp, k);
}

// Shadow-ray direction of a directional (type 1) or point (type 2) light at
// P: cpu/light.c:53,78 (unnormalised).
__device__ __forceinline__ f3 shadow_dir(uint32_t type, f3 lv, f3 P) {
  return type == 1 ? scale(lv, -1.0f) : sub(lv, P);
}

// The unshadowed contribution of a directional or point light,
// cpu/light.c:49-66 and 68-98; P = hit point, N = interpolated (unnormalised)
// normal, m = material.
__device__ __forceinline__ col light_lit(uint32_t type, col lc, f3 lv, const float* m, f3 P,
                                         f3 N) {
  if (type == 1) {  // DIRECTIONAL
    f3 Ldir = scale(lv, -1.0f);
    col tmp = color_mul2(lc, init_color(m[3], m[4], m[5]));
    tmp = color_mul(tmp, dot(Ldir, N));
    f3 inc_o = add(P, scale(lv, -10.0f));
    return specular(tmp, inc_o, lv, P, N, m);
  }
  // POINT: "L" is minus the light position
  f3 to_l = sub(lv, P);
  f3 Lp = scale(lv, -1.0f);
  f3 Nf = N;
  if (dot(Lp, Nf) < 0.0f) Nf = scale(Nf, -1.0f);
  float dist = length(sub(lv, P));
  col tmp = color_mul2(lc, init_color(m[3], m[4], m[5]));
  tmp = color_mul(tmp, dot(Lp, Nf) * 1.0f / dist);
  f3 inc_o = add(P, scale(to_l, -10.0f));
  return specular(tmp, inc_o, to_l, P, N, m);
}

// cpu/light.c:33-100 for the lanes with hit.  The light loop is wave-uniform
// so shadow queries run converged.
template <int ACCEL, bool COUNT>
__device__ col apply_light(const KParams& p, bool hit, const float* m, f3 P, f3 N, Stack& s,
                           WaveCtx& w, WorkCount& wc) {
  col acc = init_color(0.0f, 0.0f, 0.0f);
  for (uint32_t li = 0; li < p.nlight; li++) {
    const float* L = p.light + RT_LIGHT_FLOATS_D * li;
    uint32_t type = __float_as_uint(L[0]);
    col lc = init_color(L[1], L[2], L[3]);
    f3 lv = f3{L[4], L[5], L[6]};
    if (type == 0) {  // AMBIENT
      if (hit) acc = color_add(acc, color_mul2(lc, init_color(m[0], m[1], m[2])));
    } else if (type == 1 || type == 2) {
      s.slot = li & 1u;
      bool sh = shadow_q<ACCEL, COUNT>(p, P, shadow_dir(type, lv, P), hit, s, w, wc);
      if (hit && !sh) acc = color_add(acc, light_lit(type, lc, lv, m, P, N));
    }
  }
  return acc;
}

// Camera rays: the triangles of this tile's candidate list (csrc/rt_cand.hip)
// and of the global list, tested with the reference's exact arithmetic after
// the walk -- the ones whose float Moller-Trumbore error region reaches
// beyond the walk's culling slack.  Wave-uniform loop, scalar record loads.
template <bool COUNT>
__device__ __forceinline__ void cand_closest(const KParams& p, const Ray& r, bool act, uint32_t tile,
                                             Best& b, WorkCount& wc) {
  if (!p.cand_start || __ballot(act) == 0) return;
  // Depth skip: a candidate's float new_dist is at least |pos - o| +
  // cand_skip[prim] (csrc/rt_cand.hip), so one whose bound exceeds every
  // lane's best - |pos - o| (plus the float error of that difference)
  // cannot win here -- one scalar compare instead of a test.
  float bl = -__builtin_inff();
  if (act)
    bl = b.dist == __builtin_inff() ? __builtin_inff()
                                    : (b.dist - length(sub(p.pos, r.o))) + (2e-3f + 4e-7f * b.dist);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) bl = fmaxf(bl, __shfl_xor(bl, off));
  const float bmax = __uint_as_float(uni(__float_as_uint(bl)));
  const uint32_t s = uni(p.cand_start[tile]), e = uni(p.cand_start[tile + 1]);
  const int lane = __lane_id();
  uint32_t tested = 0;
  // 64 entries per round trip: each lane loads one entry and its skip bound,
  // the wave then tests the survivors one after another
  for (uint32_t base = s; base < e; base += 64) {
    uint32_t prim = 0;
    bool keep = false;
    if (base + lane < e) {
      prim = p.cand[base + lane];
      keep = !(p.cand_skip[prim] > bmax);
    }
    uint64_t m = __ballot(keep);
    while (m) {
      const int j = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const float4* q = p.tri_prim + 3 * (size_t)uni(__shfl(prim, j));
      float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
      if (act) consider(r, q0, q1, q2, b);
      tested++;
    }
  }
  for (uint32_t k = 0; k < p.n_cand_global; k++) {
    const float4* q = p.tri_prim + 3 * (size_t)uni(p.cand_global[k]);
    float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
    if (act) consider(r, q0, q1, q2, b);
  }
  if (COUNT) wc.tris += tested + p.n_cand_global;
}

// One camera sample (cpu/raytracer.c:19-34) for every lane of the wave: the
// recursion becomes a wave-uniform bounce loop; local terms are buffered and
// folded deepest-first.  valid = the lane owns a pixel.
template <int ACCEL, bool COUNT>
__device__ __forceinline__ col trace_path(const KParams& p, bool valid, f3 o, f3 d, float coef, Stack& s,
                          WaveCtx& w, WorkCount& wc, uint32_t tile) {
  col terms[kMaxDepth];
  int depth = 0;
  bool alive = valid;
  for (;;) {
    alive = alive && !((double)coef < 0.01);  // checked before the query
    uint64_t am = __ballot(alive);
    if (am == 0) break;
    wc.closest += (uint32_t)__popcll(am);  // wave-uniform counters (SGPRs)
    Ray r = make_ray(p, o, d);
    Best b;
    b.dist = __builtin_inff();
    b.t_cut = __builtin_inff();
    b.prim = 0xffffffffu;
    b.obj = 0;
    b.u = b.v = 0.0f;
#if RT_BEST_T
    b.t = 0.0f;
#else
    b.pt = o;
#endif
    closest_q<ACCEL, COUNT>(p, r, alive, depth, b, s, w, wc);
    if (ACCEL != RT_ACCEL_FLAT_D && depth == 0) cand_closest<COUNT>(p, r, alive, tile, b, wc);
    bool hit = alive && b.dist != __builtin_inff();
    f3 N = f3{0.0f, 0.0f, 0.0f};
    wc.hits += (uint32_t)__popcll(__ballot(hit));
    bool zero = false;
    if (hit) {
      const float* nm = p.nrm + 9 * (size_t)b.prim;
      float w0 = 1.0f - b.u - b.v;
      N = add(add(scale(ld3(nm), w0), scale(ld3(nm + 3), b.u)), scale(ld3(nm + 6), b.v));
      zero = is_zero(N);  // cpu/hit.c:79 would skip this object; see DESIGN.md
    }
    wc.zero_normal += (uint32_t)__popcll(__ballot(zero));
    hit = hit && !zero;
    const float* m = p.mat + RT_MAT_FLOATS_D * (hit ? b.obj : 0u);
#if RT_BEST_T
    // the winner's hit point, same operations as hit_dist (same bits)
    f3 P = hit ? add(r.o, scale(r.nd, b.t * r.dlen)) : o;
#else
    f3 P = b.pt;
#endif
    col local = apply_light<ACCEL, COUNT>(p, hit, m, P, N, s, w, wc);
    alive = hit;
#ifdef RT_DBG_NO_BOUNCE  // timing breakdown only (wrong images)
    alive = false;
#endif
    bool deep = hit && depth == kMaxDepth;
    wc.overflow += (uint32_t)__popcll(__ballot(deep));
    if (hit) {
      if (deep) {
        alive = false;
      } else {
        terms[depth++] = color_mul(local, coef);
        d = bounce_dir(d, N);
        o = P;
        coef = m[10] * coef;
      }
    }
  }
  col acc = init_color(0.0f, 0.0f, 0.0f);
  for (int k = depth - 1; k >= 0; --k) acc = color_add(acc, terms[k]);
  return acc;
}

template <int ACCEL, bool COUNT, int MINW>
__global__ __launch_bounds__(64, MINW) void render_kernel(KParams p) {
  const int lane = threadIdx.x & 63;
  WorkCount wc = {};
  __shared__ uint32_t s_idx[ACCEL == RT_ACCEL_FLAT_D ? 1 : kLdsStack * 64];
  __shared__ float s_t[ACCEL == RT_ACCEL_FLAT_D ? 1 : kLdsStack * 64];
  __shared__ uint32_t s_ws[ACCEL == RT_ACCEL_FLAT_D ? 1 : kWaveStack];
  __shared__ float4 s_stk2[ACCEL == RT_ACCEL_FLAT_D ? 1 : 2 * kStack2];
  __shared__ float4 s_stage[ACCEL == RT_ACCEL_FLAT_D ? kStageFlat : kStageOct];
  __shared__ uint64_t s_stkm[ACCEL == RT_ACCEL_FLAT_D ? 1 : kStack2];
  Stack stk;
  stk.idx = s_idx;
  stk.tt = s_t;
  stk.spill = p.spill + ((size_t)blockIdx.x * 64 + (size_t)lane) * kSpillStack;
  stk.lane = lane;
  stk.sp = 0;
  stk.occ = stk.occ2 = 0xffffffffu;
  stk.slot = 0;
  WaveCtx w;
  w.ws = s_ws;
  w.stk2 = s_stk2;
  w.stkm = s_stkm;
  w.stage = s_stage;
  w.lane = lane;
  // Tile scheduling: the rank's tiles are cut into RT_BANDS contiguous bands
  // (image stripes); workgroup b starts on band b % RT_BANDS and moves on to
  // the other bands when its own is drained.  Default one band: every wave
  // pulls the next tile in scanline order (rt_kernels.h says why).
  const uint32_t nt = (uint32_t)p.ntiles_local;
  const uint32_t home = (uint32_t)blockIdx.x % RT_BANDS;
  uint32_t probe = 0;
  for (;;) {
    uint32_t band = (home + probe) % RT_BANDS;
    uint32_t lo = (uint32_t)(((uint64_t)nt * band) / RT_BANDS);
    uint32_t hi = (uint32_t)(((uint64_t)nt * (band + 1)) / RT_BANDS);
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(p.tile_counter + band, 1u);
    t = uni(t);
    if (t >= hi - lo) {
      if (++probe == RT_BANDS) break;  // every band drained: the wave exits
      continue;
    }
    t += lo;
    uint32_t g = t * (uint32_t)p.nranks + (uint32_t)p.rank;  // global tile index
    int ty = (int)(g / (uint32_t)p.tiles_x), tx = (int)(g % (uint32_t)p.tiles_x);
    int pr = ty * 8 + (lane >> 3), pc = tx * 8 + (lane & 7);
    // PPM (row, col) -> framebuffer slot (j, i) of cpu/raytracer.c:71,128-134
    int ii = p.W - pc, jj = p.H - pr;
    bool valid = pr < p.H && pc < p.W && ii >= 1 && ii <= 2 * (p.W / 2) && jj >= 1 &&
                 jj <= 2 * (p.H / 2);
    int i = ii - p.W / 2, j = jj - p.H / 2;
    col acc = init_color(0.0f, 0.0f, 0.0f);
    wc.pixels += (uint32_t)__popcll(__ballot(valid));
    // for (float k = i; k < i + 1; k += 0.5) for (float l = j; ...)  (cpu/raytracer.c:55-58)
    for (int sk = 0; sk < 2; sk++) {
      float k = (float)i + 0.5f * (float)sk;
      for (int sl = 0; sl < 2; sl++) {
        float l = (float)j + 0.5f * (float)sl;
        f3 point = add(add(p.C, scale(p.u, k)), scale(p.v, l));
        f3 dir = normalize(sub(p.pos, point));
        col sc = trace_path<ACCEL, COUNT>(p, valid, point, dir, 1.0f, stk, w, wc, t);
        acc = color_add(acc, color_mul(sc, 0.25f));
      }
    }
    if (!valid) acc = col{0.0f, 0.0f, 0.0f};
    float* out = p.out + ((size_t)t * 64 + (size_t)lane) * 3;
    out[0] = acc.r;
    out[1] = acc.g;
    out[2] = acc.b;
  }
  // the counters are wave totals already: one atomic per counter per wave
  uint32_t v[8] = {wc.closest, wc.shadow,   wc.pixels,      wc.nodes,
                   wc.tris,    wc.overflow, wc.zero_normal, wc.hits};
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (lane == 0 && v[k]) atomicAdd(p.stats + k, (unsigned long long)v[k]);
}

// tiles of all ranks (rank-major, as gathered) -> PPM-order image
__global__ __launch_bounds__(256) void assemble_kernel(const float* __restrict__ tiles,
                                                       float* __restrict__ rgb, int W, int H,
                                                       int tiles_x, int ntiles, int nranks,
                                                       int tiles_per_rank) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t npx = (size_t)W * (size_t)H;
  if (idx >= npx) return;
  int row = (int)(idx / (size_t)W), col = (int)(idx % (size_t)W);
  int g = (row >> 3) * tiles_x + (col >> 3);
  int rank = g % nranks, local = g / nranks;
  int lane = ((row & 7) << 3) | (col & 7);
  const float* src = tiles + (((size_t)rank * tiles_per_rank + local) * 64 + lane) * 3;
  rgb[3 * idx + 0] = src[0];
  rgb[3 * idx + 1] = src[1];
  rgb[3 * idx + 2] = src[2];
  (void)ntiles;
}

}  // namespace rt

// ---------------------------------------------------------------- launchers
#ifndef RT_DEFAULT_MIN_WAVES
#define RT_DEFAULT_MIN_WAVES 4
#endif

template <int ACCEL, bool COUNT>
static void launch_render(const KParams* p, int min_waves, dim3 g, dim3 b, hipStream_t stream) {
  switch (min_waves) {
    case 2: hipLaunchKernelGGL((rt::render_kernel<ACCEL, COUNT, 2>), g, b, 0, stream, *p); break;
    case 5: hipLaunchKernelGGL((rt::render_kernel<ACCEL, COUNT, 5>), g, b, 0, stream, *p); break;
    case 3: hipLaunchKernelGGL((rt::render_kernel<ACCEL, COUNT, 3>), g, b, 0, stream, *p); break;
    default: hipLaunchKernelGGL((rt::render_kernel<ACCEL, COUNT, 4>), g, b, 0, stream, *p); break;
  }
}

extern "C" hipError_t rt_launch_render(const KParams* p, int accel, int count_work, int min_waves,
                                       int grid, hipStream_t stream) {
  dim3 g(grid), b(64);
  if (min_waves == 0) min_waves = RT_DEFAULT_MIN_WAVES;
  if (accel == RT_ACCEL_FLAT_D) {
    if (count_work)
      launch_render<RT_ACCEL_FLAT_D, true>(p, min_waves, g, b, stream);
    else
      launch_render<RT_ACCEL_FLAT_D, false>(p, min_waves, g, b, stream);
  } else {
    if (count_work)
      launch_render<RT_ACCEL_OCTREE_D, true>(p, min_waves, g, b, stream);
    else
      launch_render<RT_ACCEL_OCTREE_D, false>(p, min_waves, g, b, stream);
  }
  return hipGetLastError();
}

extern "C" hipError_t rt_launch_assemble(const float* tiles, float* rgb, int W, int H, int tiles_x,
                                         int ntiles, int nranks, int tiles_per_rank,
                                         hipStream_t stream) {
  size_t npx = (size_t)W * (size_t)H;
  dim3 g((unsigned)((npx + 255) / 256)), b(256);
  hipLaunchKernelGGL(rt::assemble_kernel, g, b, 0, stream, tiles, rgb, W, H, tiles_x, ntiles,
                     nranks, tiles_per_rank);
  return hipGetLastError();
}
