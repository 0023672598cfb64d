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
// force, cpu/hit.c:72-109) streamed through LDS; OCTREE walks the octree
// (host/accel.c or csrc/rt_build.hip) front to back with conservative
// distance culling, as a wave-wide staged packet (coherent queries) or one
// stack per lane (incoherent ones), then tests the camera-ray candidate
// lists of csrc/rt_cand.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_cull.h"
#include "rt_device.h"
#include "rt_kernels.h"
#include "rt_reflect.h"
#include "rt_tiles.h"

namespace rt {

static constexpr float kEps = 0.0000001f;  // cpu/hit.c:7 (float)1e-7

// The workgroup is one wave and a wave's LDS instructions execute in issue
// order, so LDS staging needs no s_barrier: only a compiler barrier that
// keeps the LDS reads and writes in source order.
__device__ __forceinline__ void wave_sync() { __asm__ volatile("" ::: "memory"); }

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
  float dlen;  // length(d)
  float eps;   // culling slack (world units) for this origin
  f3 oh, ol;   // o + eps, o - eps: the grown slab planes' offsets (rt_cull.h)
};

__device__ __forceinline__ Ray make_ray(const KParams& p, f3 o, f3 d, float eps_rel) {
  Ray r;
  r.o = o;
  r.d = d;
  r.dlen = length(d);
  r.eps = rt_cull_eps(eps_rel, o.x - p.scene_c.x, o.y - p.scene_c.y, o.z - p.scene_c.z,
                      p.scene_cmag, p.scene_r);
  r.oh = f3{o.x + r.eps, o.y + r.eps, o.z + r.eps};
  r.ol = f3{o.x - r.eps, o.y - r.eps, o.z - r.eps};
  return r;
}

// The hit point o + normalize(d) * (t*|d|) (cpu/hit.c:35-37,58), with
// normalize(d) recomputed here (the same IEEE divisions every time, so the
// same bits) rather than kept live through the walks.
__device__ __forceinline__ f3 hit_point(const Ray& r, float t) {
  f3 nd{r.d.x / r.dlen, r.d.y / r.dlen, r.d.z / r.dlen};
  return add(r.o, scale(nd, t * r.dlen));
}

// new_dist = |hit point - o| (cpu/hit.c:58)
__device__ __forceinline__ float hit_dist(const Ray& r, float t) {
  return length(sub(hit_point(r, t), r.o));
}

// Conservative pre-filter of the Moller-Trumbore test.  h, a, s.h, d.q, e2.q
// are the reference's own float values (same operations); only the IEEE
// division f = 1/a is replaced by v_rcp_f32 (1 ulp).  A triangle is dropped
// only when the reference's u, v, t (which differ from these by a few ulps)
// are certain to fail cpu/hit.c:20-33, or when its distance certainly exceeds
// t_cut (closest hit: it cannot beat the current winner, ties included);
// survivors are re-tested exactly.  DESIGN.md "Exact MT with a cheap reject".
__device__ __forceinline__ bool mt_candidate(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float t_cut) {
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
}

// mt_candidate for two triangles at once (brute-force loops): the two
// dependency chains are independent, so they interleave and hide each
// other's VALU latency; the stages still end early when every lane of the
// wave has rejected both (ballot).  Same float operations, same decisions.
__device__ __forceinline__ void mt_candidate2(f3 o, f3 d, const float4* qa, const float4* qb,
                                              float t_cut, bool& ca, bool& cb) {
  const float m = 1e-5f;
  const f3 v0a{qa[0].x, qa[0].y, qa[0].z}, e1a{qa[0].w, qa[1].x, qa[1].y}, e2a{qa[1].z, qa[1].w, qa[2].x};
  const f3 v0b{qb[0].x, qb[0].y, qb[0].z}, e1b{qb[0].w, qb[1].x, qb[1].y}, e2b{qb[1].z, qb[1].w, qb[2].x};
  const f3 ha = cross(d, e2a), hb = cross(d, e2b);
  const float aa = dot(e1a, ha), ab = dot(e1b, hb);
  const float ra = __builtin_amdgcn_rcpf(aa), rb = __builtin_amdgcn_rcpf(ab);
  const f3 sa = sub(o, v0a), sb = sub(o, v0b);
  const float ua = dot(sa, ha) * ra, ub = dot(sb, hb) * rb;
  ca = !(aa > -kEps && aa < kEps) && !(ua < -1e-30f || ua > 1.0f + m);
  cb = !(ab > -kEps && ab < kEps) && !(ub < -1e-30f || ub > 1.0f + m);
  if (__ballot(ca || cb) == 0) return;
  const f3 qva = cross(sa, e1a), qvb = cross(sb, e1b);
  const float va = dot(d, qva) * ra, vb = dot(d, qvb) * rb;
  ca = ca && !(va < -1e-30f || ua + va > 1.0f + m);
  cb = cb && !(vb < -1e-30f || ub + vb > 1.0f + m);
  if (__ballot(ca || cb) == 0) return;
  const float ta = dot(e2a, qva) * ra, tb = dot(e2b, qvb) * rb;
  ca = ca && !(ta < kEps * (1.0f - m) || ta > t_cut);
  cb = cb && !(tb < kEps * (1.0f - m) || tb > t_cut);
}

struct Best {
  float dist;  // +inf = none
  float t_cut; // parametric bound beyond which no triangle can win (+inf = none)
  uint32_t prim, obj;
  float u, v;
  float t;  // the winner's MT t; its hit point is hit_point(r, t)
};

__device__ __forceinline__ void consider_exact(const Ray& r, const float4& q0, const float4& q1,
                                               const float4& q2, Best& b);

__device__ __forceinline__ void consider(const Ray& r, const float4& q0, const float4& q1,
                                         const float4& q2, Best& b) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  if (!mt_candidate(r.o, r.d, v0, e1, e2, b.t_cut)) return;
  consider_exact(r, q0, q1, q2, b);
}

// The reference's exact test of a prefilter survivor and the lexicographic
// (new_dist, prim) update (cpu/hit.c:15-37,58-59,82).
__device__ __forceinline__ void consider_exact(const Ray& r, const float4& q0, const float4& q1,
                                               const float4& q2, Best& b) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  float t, u, v;
  if (!mt_test(r.o, r.d, v0, e1, e2, t, u, v)) return;
  float nd = hit_dist(r, t);
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
    b.t = t;
  }
}

// consider() for wave-converged loops over LDS-broadcast records (the packet
// walk's leaves, the candidate lists): the same prefilter decisions, but one
// wave-uniform exit after the u stage instead of a divergent branch per
// stage.  Each divergent stage cost an exec save / branch / restore of scalar
// instructions per record -- as many SALU as VALU in those loops
// (profiles/r04t_c5/pmc_sq.json: 2.13 G SALU to 3.89 G VALU per trace launch);
// the v and t stages run for the whole wave once any lane passes u (a
// divergent stage costs the wave the same VALU cycles anyway).  act: the
// lane's query; the call itself must be wave-uniform.
#ifndef RT_CONSIDER_W
#define RT_CONSIDER_W 1
#endif
__device__ __forceinline__ void consider_w(const Ray& r, bool act, const float4& q0, const float4& q1,
                                           const float4& q2, Best& b) {
#if RT_CONSIDER_W
  const float m = 1e-5f;  // as mt_candidate
  const f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  const f3 h = cross(r.d, e2);
  const float a = dot(e1, h);
  const float rc = __builtin_amdgcn_rcpf(a);
  const f3 s = sub(r.o, v0);
  const float u = dot(s, h) * rc;
  bool c = act && !(a > -kEps && a < kEps) && !(u < -1e-30f || u > 1.0f + m);
  if (__ballot(c) == 0) return;
  const f3 q = cross(s, e1);
  const float v = dot(r.d, q) * rc;
  const float t = dot(e2, q) * rc;
  c = c && !(v < -1e-30f || u + v > 1.0f + m) && !(t < kEps * (1.0f - m) || t > b.t_cut);
  if (c) consider_exact(r, q0, q1, q2, b);
#else
  if (act) consider(r, q0, q1, q2, b);
#endif
}

// Records [0, n) of the LDS stage tested as broadcasts (consider_w).
// Converged call.  (The next record's reads issued during a test -- the
// index clamped, no branch -- measured slower: trace 6.05 -> 6.51 ms on C5,
// profiles/r05q_consider_w/ab_lds_pipe.log; round 1 found the same.)
__device__ __forceinline__ void stage_test(const Ray& r, bool act, uint32_t n, Best& b, const float4* stage) {
  for (uint32_t k = 0; k < n; k++) consider_w(r, act, stage[3 * k], stage[3 * k + 1], stage[3 * k + 2], b);
}

// Any hit with new_dist > 0.01 (cpu/hit.c:93-109: collide_dist > 0 <=>
// shadowed, cpu/light.c:24-31).  Early exit is exact for an object none of
// whose triangles can interpolate an exactly zero normal (record flag bit 0,
// host/accel.c): its closest hit then counts in collide_dist whatever
// triangle the walk met first.  A hit on a flagged object sets `risk`
// (reported as RT_EZERONORMAL, never silent).
__device__ __forceinline__ bool any_hit_exact(const Ray& r, const float4& q0, const float4& q1,
                                              const float4& q2, uint32_t& risk);

__device__ __forceinline__ bool any_hit_rec(const Ray& r, const float4& q0, const float4& q1,
                                            const float4& q2, uint32_t& risk) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  if (!mt_candidate(r.o, r.d, v0, e1, e2, __builtin_inff())) return false;
  return any_hit_exact(r, q0, q1, q2, risk);
}

// the exact test of a prefilter survivor (any_hit_rec)
__device__ __forceinline__ bool any_hit_exact(const Ray& r, const float4& q0, const float4& q1,
                                              const float4& q2, uint32_t& risk) {
  f3 v0{q0.x, q0.y, q0.z}, e1{q0.w, q1.x, q1.y}, e2{q1.z, q1.w, q2.x};
  float t, u, v;
  if (!mt_test(r.o, r.d, v0, e1, e2, t, u, v)) return false;
  if (!((double)hit_dist(r, t) > 0.01)) return false;
  risk |= __float_as_uint(q2.w) & RT_REC_ZERO_RISK;
  return true;
}

// -------------------------------------------------------------- OCTREE
// Per-lane traversal stack: the first kLdsStack entries live in LDS, laid
// out [entry][lane] so every lane hits its own bank; deeper entries spill to
// a per-lane area in global memory (rare: typical depth is < 16).
#ifndef RT_LDS_STACK
#define RT_LDS_STACK 10
#endif
static constexpr int kLdsStack = RT_LDS_STACK;  // per-lane stack entries in LDS (deeper: global spill)
static constexpr int kSpillStack = RT_SPILL_STACK;

struct Stack {
  uint32_t* idx;  // LDS, kLdsStack x 64
  float* tt;      // LDS, kLdsStack x 64
  uint2* spill;   // this lane's first spill entry; entry k at spill[k * stride]
  uint32_t stride;  // lanes of the launch: spill entries are [entry][lane], so the
                    // lanes of a wave at the same depth touch adjacent words
  int lane;
  int sp;
};

// Counters of one lane's own walk (divergent code); folded into the wave's
// WorkCount after the walk (absorb).
struct LaneCount {
  uint32_t nodes, tris, overflow;
  uint32_t risk;           // any hit on an object whose normal can vanish (any_hit_rec)
  uint32_t lnodes, ltris;  // this lane's own visits / tests (COUNT pass)
  uint32_t spills;         // pushes beyond the LDS part of the stack (COUNT pass)
  uint32_t unproven;       // exact reflection walk: queries outside its bound's assumptions
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
__device__ __forceinline__ void absorb(WorkCount& wc, const LaneCount& lc, bool shadow) {
  if (COUNT) {
    wc.nodes += wave_sum(lc.nodes);
    wc.tris += wave_sum(lc.tris);
    const uint32_t ln = wave_sum(lc.lnodes), lt = wave_sum(lc.ltris);
    if (shadow) {
      wc.sh_nodes += ln;
      wc.sh_tris += lt;
    } else {
      wc.cl_nodes += ln;
      wc.cl_tris += lt;
    }
  }
  wc.overflow += wave_sum(lc.overflow);
  wc.zero_risk += (uint32_t)__popcll(__ballot(lc.risk != 0));
  wc.cl_unproven += (uint32_t)__popcll(__ballot(lc.unproven != 0));
  if (COUNT) wc.stack_spills += wave_sum(lc.spills);
}

__device__ __forceinline__ void push(Stack& s, uint32_t i, float t, LaneCount& wc) {
  if (s.sp < kLdsStack) {
    s.idx[s.sp * 64 + s.lane] = i;
    s.tt[s.sp * 64 + s.lane] = t;
  } else if (s.sp < kLdsStack + kSpillStack) {
    s.spill[(size_t)(s.sp - kLdsStack) * s.stride] = make_uint2(i, __float_as_uint(t));
    wc.spills++;
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
    uint2 e = s.spill[(size_t)(s.sp - kLdsStack) * s.stride];
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

// Shadow walk box test (csrc/rt_shadow.hip): the box grown by mu eps instead
// of eps, and reaching parameters t >= -nu eps / |d| (a float accept may sit
// slightly behind the origin).  mn = the node's (mu, nu), both >= 1.
__device__ __forceinline__ bool box_hit_sh(const Ray& r, f3 inv, float4 lo, float4 hi, float2 mn) {
  const float e = r.eps * mn.x;
  float tmin;
  const float ohx = r.o.x + e, ohy = r.o.y + e, ohz = r.o.z + e;
  const float olx = r.o.x - e, oly = r.o.y - e, olz = r.o.z - e;
  float tx0 = fmaf(lo.x, inv.x, -(ohx * inv.x)), tx1 = fmaf(hi.x, inv.x, -(olx * inv.x));
  float ty0 = fmaf(lo.y, inv.y, -(ohy * inv.y)), ty1 = fmaf(hi.y, inv.y, -(oly * inv.y));
  float tz0 = fmaf(lo.z, inv.z, -(ohz * inv.z)), tz1 = fmaf(hi.z, inv.z, -(olz * inv.z));
  tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
  const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  return tmax >= fmaxf(tmin, -(mn.y * r.eps) / r.dlen);
}

__device__ __forceinline__ bool rt_prune(float t_enter, float dlen, float best, float eps) {
  return t_enter * dlen > rt_prune_limit(best, eps);
}

// octant nearest to the origin side (rt_cull.h: bit a = upper half of axis a)
__device__ __forceinline__ uint32_t near_octant(f3 d) {
  return (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
}


// child-mask bit o moved to bit o ^ dm (the visiting order's index space)
__device__ __forceinline__ uint32_t mask_xor(uint32_t m, uint32_t dm) {
  if (dm & 1u) m = ((m & 0x55u) << 1) | ((m & 0xAAu) >> 1);
  if (dm & 2u) m = ((m & 0x33u) << 2) | ((m & 0xCCu) >> 2);
  if (dm & 4u) m = ((m & 0x0Fu) << 4) | ((m & 0xF0u) >> 4);
  return m;
}

// Interior node: test the children's boxes and push the hits far-to-near in
// octant order (j = 7..0, octant j ^ dm: a valid front-to-back order for the
// disjoint octant cells), so the nearest child is popped first.  Software-
// pipelined: child k+1's box is in flight while child k is tested.
// CLOSEST pushes (node, entry t) and prunes by best; any-hit pushes the
// child's own (first, info) words from its box record, so a pop needs no
// node fetch -- one dependent load per step instead of two.  (The per-lane
// any-hit walk uses push_children_any: measured on C5, 16.18 vs 16.33 ms.)
#ifndef RT_CHILD_AHEAD
#define RT_CHILD_AHEAD 1
#endif
template <bool CLOSEST, bool COUNT>
__device__ __forceinline__ void push_children(const float4* __restrict__ node, const Ray& r, f3 inv,
                                              uint32_t dm, uint32_t first, uint32_t info,
                                              float best, Stack& s, LaneCount& wc) {
  uint32_t mask = RT_NODE_MASK(info);
  uint32_t mj = mask_xor(mask, dm);
  if (!mj) return;
#if RT_CHILD_AHEAD >= 2
  // two child boxes in flight while one is tested: a cold node (the per-lane
  // reflection walks of an 8-way split's longest items) costs half the
  // serialised load latencies of one-ahead
  auto next_child = [&](uint32_t& ci) {
    const int j = 31 - __clz(mj);
    mj &= ~(1u << j);
    ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
    if (COUNT) wc.nodes += lanes_distinct(ci);
  };
  uint32_t ca, cb = 0;
  next_child(ca);
  float4 alo = node[2 * ca], ahi = node[2 * ca + 1], blo, bhi;
  bool hb = mj != 0u;
  if (hb) {
    next_child(cb);
    blo = node[2 * cb];
    bhi = node[2 * cb + 1];
  }
  for (;;) {
    const float4 clo = alo, chi = ahi;
    const uint32_t cc = ca;
    const bool more = hb;
    if (hb) {
      alo = blo;
      ahi = bhi;
      ca = cb;
      hb = mj != 0u;
      if (hb) {
        next_child(cb);
        blo = node[2 * cb];
        bhi = node[2 * cb + 1];
      }
    }
    const float t0 = box_enter(r, inv, clo, chi);
    if (CLOSEST) {
      if (t0 != __builtin_inff() && !(best != __builtin_inff() && rt_prune(t0, r.dlen, best, r.eps)))
        push(s, cc, t0, wc);
    } else if (t0 != __builtin_inff()) {
      push(s, __float_as_uint(clo.w), chi.w, wc);
    }
    if (!more) break;
  }
  return;
#endif
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
    if (CLOSEST) {
      if (t0 != __builtin_inff() && !(best != __builtin_inff() && rt_prune(t0, r.dlen, best, r.eps)))
        push(s, cc, t0, wc);
    } else if (t0 != __builtin_inff()) {
      push(s, __float_as_uint(clo.w), chi.w, wc);
    }
    if (!more) break;
  }
}

// Any-hit interior node: the children's boxes in storage order (increasing
// octant), reversed when the ray's direction octant is mostly negative, so
// the walk still tends to pop the nearer children first; no per-child
// octant arithmetic (any-hit needs no exact front-to-back order).  Child
// k+1's box is in flight while child k is tested.
template <bool COUNT>
__device__ __forceinline__ void push_children_any(const float4* __restrict__ node,
                                                  const float2* __restrict__ mu, const Ray& r,
                                                  f3 inv, uint32_t dm, uint32_t first,
                                                  uint32_t info, Stack& s, LaneCount& wc) {
  const int cnt = (int)RT_NODE_COUNT(info);
  const bool up = __popc(dm) >= 2;  // storage order = far-to-near for dm = 7
  int k = up ? 0 : cnt - 1;
  const int step = up ? 1 : -1;
  uint32_t ci = first + (uint32_t)k;
  float4 nlo = node[2 * ci], nhi = node[2 * ci + 1];
  // exact-shadow mode (mu != NULL, a kernel argument: a uniform branch)
  float2 nmu = mu ? mu[ci] : make_float2(1.0f, 0.0f);
  if (COUNT) wc.nodes += lanes_distinct(ci);
  for (int n = 0; n < cnt; n++) {
    float4 clo = nlo, chi = nhi;
    const float2 cmu = nmu;
    if (n + 1 < cnt) {
      ci += (uint32_t)step;
      nlo = node[2 * ci];
      nhi = node[2 * ci + 1];
      if (mu) nmu = mu[ci];
      if (COUNT) wc.nodes += lanes_distinct(ci);
    }
    const bool h = mu ? box_hit_sh(r, inv, clo, chi, cmu) : box_enter(r, inv, clo, chi) != __builtin_inff();
    if (h) push(s, __float_as_uint(clo.w), chi.w, wc);
  }
}

// A leaf's records, software-pipelined: record k+1 is in flight while record
// k is tested.  ANY: returns true at the first any-hit.
#ifndef RT_REC_AHEAD
#define RT_REC_AHEAD 1
#endif
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool leaf_lane(const float4* __restrict__ tri, uint32_t first,
                                          uint32_t cnt, const Ray& r, Best& b, LaneCount& wc) {
  const float4* q = tri + 3 * (size_t)first;
#if RT_REC_AHEAD >= 2
  if (!ANY) {  // closest hit: two records in flight while one is tested
    float4 a0 = q[0], a1 = q[1], a2 = q[2], b0, b1, b2;
    if (cnt > 1) {
      b0 = q[3];
      b1 = q[4];
      b2 = q[5];
    }
    for (uint32_t k = 0; k < cnt; k++) {
      const float4 q0 = a0, q1 = a1, q2 = a2;
      if (k + 1 < cnt) {
        a0 = b0;
        a1 = b1;
        a2 = b2;
        if (k + 2 < cnt) {
          b0 = q[3 * (k + 2)];
          b1 = q[3 * (k + 2) + 1];
          b2 = q[3 * (k + 2) + 2];
        }
      }
      if (COUNT) {
        wc.tris += lanes_distinct(first + k);
        wc.ltris++;
      }
      consider(r, q0, q1, q2, b);
    }
    return false;
  }
#endif
  float4 n0 = q[0], n1 = q[1], n2 = q[2];
  for (uint32_t k = 0; k < cnt; k++) {
    float4 q0 = n0, q1 = n1, q2 = n2;
    if (k + 1 < cnt) {
      n0 = q[3 * (k + 1)];
      n1 = q[3 * (k + 1) + 1];
      n2 = q[3 * (k + 1) + 2];
    }
    if (COUNT) {
      wc.tris += lanes_distinct(first + k);
      wc.ltris++;
    }
    if (ANY) {
      if (any_hit_rec(r, q0, q1, q2, wc.risk)) return true;
    } else {
      consider(r, q0, q1, q2, b);
    }
  }
  return false;
}

// Per-lane closest-hit walk (each lane its own stack).
template <bool COUNT>
__device__ void oct_closest(const KParams& p, const Ray& r, Best& b, Stack& s, LaneCount& wc) {
  const float4* __restrict__ node = p.node;
  f3 inv = inv_dir(r.d);
  uint32_t dm = near_octant(r.d);
  s.sp = 0;
  wave_sync();
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
    if (COUNT) {
      wc.nodes += lanes_distinct(ni);
      wc.lnodes++;
    }
    if (info & RT_NODE_LEAF)
      leaf_lane<false, COUNT>(p.tri, first, RT_LEAF_COUNT(info), r, b, wc);
    else
      push_children<true, COUNT>(node, r, inv, dm, first, info, b.dist, s, wc);
  }
  wave_sync();
}

// Per-lane any-hit walk; a stack entry holds the node's own (first, info).
template <bool COUNT>
__device__ bool oct_any(const KParams& p, const Ray& r, Stack& s, LaneCount& wc) {
  const float4* __restrict__ node = p.node;
  f3 inv = inv_dir(r.d);
  uint32_t dm = near_octant(r.d);
  s.sp = 0;
  wave_sync();
  {
    float4 lo = node[0], hi = node[1];
    if (COUNT) wc.nodes += lanes_distinct(0);
    const bool h = p.node_mu ? box_hit_sh(r, inv, lo, hi, p.node_mu[0])
                             : box_enter(r, inv, lo, hi) != __builtin_inff();
    if (h) push(s, __float_as_uint(lo.w), hi.w, wc);
  }
  Best unused;
  while (s.sp > 0) {
    uint32_t first;
    float info_bits;
    pop(s, first, info_bits);
    uint32_t info = __float_as_uint(info_bits);
    if (COUNT) wc.lnodes++;
    if (info & RT_NODE_LEAF) {
      if (leaf_lane<true, COUNT>(p.tri, first, RT_LEAF_COUNT(info), r, unused, wc)) {
        s.sp = 0;
        wave_sync();
        return true;
      }
    } else {
      push_children_any<COUNT>(node, p.node_mu, r, inv, dm, first, info, s, wc);
    }
  }
  wave_sync();
  return false;
}

// ------------------------------------------- exact reflection walk (policy 5)
// Reflection rays (bounce depth >= 1) with each node's box grown by the
// reach of the float Moller-Trumbore test's error region for THIS ray
// (csrc/rt_reflect.hip, DESIGN.md §2 "Reflection rays: exact by proof"): the
// node's normal cone bounds the ray's cosine with every plane below it, the
// 1e-7f accept threshold bounds it from below where the cone does not, and
// the origin's distance to the box bounds |S| = |o - v0|.  Pruning and the
// crossings behind the origin take the distance error the same way.
struct RfRay {
  f3 dh;     // d / |d| (rounded; psi covers the rounding of |axis . dh|)
  bool ok;   // |d| <= RT_RF_DLMAX (the floor factors' assumption), else counted
};

__device__ __forceinline__ RfRay rf_ray(const Ray& r) {
  RfRay q;
  const float inv = 1.0f / r.dlen;
  q.dh = f3{r.d.x * inv, r.d.y * inv, r.d.z * inv};
  q.ok = r.dlen <= RT_RF_DLMAX;
  return q;
}

// Node ni's bound for this ray: e = the box growth (world units, the walk's
// slack included; +inf: enter unconditionally), bh = how far behind the
// origin a crossing may lie (parametric), and the prune coefficients: a
// float accept below the node has t_f >= (t_enter * pa - pb) (parametric,
// when positive), so the node cannot win once that exceeds the best's t_cut.
struct RfB {
  float e, bh, pa, pb;
};

__device__ __forceinline__ RfB rf_bound(const float4* __restrict__ rf, uint32_t ni, const Ray& r, const RfRay& q,
                                        const float4& lo, const float4& hi) {
  const float4 A = rf[3 * (size_t)ni], B = rf[3 * (size_t)ni + 1], F = rf[3 * (size_t)ni + 2];
  const float inf = __builtin_inff();
  RfB o;
  // |S| <= (L1 distance to the box's farthest corner) + the longest edge below
  const float M = fmaxf(fabsf(r.o.x - lo.x), fabsf(r.o.x - hi.x)) + fmaxf(fabsf(r.o.y - lo.y), fabsf(r.o.y - hi.y)) +
                  fmaxf(fabsf(r.o.z - lo.z), fabsf(r.o.z - hi.z));
  const float Sb = M + B.w;
  const float c = fabsf(A.x * q.dh.x + A.y * q.dh.y + A.z * q.dh.z) - A.w;  // cosine lower bound
  float rps = inf, rho = 1.0f, kd = inf, r0 = inf;
  if (c > 2.0f * B.y) {  // the cone closes: rho <= Ra / c < 1/2
    rho = B.y / c;
    rps = B.x / (c - B.y);
    kd = B.z / c;
    r0 = B.w * (2.3841858e-7f + rho) / (1.0f - rho);
  }
  if (F.w < 0.5f) {  // the floor closes
    rps = fminf(rps, F.x);
    rho = fminf(rho, F.w);
    kd = fminf(kd, F.z);
    r0 = fminf(r0, F.y);
  }
  if (!(rho < 0.5f) || !q.ok) {
    o.e = inf;
    o.bh = inf;
    o.pa = 0.0f;
    o.pb = inf;
    return o;
  }
  // float evaluation of the bound: relative margins of 1e-5 (~100 roundings)
  const float up = 1.0f + 1e-5f, rho2 = rho * up;
  const float g = (rps * Sb + r0) * up;
  const float dist = Sb * kd * up;  // |S| kd: the crossing's distance error (world)
  o.e = r.eps + g;
  o.bh = dist / (1.0f - 2.0f * rho2) / r.dlen * up;
  // t* |d| <= [t_f |d| (1 + 2 eps)(1 - rho) + dist] / (1 - 2 rho) and t* >= the
  // grown box's entry (less the slab's rounding, covered by 2 eps as rt_prune):
  // t_f >= ((t_enter |d| (1 - 2^-21) - 2 eps)(1 - 2 rho) - dist) / (|d| (1 + 2 eps))
  const float s = (1.0f - 2.0f * rho2) * (1.0f - 4.8e-7f);
  o.pa = s * (1.0f - 1e-5f);
  o.pb = ((2.0f * r.eps) * (1.0f - 2.0f * rho2) + dist) / r.dlen * up;
  return o;
}

// slab test of the box grown by e (world), accepting parameters t >= -bh
__device__ __forceinline__ bool box_rf(const Ray& r, f3 inv, const float4& lo, const float4& hi, float e, float bh,
                                       float& tmin) {
  if (e == __builtin_inff()) {
    tmin = -__builtin_inff();
    return true;
  }
  const float ohx = r.o.x + e, ohy = r.o.y + e, ohz = r.o.z + e;
  const float olx = r.o.x - e, oly = r.o.y - e, olz = r.o.z - e;
  const float tx0 = fmaf(lo.x, inv.x, -(ohx * inv.x)), tx1 = fmaf(hi.x, inv.x, -(olx * inv.x));
  const float ty0 = fmaf(lo.y, inv.y, -(ohy * inv.y)), ty1 = fmaf(hi.y, inv.y, -(oly * inv.y));
  const float tz0 = fmaf(lo.z, inv.z, -(ohz * inv.z)), tz1 = fmaf(hi.z, inv.z, -(olz * inv.z));
  tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
  const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  return tmax >= fmaxf(tmin, -bh);
}

// Test node ci's box for the rf walk; true: visit, key = the node's lower
// bound on an accept's t_f (-inf: none) for pruning at push and pop.
__device__ __forceinline__ bool rf_visit(const float4* __restrict__ rf, uint32_t ci, const Ray& r, const RfRay& q,
                                         f3 inv, const float4& lo, const float4& hi, float& key) {
  const RfB bd = rf_bound(rf, ci, r, q, lo, hi);
  float tmin;
  if (!box_rf(r, inv, lo, hi, bd.e, bd.bh, tmin)) return false;
  key = bd.e == __builtin_inff() ? -__builtin_inff() : tmin * bd.pa - bd.pb;  // unbounded: never pruned
  return true;
}

template <bool COUNT>
__device__ void oct_closest_rf(const KParams& p, const Ray& r, Best& b, Stack& s, LaneCount& wc) {
  const float4* __restrict__ node = p.node;
  const float4* __restrict__ rf = p.node_rf;
  const f3 inv = inv_dir(r.d);
  const uint32_t dm = near_octant(r.d);
  const RfRay q = rf_ray(r);
  if (!q.ok) wc.unproven++;  // counted (RT_EINEXACT), and walked with every node unbounded
  s.sp = 0;
  wave_sync();
  {
    float key;
    if (rf_visit(rf, 0, r, q, inv, node[0], node[1], key)) push(s, 0, key, wc);
  }
  while (s.sp > 0) {
    uint32_t ni;
    float key;
    pop(s, ni, key);
    if (b.dist != __builtin_inff() && key > b.t_cut) continue;
    const float4 lo = node[2 * ni], hi = node[2 * ni + 1];
    const uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
    if (COUNT) {
      wc.nodes += lanes_distinct(ni);
      wc.lnodes++;
    }
    if (info & RT_NODE_LEAF) {
      leaf_lane<false, COUNT>(p.tri, first, RT_LEAF_COUNT(info), r, b, wc);
      continue;
    }
    // children far-to-near in octant order (push_children), each tested with
    // its own bound; child k+1's box and bound data in flight while k is tested
    const uint32_t mask = RT_NODE_MASK(info);
    uint32_t mj = mask_xor(mask, dm);
    if (!mj) continue;
    int j = 31 - __clz(mj);
    mj &= ~(1u << j);
    uint32_t ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
    float4 nlo = node[2 * ci], nhi = node[2 * ci + 1];
    if (COUNT) wc.nodes += lanes_distinct(ci);
    for (;;) {
      const float4 clo = nlo, chi = nhi;
      const uint32_t cc = ci;
      const bool more = mj != 0u;
      if (more) {
        j = 31 - __clz(mj);
        mj &= ~(1u << j);
        ci = first + (uint32_t)__popc(mask & ((1u << ((uint32_t)j ^ dm)) - 1u));
        nlo = node[2 * ci];
        nhi = node[2 * ci + 1];
        if (COUNT) wc.nodes += lanes_distinct(ci);
      }
      float ck;
      if (rf_visit(rf, cc, r, q, inv, clo, chi, ck) && !(b.dist != __builtin_inff() && ck > b.t_cut))
        push(s, cc, ck, wc);
      if (!more) break;
    }
  }
  wave_sync();
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
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

// majority ray-direction octant of the active lanes (child push order)
__device__ __forceinline__ uint32_t wave_near_octant(bool act, f3 d, uint64_t am) {
  int na = __popcll(am);
  uint32_t dm = 0;
  if (2 * __popcll(__ballot(act && d.x < 0.0f)) > na) dm |= 1u;
  if (2 * __popcll(__ballot(act && d.y < 0.0f)) > na) dm |= 2u;
  if (2 * __popcll(__ballot(act && d.z < 0.0f)) > na) dm |= 4u;
  return dm;
}

// ------------------------------------------- PACKET walk, LDS-staged records
// The 64 lanes of a wave walk the octree together: every fetch is one
// coalesced vector load by the lanes (lane k loads float4 k of the records)
// staged in LDS, then read back as broadcasts: a leaf's triangle records (3
// float4 each, 32 per chunk) or an interior node's child boxes (2 float4
// each, <= 8 children, contiguous) cost one memory round trip instead of one
// per record.  The wave stack holds the pushed child's whole node record (box
// + first/info) and the mask of the lanes that wanted it, so a pop needs no
// memory access before the next fetch is issued.  Camera rays of an 8x8 tile
// are coherent, so the union of the lanes' walks is barely larger than each
// one's.
// float4 staging slots per wave: FLAT streams 64 triangle records at a time;
// the octree walk stages one node's payload (<= 8 children, or a leaf's
// records, RT_OCT_LEAF_CAP = 32 of them in one chunk).  LDS per one-wave
// workgroup must stay <= 10 KB for 16 workgroups per CU.
static constexpr int kStageFlat = 192;
static constexpr int kStageOct = 96;
static constexpr int kStack2 = 96;  // wave stack entries (2 float4 each)
// float4 slots of the stack area: the staged walk's kStack2 x (2 float4 + a
// lane mask), or the per-lane stacks' kLdsStack x 64 x (index, t)
static constexpr int kStackArea = (2 * kStack2 * 16 + kStack2 * 8 > kLdsStack * 64 * 8
                                       ? 2 * kStack2 * 16 + kStack2 * 8
                                       : kLdsStack * 64 * 8) / 16;

struct WaveCtx {
  float4* stk2;    // kStack2 x 2 float4
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
    // two records per step (mt_candidate2: two independent chains), the
    // survivors tested exactly in record order
    uint32_t k = 0;
    for (; k + 1 < m; k += 2) {
      const float4 qa[3] = {w.stage[3 * k], w.stage[3 * k + 1], w.stage[3 * k + 2]};
      const float4 qb[3] = {w.stage[3 * k + 3], w.stage[3 * k + 4], w.stage[3 * k + 5]};
      bool ca = false, cb = false;
      if (act) mt_candidate2(r.o, r.d, qa, qb, b.t_cut, ca, cb);
      if (ca) consider_exact(r, qa[0], qa[1], qa[2], b);
      if (cb) consider_exact(r, qb[0], qb[1], qb[2], b);
    }
    if (k < m) {
      const float4 q0 = w.stage[3 * k], q1 = w.stage[3 * k + 1], q2 = w.stage[3 * k + 2];
      if (act) consider(r, q0, q1, q2, b);
    }
  }
  if (COUNT) {
    wc.tris += n;
    wc.cl_tris += n * (uint32_t)__popcll(__ballot(act));
  }
}

template <bool COUNT>
__device__ bool flat_any_w(const KParams& p, const Ray& r, bool act, WaveCtx& w, WorkCount& wc) {
  bool alive = act, hit = false;
  uint32_t risk = 0;
  const uint32_t n = p.nrec;
  if (__ballot(alive) == 0 || n == 0) return false;
  Fetch f = fetch_issue(p.tri, 3 * (int)chunk<kFlatRecs>(n, 0), w.lane);
  for (uint32_t base = 0; base < n; base += kFlatRecs) {
    uint32_t m = chunk<kFlatRecs>(n, base);
    fetch_commit(f, w);
    uint32_t nb = base + kFlatRecs;
    if (nb < n) f = fetch_issue(p.tri + 3 * (size_t)nb, 3 * (int)chunk<kFlatRecs>(n, nb), w.lane);
    if (COUNT) {
      wc.tris += m;
      wc.sh_tris += m * (uint32_t)__popcll(__ballot(alive));
    }
    // two records per step (mt_candidate2), as flat_closest_w
    uint32_t k = 0;
    for (; k + 1 < m; k += 2) {
      const float4 qa[3] = {w.stage[3 * k], w.stage[3 * k + 1], w.stage[3 * k + 2]};
      const float4 qb[3] = {w.stage[3 * k + 3], w.stage[3 * k + 4], w.stage[3 * k + 5]};
      bool ca = false, cb = false;
      if (alive) mt_candidate2(r.o, r.d, qa, qb, __builtin_inff(), ca, cb);
      if ((ca && any_hit_exact(r, qa[0], qa[1], qa[2], risk)) ||
          (cb && any_hit_exact(r, qb[0], qb[1], qb[2], risk))) {
        hit = true;
        alive = false;
      }
      if (__ballot(alive) == 0) break;
    }
    if (k < m && __ballot(alive) != 0) {
      const float4 q0 = w.stage[3 * k], q1 = w.stage[3 * k + 1], q2 = w.stage[3 * k + 2];
      if (alive && any_hit_rec(r, q0, q1, q2, risk)) {
        hit = true;
        alive = false;
      }
    }
    if (__ballot(alive) == 0) break;
  }
  wc.zero_risk += (uint32_t)__popcll(__ballot(risk != 0));
  return hit;
}

// Brute force, TRIANGLE-parallel: for a wave with few active lanes (deep
// reflection bounces, shadow rays of the lanes that hit, sky pixels), the
// lanes take turns: the active lane's ray is broadcast and the 64 lanes test
// 64 different triangles at a time, then the lexicographic (new_dist, prim)
// minimum is reduced across the wave -- the same decisions in another order
// (the key makes the winner order-independent).  Ray-parallel streaming pays
// the whole triangle list per wave however few lanes still query.
__device__ __forceinline__ Ray ray_of_lane(const Ray& r, int l) {
  Ray q;
  q.o = f3{__shfl(r.o.x, l), __shfl(r.o.y, l), __shfl(r.o.z, l)};
  q.d = f3{__shfl(r.d.x, l), __shfl(r.d.y, l), __shfl(r.d.z, l)};
  q.dlen = __shfl(r.dlen, l);
  q.eps = 0.0f;
  q.oh = q.o;
  q.ol = q.o;
  return q;
}

template <bool COUNT>
__device__ void flat_closest_tp(const KParams& p, const Ray& r, bool act, Best& b, WorkCount& wc) {
  const uint32_t n = p.nrec;
  const int lane = (int)(threadIdx.x & 63);
  uint64_t am = __ballot(act);
  if (COUNT) {
    wc.tris += n * (uint32_t)__popcll(am);
    wc.cl_tris += n * (uint32_t)__popcll(am);
  }
  while (am) {
    const int l = __ffsll((unsigned long long)am) - 1;
    am &= am - 1;
    const Ray q = ray_of_lane(r, l);
    Best mb;
    mb.dist = __builtin_inff();
    mb.t_cut = __builtin_inff();
    mb.prim = 0xffffffffu;
    mb.obj = 0;
    mb.u = mb.v = 0.0f;
    mb.t = 0.0f;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      if (i < n) {
        const float4* t = p.tri + 3 * (size_t)i;
        consider(q, t[0], t[1], t[2], mb);
      }
    }
    // wave minimum of (dist, prim); the winner's obj, u, v, t travel with it
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float od = __shfl_xor(mb.dist, off);
      const uint32_t op = __shfl_xor(mb.prim, off), oo = __shfl_xor(mb.obj, off);
      const float ou = __shfl_xor(mb.u, off), ov = __shfl_xor(mb.v, off), ot = __shfl_xor(mb.t, off);
      if (od < mb.dist || (od == mb.dist && op < mb.prim)) {
        mb.dist = od;
        mb.prim = op;
        mb.obj = oo;
        mb.u = ou;
        mb.v = ov;
        mb.t = ot;
      }
    }
    if (lane == l) {
      b.dist = mb.dist;
      b.prim = mb.prim;
      b.obj = mb.obj;
      b.u = mb.u;
      b.v = mb.v;
      b.t = mb.t;
    }
  }
}

template <bool COUNT>
__device__ bool flat_any_tp(const KParams& p, const Ray& r, bool act, WorkCount& wc) {
  const uint32_t n = p.nrec;
  const int lane = (int)(threadIdx.x & 63);
  uint64_t am = __ballot(act);
  bool res = false;
  uint32_t risk = 0;  // per lane: any tested triangle's flag (conservative)
  while (am) {
    const int l = __ffsll((unsigned long long)am) - 1;
    am &= am - 1;
    const Ray q = ray_of_lane(r, l);
    bool hit = false;
    uint32_t base = 0;
    for (; base < n && !hit; base += 64) {  // hit is wave-uniform (ballot)
      const uint32_t i = base + (uint32_t)lane;
      bool h = false;
      if (i < n) {
        const float4* t = p.tri + 3 * (size_t)i;
        h = any_hit_rec(q, t[0], t[1], t[2], risk);
      }
      hit = __ballot(h) != 0;
    }
    if (COUNT) {
      const uint32_t tested = base < n ? base : n;
      wc.tris += tested;
      wc.sh_tris += tested;
    }
    if (lane == l) res = hit;
  }
  wc.zero_risk += (uint32_t)__popcll(__ballot(risk != 0));
  return res;
}

// Interior node whose child boxes are staged: test them, push the ones any
// lane wants (with the mask of the lanes that want each) far-to-near in
// octant order, so the nearest child ends on top of the stack.
template <bool ANY>
__device__ __forceinline__ void stage_push_children(const Ray& r, f3 inv, uint32_t dm,
                                                    uint32_t info, bool want, float limit,
                                                    int& sp, WaveCtx& w, WorkCount& wc,
                                                    const float2* __restrict__ mu = nullptr) {
  uint32_t mask = RT_NODE_MASK(info), cnt = RT_NODE_COUNT(info);
  uint64_t lanes[8];
  uint32_t hitmask = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) {
    lanes[c] = 0;
    if ((uint32_t)c < cnt) {
      float4 clo = w.stage[2 * c], chi = w.stage[2 * c + 1];
      bool w2;
      if (ANY) {
        w2 = want && (mu ? box_hit_sh(r, inv, clo, chi, mu[c])  // exact-shadow mode's grown boxes
                         : box_enter(r, inv, clo, chi) != __builtin_inff());
      } else {
        float t0 = box_enter(r, inv, clo, chi);
        w2 = want && t0 != __builtin_inff() && !(t0 * r.dlen > limit);
      }
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
    if (COUNT) {
      wc.nodes++;
      wc.cl_nodes += (uint32_t)__popcll(__ballot(want));
    }
    fetch_commit(f, w);
    if (leaf) {
      for (uint32_t base = 0; base < cnt; base += kOctRecs) {
        uint32_t m = chunk<kOctRecs>(cnt, base);
        if (base) stage_load(tri + 3 * (size_t)(first + base), 3 * (int)m, w);
        stage_test(r, want, m, b, w.stage);
      }
      limit = rt_prune_limit(b.dist, r.eps);
      if (COUNT) {
        wc.tris += cnt;
        wc.cl_tris += cnt * (uint32_t)__popcll(__ballot(want));
      }
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
  uint32_t risk = 0;
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
    if (COUNT) {
      wc.nodes++;
      wc.sh_nodes += (uint32_t)__popcll(__ballot(want));
    }
    if (info & RT_NODE_LEAF) {
      uint32_t cnt = RT_LEAF_COUNT(info);
      for (uint32_t base = 0; base < cnt && __ballot(want) != 0; base += kOctRecs) {
        uint32_t m = chunk<kOctRecs>(cnt, base);
        stage_load(tri + 3 * (size_t)(first + base), 3 * (int)m, w);
        if (COUNT) wc.tris += m;
        for (uint32_t k = 0; k < m; k++) {
          if (COUNT) wc.sh_tris += (uint32_t)__popcll(__ballot(want));
          float4 q0 = w.stage[3 * k], q1 = w.stage[3 * k + 1], q2 = w.stage[3 * k + 2];
          if (want && any_hit_rec(r, q0, q1, q2, risk)) {
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
      stage_push_children<true>(r, inv, dm, info, want, 0.0f, sp, w, wc,
                                p.node_mu ? p.node_mu + first : nullptr);
    }
  }
  wc.zero_risk += (uint32_t)__popcll(__ballot(risk != 0));
  return hit;
}

// Traversal policy of an instantiation (RT_POLICY_*, rt_kernels.h).  The
// default: closest-hit queries walk as a staged packet while at least
// kPacketMin lanes query at a bounce depth <= kPacketMaxDepth (camera rays;
// reflections are incoherent), else per lane;
// shadow queries walk per lane, except directional-light shadows (parallel
// rays, cpu/light.c:53) under RT_POLICY_DIR_STAGED.
static constexpr int kPacketMin = 8;
// (The camera packet walk with the next node's payload copied global -> LDS
// while a leaf is tested measured slower -- round 5, profiles/r07_prefetch/:
// a second LDS stage costs occupancy, and at full occupancy the other waves
// already cover the payload latency -- and was removed.)
// Camera rays only (round 4): the reflection rays of a wave diverge, and a
// packet walks the union of their paths through cold nodes; per lane, the
// longest items of an 8-way split (reflection-heavy tiles, tools/tile_cost.py)
// finish sooner -- slowest of 8 ranks 3.13 -> 2.95 ms, C5 at N = 1 10.07 ->
// 10.04 ms (profiles/r05s_packet_depth/; round 2 measured 0 and 1 equal at N = 1)
#ifndef RT_HEAVY_PRIO
#define RT_HEAVY_PRIO 1
#endif
#ifndef RT_PACKET_MAX_DEPTH
#define RT_PACKET_MAX_DEPTH 0
#endif
static constexpr int kPacketMaxDepth = RT_PACKET_MAX_DEPTH;

// Brute force: triangle-parallel when the list is long enough to fill the
// lanes and at most kTpMaxLanes lanes query (ray-parallel streaming costs the
// same list per wave whatever the active count; triangle-parallel costs it
// once per active lane, spread over 64 lanes).  Measured on C2 (spheres,
// 4,812 triangles, 1080p, flat): never 262 ms, <= 32 lanes 160, <= 48 160,
// <= 56 159, always 250; shadows always triangle-parallel 170
// (profiles/r02q_flat_tp/).
static constexpr int kTpMaxLanes = 48;
__device__ __forceinline__ bool use_tp(const KParams& p, bool act) {
  return p.nrec >= 256u && __popcll(__ballot(act)) <= kTpMaxLanes;
}

// Closest-hit query; converged call, act = lane has a query.
template <int ACCEL, bool COUNT, int POL>
__device__ __forceinline__ void closest_q(const KParams& p, const Ray& r, bool act, int depth, Best& b,
                                          Stack& s, WaveCtx& w, WorkCount& wc) {
  if (ACCEL == RT_ACCEL_FLAT_D) {
    if (use_tp(p, act))
      flat_closest_tp<COUNT>(p, r, act, b, wc);
    else
      flat_closest_w<COUNT>(p, r, act, b, w, wc);
    return;
  }
  if (POL == RT_POLICY_EXACT_REFL && depth > 0) {  // reflection rays: the proven walk
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    if (act) oct_closest_rf<COUNT>(p, r, b, s, lc);
    absorb<COUNT>(wc, lc, false);
    return;
  }
  bool staged = POL == RT_POLICY_STAGED ||
                (POL != RT_POLICY_LANE && __popcll(__ballot(act)) >= kPacketMin &&
                 depth <= kPacketMaxDepth);
  if (staged) {
    staged_closest<COUNT>(p, r, act, b, w, wc);
  } else {
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    if (act) oct_closest<COUNT>(p, r, b, s, lc);
    absorb<COUNT>(wc, lc, false);
    if (COUNT && depth > 0) {
      uint32_t mn = lc.lnodes, mt = lc.ltris;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        mn = max(mn, (uint32_t)__shfl_xor((int)mn, off));
        mt = max(mt, (uint32_t)__shfl_xor((int)mt, off));
      }
      wc.sec_lane_nodes = max(wc.sec_lane_nodes, uni(mn));
      wc.sec_lane_tris = max(wc.sec_lane_tris, uni(mt));
    }
  }
}

// Shadow query through the light's buffer (csrc/rt_lightbuf.hip): the
// triangles listed in the cell the ray's origin projects to, in key order,
// up to the first any-hit -- for a point light also the opposite cell, whose
// triangles lie beyond the light (cpu/rt's shadow ray does not stop there,
// cpu/hit.c:93-109) -- then the light's global list.  Per lane.
// The cells a shadow ray's query scans and their entry ranges (the first
// memory round trip of a query; shade_record can issue it early).
struct LbRange {
  uint32_t rs[2], re[2];
  float lim;  // key limit of the first range (the second: none)
};

__device__ __forceinline__ LbRange lbuf_range(const RtLightBuf& L, const Ray& r) {
  uint32_t cell[2] = {0xffffffffu, 0xffffffffu};
  float lim = __builtin_inff();  // key limit of cell[0] (cell[1]: none)
  if (L.kind == RT_LB_DIR) {
    // the same float operations the build's margins assume (no contraction)
    const float pu = r.o.x * L.u[0] + r.o.y * L.u[1] + r.o.z * L.u[2];
    const float pv = r.o.x * L.v[0] + r.o.y * L.v[1] + r.o.z * L.v[2];
    const float pw = r.o.x * L.w[0] + r.o.y * L.w[1] + r.o.z * L.w[2];
    const float fx = (pu - L.u0) * L.inv_cs, fy = (pv - L.v0) * L.inv_cs;
    if (fx >= 0.0f && fy >= 0.0f && fx < (float)L.nx && fy < (float)L.ny) {
      cell[0] = (uint32_t)fy * L.nx + (uint32_t)fx;
      lim = -pw;  // keys are minus the triangles' depth bounds toward the light
    }
  } else {
    // from the light to the origin: -d, the ray's own direction negated
    const f3 x{-r.d.x, -r.d.y, -r.d.z};
    const float ax = fabsf(x.x), ay = fabsf(x.y), az = fabsf(x.z);
    uint32_t a = 0;
    float m = ax, xa = x.x, xj = x.y, xk = x.z;
    if (ay > m) {
      a = 1;
      m = ay;
      xa = x.y;
      xj = x.z;
      xk = x.x;
    }
    if (az > m) {
      a = 2;
      m = az;
      xa = x.z;
      xj = x.x;
      xk = x.y;
    }
    if (m > 0.0f) {
      const uint32_t n = L.nx;
      const float sc = xj / m, tc = xk / m;
      const uint32_t f = 2u * a + (xa < 0.0f ? 1u : 0u);
      const uint32_t ix = min((uint32_t)((sc + 1.0f) * L.half_n), n - 1u);
      const uint32_t iy = min((uint32_t)((tc + 1.0f) * L.half_n), n - 1u);
      const uint32_t jx = min((uint32_t)((1.0f - sc) * L.half_n), n - 1u);
      const uint32_t jy = min((uint32_t)((1.0f - tc) * L.half_n), n - 1u);
      cell[0] = (f * n + iy) * n + ix;
      cell[1] = ((f ^ 1u) * n + jy) * n + jx;
      lim = length(x) * (1.0f + 1e-6f);  // keys: nearest distance from the light
    }
  }
  // both cells' entry ranges (independent loads)
  LbRange g;
  g.lim = lim;
  for (int h = 0; h < 2; h++) {
    g.rs[h] = 0u;
    g.re[h] = 0u;
    if (cell[h] != 0xffffffffu) {
      g.rs[h] = L.start[cell[h]];
      g.re[h] = L.start[cell[h] + 1];
    }
  }
  return g;
}

// Each range's entries -- the record inline, its key in the prim slot: one
// contiguous load per test, no prim -> record indirection, the next record's
// load in flight (RT_LB_AHEAD).  Then the global list.
// The next entry's record in flight while an entry is tested (round 5):
// +12 VGPRs, so the shade kernel runs at 7 waves per SIMD (RT_SHADE_MIN_WAVES)
// instead of 8 -- C5 shade 1.96 -> 1.85 ms (profiles/r07_shade/; at 8 waves
// it spills: 1.92; at 6: 1.93).  Round 3 measured the lookahead at 8 waves
// only (spills, 2.72 ms).
#ifndef RT_LB_AHEAD
#define RT_LB_AHEAD 1
#endif
template <bool COUNT>
__device__ bool lbuf_scan(const KParams& p, const RtLightBuf& L, const Ray& r, const LbRange& g, LaneCount& lc) {
  for (int h = 0; h < 2; h++) {
    const float q = h == 0 ? g.lim : __builtin_inff();
#if RT_LB_AHEAD
    // the next entry's record in flight while this one is tested
    uint32_t k = g.rs[h];
    const uint32_t e = g.re[h];
    float4 n0, n1, n2;
    if (k < e) {
      const float4* t = L.rec + 3 * (size_t)k;
      n0 = t[0];
      n1 = t[1];
      n2 = t[2];
    }
    for (; k < e; k++) {
      const float4 a0 = n0, a1 = n1, a2 = n2;
      if (k + 1 < e) {
        const float4* t = L.rec + 3 * (size_t)(k + 1);
        n0 = t[0];
        n1 = t[1];
        n2 = t[2];
      }
      if (a2.y > q) break;
      if (COUNT) {
        lc.tris += lanes_distinct(k);
        lc.ltris++;
      }
      if (any_hit_rec(r, a0, a1, a2, lc.risk)) return true;
    }
#else
    for (uint32_t k = g.rs[h]; k < g.re[h]; k++) {
      const float4* t = L.rec + 3 * (size_t)k;
      const float4 a0 = t[0], a1 = t[1], a2 = t[2];
      if (a2.y > q) break;
      if (COUNT) {
        lc.tris += lanes_distinct(k);
        lc.ltris++;
      }
      if (any_hit_rec(r, a0, a1, a2, lc.risk)) return true;
    }
#endif
  }
  for (uint32_t k = 0; k < L.nglobal; k++) {
    const float4* t = p.tri_prim + 3 * (size_t)L.global[k];
    if (COUNT) {
      lc.tris += lanes_distinct(L.global[k]);
      lc.ltris++;
    }
    if (any_hit_rec(r, t[0], t[1], t[2], lc.risk)) return true;
  }
  return false;
}

template <bool COUNT>
__device__ bool lbuf_any(const KParams& p, const RtLightBuf& L, const Ray& r, LaneCount& lc) {
  return lbuf_scan<COUNT>(p, L, r, lbuf_range(L, r), lc);
}

// Shadow query (collide_dist > 0.01, cpu/light.c:24-31) of a light of the
// given type; converged call.
template <int ACCEL, bool COUNT, int POL>
__device__ __forceinline__ bool shadow_q(const KParams& p, f3 o, f3 d, uint32_t type, uint32_t li,
                                         bool act, Stack& s, WaveCtx& w, WorkCount& wc, bool* defer = nullptr,
                                         const LbRange* pre = nullptr, bool can_defer = true) {
  uint64_t am = __ballot(act);
  wc.shadow += (uint32_t)__popcll(am);
  Ray r = make_ray(p, o, d, p.eps_rel);
  if (ACCEL == RT_ACCEL_FLAT_D)
    return use_tp(p, act) ? flat_any_tp<COUNT>(p, r, act, wc) : flat_any_w<COUNT>(p, r, act, w, wc);
  if (POL == RT_POLICY_LBUF) {  // every such light has a buffer (rt_hip.cpp): no walk, no global prims
    const RtLightBuf& L = p.lbuf[li];
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    bool hit = act && (pre ? lbuf_scan<COUNT>(p, L, r, *pre, lc) : lbuf_any<COUNT>(p, L, r, lc));
    absorb<COUNT>(wc, lc, true);
    if (L.proven) {  // as below
      const bool out = act && !(o.x >= L.olo[0] && o.x <= L.ohi[0] && o.y >= L.olo[1] && o.y <= L.ohi[1] &&
                                o.z >= L.olo[2] && o.z <= L.ohi[2]);
      if (defer && can_defer && p.oob) {
        *defer = out;
        if (out) hit = false;
      } else {
        wc.sh_unproven += (uint32_t)__popcll(__ballot(out));
      }
    }
    return hit;
  }
  bool staged = POL == RT_POLICY_STAGED ||
                (POL == RT_POLICY_DIR_STAGED && type == 1 && __popcll(am) >= kPacketMin);
  bool hit, walked = true;
  if (staged) {
    hit = staged_any<COUNT>(p, r, act, w, wc);
  } else if (p.lbuf && p.lbuf[li].kind != RT_LB_NONE) {
    walked = false;
    const RtLightBuf& L = p.lbuf[li];
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    hit = act && (pre ? lbuf_scan<COUNT>(p, L, r, *pre, lc) : lbuf_any<COUNT>(p, L, r, lc));
    absorb<COUNT>(wc, lc, true);
    if (L.proven) {
      // the proof assumed origins in its box; the rare others (hit points of
      // float garbage hits far past a triangle, e.g. camera rays grazing a
      // ground plane at the horizon) are decided by brute force over every
      // record after the pass (cpu/hit.c:93-109)
      const bool out = act && !(o.x >= L.olo[0] && o.x <= L.ohi[0] && o.y >= L.olo[1] && o.y <= L.ohi[1] &&
                                o.z >= L.olo[2] && o.z <= L.ohi[2]);
      if (defer && can_defer && p.oob) {  // decided GPU-wide after the pass (rt_launch_shade_fixup)
        *defer = out;
        if (out) hit = false;
      } else {  // (lights past the 32nd) counted, never assumed: RT_EINEXACT
        wc.sh_unproven += (uint32_t)__popcll(__ballot(out));
      }
    }
  } else {
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    hit = act && oct_any<COUNT>(p, r, s, lc);
    absorb<COUNT>(wc, lc, true);
  }
  // the prims whose float error region no slack multiplier bounds
  // (csrc/rt_shadow.hip): tested by every ray the walk found unshadowed (a
  // light buffer's proof covers its light's queries without them)
  if (walked && p.n_sh_global && __ballot(act && !hit)) {
    uint32_t risk = 0;
    for (uint32_t k = 0; k < p.n_sh_global; k++) {
      const float4* q = p.tri_prim + 3 * (size_t)uni(p.sh_global[k]);
      const float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
      if (act && !hit) hit = any_hit_rec(r, q0, q1, q2, risk);
      if (__ballot(act && !hit) == 0) break;
    }
    wc.zero_risk += (uint32_t)__popcll(__ballot(risk != 0));
  }
  // point lights (exact-shadow mode): the cosine bound assumed origins within
  // sh_omax of the scene centre
  if (walked && type == 2 && p.node_mu) {
    const float m = fmaxf(fabsf(o.x - p.scene_c.x), fmaxf(fabsf(o.y - p.scene_c.y), fabsf(o.z - p.scene_c.z)));
    wc.sh_unproven += (uint32_t)__popcll(__ballot(act && !(m <= p.sh_omax)));
  }
  return hit;
}

// pow of cpu/light.c:20, out of line: inlined, its f64 polynomial
// coefficients were hoisted out of the path loop and spilled to scratch.
#ifndef RT_SPEC_POW_INLINE
#define RT_SPEC_POW_INLINE __noinline__
#endif
__device__ RT_SPEC_POW_INLINE float spec_pow(double x, double e) { return (float)pow(fmax(x, 0.0), e); }

// cpu/light.c:7-22
__device__ __forceinline__ col specular(col tmp, f3 inc_o, f3 inc_d, f3 P, f3 N, const float* m) {
  col k = init_color(m[6], m[7], m[8]);
  f3 V = sub(inc_o, P);
  f3 R = sub(inc_d, scale(N, 2.0f * dot(N, inc_d)));
  R = normalize(R);
  V = normalize(V);
  float ls = spec_pow((double)dot(R, V), (double)m[9]);
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
template <int ACCEL, bool COUNT, int POL>
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
      const uint64_t c0 = COUNT ? __builtin_readcyclecounter() : 0ull;
      bool sh = shadow_q<ACCEL, COUNT, POL>(p, P, shadow_dir(type, lv, P), type, li, hit, s, w, wc);
      if (COUNT) {
        const uint32_t dc = (uint32_t)(__builtin_readcyclecounter() - c0);
        wc.cy_shadow += dc;
        if (type == 1) wc.cy_shadow_dir += dc;
      }
      if (hit && !sh) acc = color_add(acc, light_lit(type, lc, lv, m, P, N));
    }
  }
  return acc;
}

// Camera rays: the triangles of this tile's candidate list (csrc/rt_cand.hip)
// and of the global list, tested with the reference's exact arithmetic after
// the walk -- the ones whose float Moller-Trumbore error region reaches
// beyond the walk's culling slack.
// Entries [s, e) of the candidate list (kOctRecs per round: each lane loads
// one entry and its skip bound, the survivors' records are gathered in
// parallel -- one memory round trip -- into the LDS stage, compacted, then
// tested one after another as LDS broadcasts).  bmax: entries whose depth
// skip bound exceeds it cannot win any lane.  Returns the entries tested.
#ifndef RT_CAND_AHEAD
#define RT_CAND_AHEAD 0
#endif
template <bool COUNT>
__device__ __forceinline__ uint32_t cand_range(const KParams& p, const Ray& r, bool act, uint32_t s, uint32_t e,
                                               float bmax, Best& b, WaveCtx& w) {
  const int lane = w.lane;
  uint32_t tested = 0;
#if RT_CAND_AHEAD
  // the next round's entries (prim, skip bound) in flight while this round's
  // records are gathered and tested
  uint32_t nprim = 0;
  float nskip = 0.0f;
  if (lane < kOctRecs && s + lane < e) {
    nprim = p.cand[s + lane];
    nskip = p.cand_skip[s + lane];
  }
#endif
  for (uint32_t base = s; base < e; base += kOctRecs) {
    uint32_t prim = 0;
    bool keep = false;
#if RT_CAND_AHEAD
    if (lane < kOctRecs && base + lane < e) {
      prim = nprim;
      keep = !(nskip > bmax);
    }
    if (lane < kOctRecs && base + kOctRecs + lane < e) {
      nprim = p.cand[base + kOctRecs + lane];
      nskip = p.cand_skip[base + kOctRecs + lane];
    }
#else
    if (lane < kOctRecs && base + lane < e) {
      prim = p.cand[base + lane];
      keep = !(p.cand_skip[base + lane] > bmax);
    }
#endif
    const uint64_t m = __ballot(keep);
    if (m == 0) continue;
    const uint32_t n = (uint32_t)__popcll(m);
    const uint32_t slot = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    float4 g0, g1, g2;
    if (keep) {
      const float4* q = p.tri_prim + 3 * (size_t)prim;
      g0 = q[0];
      g1 = q[1];
      g2 = q[2];
    }
    wave_sync();  // after the previous readers of stage
    if (keep) {
      w.stage[3 * slot] = g0;
      w.stage[3 * slot + 1] = g1;
      w.stage[3 * slot + 2] = g2;
    }
    wave_sync();
    // (two candidates per step as two scalar chains, as the brute-force loops
    // do, measured slower here: C5 frame 15.96 -> 16.10 ms,
    // profiles/r03f_bench/ab.log; two per packed-float instruction, RT_CAND_PK
    // of round 3, slower too: profiles/r04e_pk/ab.log)
    stage_test(r, act, n, b, w.stage);
    tested += n;
  }
  return tested;
}

template <bool COUNT>
__device__ __forceinline__ void cand_closest(const KParams& p, const Ray& r, bool act, uint32_t tile,
                                             Best& b, WaveCtx& w, WorkCount& wc) {
  if (!p.cand_start || __ballot(act) == 0) return;
    // Depth skip: a candidate's float new_dist is at least |pos - o| + its
    // entry's cand_skip (csrc/rt_cand.hip), so one whose bound exceeds every
    // lane's best - |pos - o| (plus the float error of that difference)
    // cannot win here -- one compare instead of a test.  (A per-lane test of
    // the footprint's image-space band, measured: the bands of the long
    // footprints are 6-34 pixels wide, so nearly every listed tile has lanes
    // inside; it removed 1 % of the tests and cost 2.7 ms on C5.)
    float bl = -__builtin_inff();
    if (act)
      bl = b.dist == __builtin_inff() ? __builtin_inff()
                                      : (b.dist - length(sub(p.pos, r.o))) + (2e-3f + 4e-7f * b.dist);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) bl = fmaxf(bl, __shfl_xor(bl, off));
    const float bmax = __uint_as_float(uni(__float_as_uint(bl)));
  const uint32_t tested =
      cand_range<COUNT>(p, r, act, uni(p.cand_start[tile]), uni(p.cand_start[tile + 1]), bmax, b, w);
  const uint32_t n_glob = p.n_cand_global_dev ? uni(*p.n_cand_global_dev) : p.n_cand_global;
  for (uint32_t k = 0; k < n_glob; k++) {
    const float4* q = p.tri_prim + 3 * (size_t)uni(p.cand_global[k]);
    float4 q0 = ldu(q, 0), q1 = ldu(q, 1), q2 = ldu(q, 2);
    if (act) consider(r, q0, q1, q2, b);
  }
  if (COUNT) {
    wc.tris += tested + n_glob;
    wc.cl_tris += (tested + n_glob) * (uint32_t)__popcll(__ballot(act));
  }
}

// PPM (row, col) of lane `lane` of rank-local tile t (rt_hip.h "Image
// tiling", csrc/rt_tiles.h): 8 x 8 pixels, lane = row * 8 + col.
__device__ __forceinline__ void tile_pixel(const KParams& p, uint32_t t, int lane, int& pr,
                                           int& pc) {
  int tx, ty;
  const int tb = rt_block_side(p.nranks);
  rt_tile_xy(t, (uint32_t)p.rank, (uint32_t)p.nranks, (uint32_t)rt_blocks_x(p.tiles_x, tb), (uint32_t)tb,
             &tx, &ty);
  pr = ty * 8 + (lane >> 3);
  pc = tx * 8 + (lane & 7);
}

// The wave's counters are wave totals already: one atomic per counter per
// wave.  The wave-distinct record fetches (nodes, tris) of the shade kernel's
// shadow queries go to their own slots, so each kernel's algorithmic bytes
// can be priced on its own (bench.py roofline).
__device__ __forceinline__ void flush_counts(const KParams& p, const WorkCount& wc, int lane,
                                             bool shade = false) {
  uint32_t v[RT_NSTATS] = {wc.closest, wc.shadow,   wc.pixels,      shade ? 0u : wc.nodes,
                           shade ? 0u : wc.tris,    wc.overflow, wc.zero_normal, wc.hits,
                           wc.cl_nodes, wc.cl_tris, wc.sh_nodes,   wc.sh_tris,
                           wc.cy_cam,   wc.cy_cand, wc.cy_sec,     wc.cy_shadow,
                           wc.cy_shadow_dir, wc.stack_spills, wc.zero_risk,
                           shade ? wc.nodes : 0u, shade ? wc.tris : 0u, wc.sh_unproven, wc.cl_unproven};
#pragma unroll
  for (int k = 0; k < RT_NSTATS; k++)
    if (lane == 0 && v[k])
      atomicAdd(p.stats + (size_t)(blockIdx.x % RT_STAT_SETS) * RT_STAT_STRIDE + k, (unsigned long long)v[k]);
}

// ---------------------------------------------------------- wavefront split
// A render is three launches.  trace_kernel follows every camera sample's
// path of closest hits (cpu/raytracer.c:19-34) and appends one hit record per
// hit -- the bounce never depends on the shading: ray_bounce takes only the
// hit (cpu/raytracer.c:28, cpu/ray.c:16-25) and the next coefficient only the
// material (cpu/raytracer.c:29).  shade_kernel then runs the shadow queries
// and Phong terms of every record (cpu/light.c:33-100) with the 64 lanes of a
// wave on 64 records -- no lane idles on a sky pixel or an ended path -- in a
// lean kernel that keeps more waves resident than the walk-heavy trace, and
// writes the record's term color_mul(local, coef) (cpu/raytracer.c:30).
// fold_kernel sums each path's terms deepest-first (color_add(reflection,
// term) from the deepest call outwards) and a pixel's four samples in the
// reference's order.  The same operations on the same values as the
// recursion, so the same bits; a path's length is bounded only by
// RT_MAX_BOUNCES (cpu/rt: by its stack).

// Hit record, 2 float4: P.xyz N.x | N.y N.z coef bits(obj); its path's
// previous record in hit_prev.  Record index = region | (slot << 3).
__device__ __forceinline__ size_t rec_addr(const KParams& p, uint32_t idx) {
  return (size_t)(idx & 7u) * p.hit_cap + (idx >> 3);
}

// Camera sample smp of lane `lane` of rank-local tile t: its ray (origin on
// the film, direction towards the eye) exactly as cpu/raytracer.c:55-60
// computes it; false when the lane's pixel lies outside the framebuffer's
// even-sized area (its ray is still defined).
__device__ __forceinline__ bool camera_sample(const KParams& p, uint32_t t, int smp, int lane, f3& point, f3& dir) {
  int pr, pc;
  tile_pixel(p, t, lane, pr, pc);
  // PPM (row, col) -> framebuffer slot (j, i) of cpu/raytracer.c:71,128-134
  const int ii = p.W - pc, jj = p.H - pr;
  const bool valid = pr < p.H && pc < p.W && ii >= 1 && ii <= 2 * (p.W / 2) && jj >= 1 && jj <= 2 * (p.H / 2);
  const int i = ii - p.W / 2, j = jj - p.H / 2;
  // for (float k = i; k < i + 1; k += 0.5) for (float l = j; ...)  (cpu/raytracer.c:55-58)
  const float k = (float)i + 0.5f * (float)(smp >> 1);
  const float l = (float)j + 0.5f * (float)(smp & 1);
  point = add(add(p.C, scale(p.u, k)), scale(p.v, l));
  dir = normalize(sub(p.pos, point));
  return valid;
}

// One camera sample for every lane of the wave (trace_kernel): the
// recursion as a wave-uniform bounce loop, a hit record appended per hit (one
// atomic per wave and bounce, on the item stream's own counter x).  Returns
// the lane's deepest record (RT_NO_REC: none).  valid = the lane owns a pixel.
template <int ACCEL, bool COUNT, int POL>
__device__ __forceinline__ uint32_t trace_path(const KParams& p, bool valid, f3 o, f3 d,
                                               uint32_t x, Stack& s, WaveCtx& w, WorkCount& wc,
                                               uint32_t tile, int depth = 0, float coef = 1.0f,
                                               uint32_t prev = RT_NO_REC) {
  // depth: wave-uniform, queries so far on this path
  bool alive = valid;
  for (;;) {
    alive = alive && !((double)coef < 0.01);  // checked before the query
    uint64_t am = __ballot(alive);
    if (am == 0) break;
    wc.closest += (uint32_t)__popcll(am);  // wave-uniform counters (SGPRs)
    Ray r = make_ray(p, o, d, depth == 0 ? p.eps_rel_cam : p.eps_rel);
    Best b;
    b.dist = __builtin_inff();
    b.t_cut = __builtin_inff();
    b.prim = 0xffffffffu;
    b.obj = 0;
    b.u = b.v = 0.0f;
    b.t = 0.0f;
    uint64_t c0 = COUNT ? __builtin_readcyclecounter() : 0ull;
    closest_q<ACCEL, COUNT, POL>(p, r, alive, depth, b, s, w, wc);
    if (COUNT) {
      const uint64_t c1 = __builtin_readcyclecounter();
      (depth == 0 ? wc.cy_cam : wc.cy_sec) += (uint32_t)(c1 - c0);
      c0 = c1;
    }
    if (ACCEL != RT_ACCEL_FLAT_D && depth == 0) cand_closest<COUNT>(p, r, alive, tile, b, w, wc);
    if (COUNT) wc.cy_cand += (uint32_t)(__builtin_readcyclecounter() - c0);
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
    const uint64_t hm = __ballot(hit);
    if (hm == 0) break;
    uint32_t base = 0;
    if (w.lane == 0) base = atomicAdd(p.hit_count + 32u * x, (uint32_t)__popcll(hm));
    base = uni(base);
    bool deep = false;
    if (hit) {
      const uint32_t slot = base + (uint32_t)__popcll(hm & ((1ull << w.lane) - 1ull));
      const f3 P = hit_point(r, b.t);  // the winner's hit point, same bits
      if (slot < p.hit_cap) {  // else: counted, and rt_hip_stats reports the overflow
        const size_t a = (size_t)x * p.hit_cap + slot;
        p.hit[2 * a] = make_float4(P.x, P.y, P.z, N.x);
        p.hit[2 * a + 1] = make_float4(N.y, N.z, coef, __uint_as_float(b.obj));
        p.hit_prev[a] = prev;
      }
      prev = x | (slot << 3);
      const float ncoef = p.mat[RT_MAT_FLOATS_D * (size_t)b.obj + 10] * coef;  // obj.nr * coef
      if (depth + 1 >= RT_MAX_BOUNCES) {
        deep = !((double)ncoef < 0.01);  // cpu/rt would query again: never silent
      } else {
        d = bounce_dir(d, N);
        o = P;
        coef = ncoef;
      }
    }
    wc.overflow += (uint32_t)__popcll(__ballot(deep));
    alive = hit && depth + 1 < RT_MAX_BOUNCES;
    ++depth;
  }
  return prev;
}

template <int ACCEL, bool COUNT, int POL>
__global__ __launch_bounds__(64, RT_TRACE_MIN_WAVES) void trace_kernel(KParams p) {
  const int lane = threadIdx.x & 63;
  WorkCount wc = {};
  // The per-lane stacks and the staged wave stack share one LDS area: a
  // wave runs one walk at a time and every walk starts and ends with an
  // empty stack (wave_sync() at both ends orders the accesses).
  __shared__ float4 s_stack[ACCEL == RT_ACCEL_FLAT_D ? 1 : kStackArea];
  __shared__ float4 s_stage[ACCEL == RT_ACCEL_FLAT_D ? kStageFlat : kStageOct];
  const size_t gl = (size_t)blockIdx.x * 64 + (size_t)lane;
  Stack stk;
  stk.idx = (uint32_t*)s_stack;
  stk.tt = (float*)s_stack + kLdsStack * 64;
  stk.spill = p.spill + gl;
  stk.stride = gridDim.x * 64u;
  stk.lane = lane;
  stk.sp = 0;
  WaveCtx w;
  w.stk2 = s_stack;
  w.stkm = (uint64_t*)(s_stack + 2 * kStack2);
  w.stage = s_stage;
  w.lane = lane;
  // Work item = (tile t, sample s): the four samples of a tile run on four
  // waves, so a tile of long mirror paths (C2: the worst tile cost 7.7x a
  // balanced schedule's whole frame, tools/tile_cost.py) is no longer one
  // wave's serial critical path.  Items come in 8 streams, stream x = the
  // tiles t = x (mod 8) in scanline order, 4 items each: workgroup b (on XCD
  // b mod 8, the dispatcher's round robin) pulls from stream b mod 8, so a
  // tile's samples share one XCD's L2, all XCDs work on the same few tile
  // rows (their geometry stays in the Infinity Cache), and the item counters'
  // atomic traffic is split 8 ways; a drained stream's waves move on to the
  // next.  Each item writes its lanes' deepest hit records.  With camera
  // candidate lists the tiles come longest-first (rt_cand_order): a tile's
  // list length predicts its cost, and the heavy tiles -- the horizon's
  // grazing rays, up to 20x the mean on C5 -- no longer finish the kernel.
  const uint32_t nt = (uint32_t)p.ntiles_local;
  const uint32_t home = (uint32_t)blockIdx.x & 7u;
  uint32_t probe = 0;
  bool first = true;
  unsigned long long wave_cost = 0;  // lane 0: this wave's item clocks (p.item_cost)
  // Items of the heavy tiles (the front of the work order) run at raised
  // wave priority: with 5 waves per SIMD a long mirror path otherwise shares
  // its SIMD's issue slots to the end and becomes the rank's critical path.
  const uint32_t n_heavy = p.n_heavy ? uni(*p.n_heavy) : 0u;
  for (;;) {
    const uint32_t x = (home + probe) & 7u;
    const uint32_t nx = nt > x ? (nt - x + 7u) / 8u : 0u;  // tiles of stream x
    // the first (gridDim.x - x + 7) / 8 items of stream x go one to each of
    // its home waves without an atomic (a small frame's few thousand waves
    // would otherwise queue on 8 counters), the rest through its counter
    uint32_t q = 0;
    if (first) {
      q = (uint32_t)blockIdx.x >> 3;
      first = false;
    } else {
      if (lane == 0) q = atomicAdd(p.tile_counter + 32u * x, 1u);
      q = uni(q) + (gridDim.x - x + 7u) / 8u;
    }
    if (q >= 4u * nx) {
      if (++probe == 8u) break;  // every stream drained: the wave exits
      continue;
    }
    const uint32_t pos = 8u * (q >> 2) + x;  // the tile's place in the work order
    const uint32_t u = 4u * (p.tile_order ? p.tile_order[pos] : pos) + (q & 3u);  // item 4t + s
    const bool prio = RT_HEAVY_PRIO && pos < n_heavy;
    if (prio) __builtin_amdgcn_s_setprio(3);
    const unsigned long long c0 = (COUNT || p.item_cost) ? __builtin_readcyclecounter() : 0ull;
    const uint32_t ph0[3] = {wc.cy_cam, wc.cy_cand, wc.cy_sec};
    wc.sec_lane_nodes = wc.sec_lane_tris = 0;
    const uint32_t t = u >> 2;
    const int smp = (int)(u & 3u);
    f3 point, dir;
    const bool valid = camera_sample(p, t, smp, lane, point, dir);
    if (smp == 0) wc.pixels += (uint32_t)__popcll(__ballot(valid));
    p.last[(size_t)u * 64 + lane] =
        trace_path<ACCEL, COUNT, POL>(p, valid, point, dir, x, stk, w, wc, t, 0, 1.0f, RT_NO_REC);
    if (prio) __builtin_amdgcn_s_setprio(0);
    if (p.item_cost && lane == 0) {  // the next frame's work order (rt_cand_order)
      const unsigned long long cy = __builtin_readcyclecounter() - c0;
      p.item_cost[u] = cy < 0xffffffffull ? (uint32_t)cy : 0xffffffffu;
      wave_cost += cy;
    }
    if (COUNT && p.tile_cycles && lane == 0) {
      // [0] the item's clocks, [1..3] its phase clocks (camera walk, camera
      // candidates, secondary walks), planes of 4 * ntiles_local items
      const size_t items = 4 * (size_t)p.ntiles_local;
      const uint32_t ph1[3] = {wc.cy_cam, wc.cy_cand, wc.cy_sec};
      p.tile_cycles[u] = __builtin_readcyclecounter() - c0;
#pragma unroll
      for (int k2 = 0; k2 < 3; k2++) p.tile_cycles[u + (size_t)(k2 + 1) * items] = ph1[k2] - ph0[k2];
      p.tile_cycles[u + 4 * items] = wc.sec_lane_nodes;
      p.tile_cycles[u + 5 * items] = wc.sec_lane_tris;
    }
  }
  if (p.cost_sum && lane == 0 && wave_cost) atomicAdd(p.cost_sum, wave_cost);
  flush_counts(p, wc, lane);
}

// Per-lane LDS stack of the shadow walks only (shade_kernel, default
// policy): (first, info) entries, no staged wave stack.
static constexpr int kLaneStackArea = kLdsStack * 64 * 8 / 16;

// apply_light (cpu/light.c:33-100) of hit record a, in two phases per block
// of 32 lights: first the shadow queries (only the hit point is live across
// the walks), then the Phong terms of the unshadowed lights, summed in the
// file order of the lights as the reference does.
template <int ACCEL, bool COUNT, int POL>
__device__ __forceinline__ col shade_record(const KParams& p, bool valid, size_t a, Stack& s,
                                            WaveCtx& w, WorkCount& wc, uint32_t& lit0) {
  col acc = init_color(0.0f, 0.0f, 0.0f);
  uint32_t pend = 0;  // lights 0..31 whose query was deferred (p.oob)
  for (uint32_t l0 = 0; l0 < p.nlight; l0 += 32) {
    const uint32_t l1 = p.nlight - l0 < 32u ? p.nlight : l0 + 32u;
    uint32_t lit = 0;  // bit k: light l0 + k does not shadow the point
    {
      f3 P{0.0f, 0.0f, 0.0f};
      if (valid) {
        const float4 r0 = p.hit[2 * a];
        P = f3{r0.x, r0.y, r0.z};
      }
      for (uint32_t li = l0; li < l1; li++) {
        const float* L = p.light + RT_LIGHT_FLOATS_D * li;
        const uint32_t type = __float_as_uint(L[0]);
        if (type != 1 && type != 2) continue;
        const f3 lv = f3{L[4], L[5], L[6]};
        const uint64_t c0 = COUNT ? __builtin_readcyclecounter() : 0ull;
        bool df = false;
        // (issuing the first two lights' cell-range loads before either
        // query, through shadow_q's `pre`, measured slower: shade 1.92 ->
        // 2.16 ms on C5, profiles/r04b_shade_pre/)
        // (df by address, the block-0 condition a flag: a pointer chosen per
        // block kept df on the stack, a scratch store per query)
        // (round 5, with the entries one ahead: the next light's cell ranges
        // loaded while this light's entries are scanned, shade 1.85 -> 1.98
        // ms at 7 waves per SIMD, profiles/r07_shade/)
        const bool sh = shadow_q<ACCEL, COUNT, POL>(p, P, shadow_dir(type, lv, P), type, li, valid, s, w, wc,
                                                    &df, nullptr, l0 == 0);
        if (COUNT) {
          const uint32_t dc = (uint32_t)(__builtin_readcyclecounter() - c0);
          wc.cy_shadow += dc;
          if (type == 1) wc.cy_shadow_dir += dc;
        }
        if (df) pend |= 1u << li;
        if (!sh) lit |= 1u << (li - l0);
      }
    }
    if (l0 == 0) lit0 = lit;
    if (valid && pend && l0 == 0) {  // deferred: queued with the lit bits so far
      const uint32_t q = atomicAdd(p.oob_count, 1u);
      if (q < p.oob_cap) p.oob[q] = make_uint4((uint32_t)a, pend, lit & ~pend, 0u);
    }
    if (!valid) continue;
    const float4 r0 = p.hit[2 * a], r1 = p.hit[2 * a + 1];
    const f3 P{r0.x, r0.y, r0.z}, N{r0.w, r1.x, r1.y};
    const float* m = p.mat + RT_MAT_FLOATS_D * (size_t)__float_as_uint(r1.w);
    for (uint32_t li = l0; li < l1; li++) {
      const float* L = p.light + RT_LIGHT_FLOATS_D * li;
      const uint32_t type = __float_as_uint(L[0]);
      const col lc = init_color(L[1], L[2], L[3]);
      if (type == 0)  // AMBIENT
        acc = color_add(acc, color_mul2(lc, init_color(m[0], m[1], m[2])));
      else if ((type == 1 || type == 2) && ((lit >> (li - l0)) & 1u))
        acc = color_add(acc, light_lit(type, lc, f3{L[4], L[5], L[6]}, m, P, N));
    }
  }
  return acc;
}

// shade_kernel: hit records in chunks of 64 from RT_HIT_REGIONS streams
// (workgroup b drains region b mod 8, then steals), every lane one record:
// cpu/light.c:33-100 with the shadow queries of cpu/light.c:24-31, then the
// term color_mul(local, coef) of cpu/raytracer.c:30.
template <int ACCEL, bool COUNT, int POL>
__global__ __launch_bounds__(64, ACCEL == RT_ACCEL_FLAT_D ? RT_FLAT_SHADE_MIN_WAVES
                                : ((POL == RT_POLICY_STAGED || POL == RT_POLICY_DIR_STAGED) ? RT_STAGED_SHADE_MIN_WAVES
                                                                                              : RT_SHADE_MIN_WAVES)) void shade_kernel(KParams p) {
  const int lane = threadIdx.x & 63;
  WorkCount wc = {};
  constexpr bool kStaged = POL == RT_POLICY_STAGED || POL == RT_POLICY_DIR_STAGED;
  __shared__ float4 s_stack[ACCEL == RT_ACCEL_FLAT_D ? 1 : (kStaged ? kStackArea : kLaneStackArea)];
  __shared__ float4 s_stage[ACCEL == RT_ACCEL_FLAT_D ? kStageFlat : (kStaged ? kStageOct : 1)];
  const size_t gl = (size_t)blockIdx.x * 64 + (size_t)lane;
  Stack stk;
  stk.idx = (uint32_t*)s_stack;
  stk.tt = (float*)s_stack + kLdsStack * 64;
  stk.spill = p.spill + gl;
  stk.stride = gridDim.x * 64u;
  stk.lane = lane;
  stk.sp = 0;
  WaveCtx w;
  w.stk2 = s_stack;
  w.stkm = (uint64_t*)(s_stack + 2 * kStack2);
  w.stage = s_stage;
  w.lane = lane;
  const uint32_t home = (uint32_t)blockIdx.x & 7u;
  uint32_t probe = 0;
  bool first_chunk = true;
  for (;;) {
    const uint32_t x = (home + probe) & 7u;
    const uint32_t hc = p.hit_count[32u * x];
    const uint32_t n = hc < p.hit_cap ? hc : p.hit_cap;
    const uint32_t stride = p.shade_stride > 1u ? p.shade_stride : 1u;  // verification only
    const uint32_t first = p.shade_first;
    const uint32_t ns = n > first ? (n - first + stride - 1u) / stride : 0u;  // records shaded
    // first chunk of each home wave without an atomic (as trace_kernel)
    uint32_t q = 0;
    if (first_chunk) {
      q = (uint32_t)blockIdx.x >> 3;
      first_chunk = false;
    } else {
      if (lane == 0) q = atomicAdd(p.shade_counter + 32u * x, 1u);
      q = uni(q) + (gridDim.x - x + 7u) / 8u;
    }
    if (q >= (ns + 63u) / 64u) {
      if (++probe == 8u) break;
      continue;
    }
    const uint32_t k = q * 64u + (uint32_t)lane;
    const bool valid = k < ns;
    const size_t a = (size_t)x * p.hit_cap + (size_t)k * stride + first;
    uint32_t lit = 0;
    const col local = shade_record<ACCEL, COUNT, POL>(p, valid, a, stk, w, wc, lit);
    if (valid) {
      const col tm = color_mul(local, p.hit[2 * a + 1].z);  // coef
      p.hit_term[a] = make_float4(tm.r, tm.g, tm.b, 0.0f);
      if (p.hit_lit) p.hit_lit[a] = lit;
    }
  }
  flush_counts(p, wc, lane, true);
}

// Exact-shadow mode, deferred queries (shade_kernel, p.oob): entry e's
// pending lights' shadow rays from its record's hit point by brute force over
// the nprim prim-order records (cpu/hit.c:93-109), a workgroup per
// (entry, chunk of kFixChunk records); hits ORed into the entry's w.
static constexpr uint32_t kFixChunk = 16384;
static constexpr uint32_t kFixBatch = 64;  // oob_fix_batch_kernel's queries
// (entry, pending light) queries of the deferred entries, kFixBatch + 1 when
// there are more than oob_fix_batch_kernel holds
__device__ __forceinline__ uint32_t oob_queries(const KParams& p, uint32_t n) {
  if (n > kFixBatch) return kFixBatch + 1;
  uint32_t m = 0;
  for (uint32_t e = 0; e < n; e++) m += (uint32_t)__popc(p.oob[e].y & (p.nlight >= 32 ? 0xffffffffu : (1u << p.nlight) - 1u));
  return m;
}
__global__ __launch_bounds__(256) void oob_fix_kernel(KParams p, uint32_t nprim) {
  __shared__ uint32_t bits, skip, nqs;
  const uint32_t n = min(*p.oob_count, p.oob_cap);
  if (threadIdx.x == 0) nqs = oob_queries(p, n);
  __syncthreads();
  if (nqs <= kFixBatch) return;  // oob_fix_batch_kernel decided them
  const uint32_t chunks = (nprim + kFixChunk - 1) / kFixChunk;
  for (uint64_t item = blockIdx.x; item < (uint64_t)n * chunks; item += gridDim.x) {
    const uint32_t e = (uint32_t)(item / chunks), c = (uint32_t)(item % chunks);
    const uint4 q = p.oob[e];
    if (threadIdx.x == 0) {  // one decision for the block: every lane reaches the barriers
      bits = 0;
      skip = (__atomic_load_n(&p.oob[e].w, __ATOMIC_RELAXED) & q.y) == q.y;  // all already shadowed
    }
    __syncthreads();
    if (skip) {
      __syncthreads();
      continue;
    }
    const float4 r0 = p.hit[2 * (size_t)q.x];
    const f3 P{r0.x, r0.y, r0.z};
    uint32_t mine = 0, risk = 0;
    for (uint32_t li = 0; li < 32 && li < p.nlight; li++) {
      if (!((q.y >> li) & 1u)) continue;
      const float* L = p.light + RT_LIGHT_FLOATS_D * li;
      const uint32_t type = __float_as_uint(L[0]);
      const Ray r = make_ray(p, P, shadow_dir(type, f3{L[4], L[5], L[6]}, P), p.eps_rel);
      bool h = false;
      const uint32_t end = min(nprim, (c + 1) * kFixChunk);
      for (uint32_t k = c * kFixChunk + threadIdx.x; k < end && !h; k += blockDim.x) {
        const float4* t = p.tri_prim + 3 * (size_t)k;
        h = any_hit_rec(r, t[0], t[1], t[2], risk);
      }
      if (h) mine |= 1u << li;
    }
    if (mine) atomicOr(&bits, mine);
    if (risk) atomicAdd(p.stats + 18, 1ull);  // shadow_zero_risk
    __syncthreads();
    if (threadIdx.x == 0 && bits) atomicOr(&p.oob[e].w, bits);
    __syncthreads();
  }
}

// The same decisions for the usual handful of deferred queries (C5: 4
// records, 8 queries per frame) in one pass over the records: every query
// -- (entry, pending light) -- is set up once per workgroup in LDS, and each
// thread streams its records once, testing each against every query.  The
// per-entry launch above reads all nprim records (480 MB on C5) once per
// query: 0.65 ms of HBM traffic for 8 queries.  At most kFixBatch queries.
struct FixQuery {
  Ray r;
  uint32_t e, li;
};
__global__ __launch_bounds__(256) void oob_fix_batch_kernel(KParams p, uint32_t nprim) {
  __shared__ FixQuery qs[kFixBatch];
  __shared__ uint32_t nq;
  const uint32_t n = min(*p.oob_count, p.oob_cap);
  if (threadIdx.x == 0) {
    uint32_t m = 0;
    const bool batch = oob_queries(p, n) <= kFixBatch;
    for (uint32_t e = 0; e < n && batch; e++) {
      const uint4 q = p.oob[e];
      const float4 r0 = p.hit[2 * (size_t)q.x];
      const f3 P{r0.x, r0.y, r0.z};
      for (uint32_t li = 0; li < 32 && li < p.nlight; li++) {
        if (!((q.y >> li) & 1u) || m >= kFixBatch) continue;
        const float* L = p.light + RT_LIGHT_FLOATS_D * li;
        const uint32_t type = __float_as_uint(L[0]);
        qs[m].r = make_ray(p, P, shadow_dir(type, f3{L[4], L[5], L[6]}, P), p.eps_rel);
        qs[m].e = e;
        qs[m].li = li;
        m++;
      }
    }
    nq = m;
  }
  __syncthreads();
  const uint32_t m = nq;
  uint32_t risk = 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nprim; k += gridDim.x * blockDim.x) {
    const float4* t = p.tri_prim + 3 * (size_t)k;
    const float4 a0 = t[0], a1 = t[1], a2 = t[2];
    for (uint32_t j = 0; j < m; j++) {
      const FixQuery& q = qs[j];
      if (any_hit_rec(q.r, a0, a1, a2, risk)) atomicOr(&p.oob[q.e].w, 1u << q.li);
    }
  }
  if (risk) atomicAdd(p.stats + 18, 1ull);  // shadow_zero_risk
}

// ... then each entry's record shaded again with the decided lights
// (cpu/light.c:33-100, cpu/raytracer.c:30), as shade_kernel would have.
__global__ __launch_bounds__(64) void oob_reshade_kernel(KParams p) {
  const uint32_t n = min(*p.oob_count, p.oob_cap);
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint4 q = p.oob[e];
    const size_t a = q.x;
    const uint32_t lit0 = q.z | (q.y & ~q.w);
    const float4 r0 = p.hit[2 * a], r1 = p.hit[2 * a + 1];
    const f3 P{r0.x, r0.y, r0.z}, N{r0.w, r1.x, r1.y};
    const float* m = p.mat + RT_MAT_FLOATS_D * (size_t)__float_as_uint(r1.w);
    col acc = init_color(0.0f, 0.0f, 0.0f);
    for (uint32_t li = 0; li < p.nlight && li < 32; li++) {
      const float* L = p.light + RT_LIGHT_FLOATS_D * li;
      const uint32_t type = __float_as_uint(L[0]);
      const col lc = init_color(L[1], L[2], L[3]);
      if (type == 0)  // AMBIENT
        acc = color_add(acc, color_mul2(lc, init_color(m[0], m[1], m[2])));
      else if ((type == 1 || type == 2) && ((lit0 >> li) & 1u))
        acc = color_add(acc, light_lit(type, lc, f3{L[4], L[5], L[6]}, m, P, N));
    }
    const col tm = color_mul(acc, r1.z);  // coef
    p.hit_term[a] = make_float4(tm.r, tm.g, tm.b, 0.0f);
    if (p.hit_lit) p.hit_lit[a] = lit0;
  }
}

// Shadow-query probe (tests, tools): the shadow ray of light li from each
// given origin (cpu/light.c:53,78), answered through the light's buffer
// (brute = 0) or by brute force over the nprim prim-order records (brute = 1,
// cpu/hit.c:93-109).  One thread per origin; out[i] = shadowed.
__global__ __launch_bounds__(256) void probe_shadow_kernel(KParams p, const float* __restrict__ org, uint32_t n,
                                                           uint32_t li, uint32_t nprim, int brute,
                                                           uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* L = p.light + RT_LIGHT_FLOATS_D * li;
  const uint32_t type = __float_as_uint(L[0]);
  const f3 o{org[3 * (size_t)i], org[3 * (size_t)i + 1], org[3 * (size_t)i + 2]};
  const Ray r = make_ray(p, o, shadow_dir(type, f3{L[4], L[5], L[6]}, o), p.eps_rel);
  bool hit = false;
  if (brute) {
    uint32_t risk = 0;
    for (uint32_t k = 0; k < nprim && !hit; k++) {
      const float4* t = p.tri_prim + 3 * (size_t)k;
      hit = any_hit_rec(r, t[0], t[1], t[2], risk);
    }
  } else {
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    hit = lbuf_any<false>(p, p.lbuf[li], r, lc);
  }
  out[i] = hit ? 1u : 0u;
}

// Closest-hit probe (tests, tools): ray i = (org[i], dir[i]) as a
// reflection ray queries it -- the per-lane octree walk at the secondary
// rays' culling slack (closest_q at depth > 0, default policy), or brute force
// over the nprim prim-order records (cpu/hit.c:72-91) -- out[2 i] = the
// winner's prim (~0: none), out[2 i + 1] = its new_dist bits.  One-wave
// workgroups: the walk's LDS stack is per wave, its spill area per lane.
__global__ __launch_bounds__(64) void probe_closest_kernel(KParams p, const float* __restrict__ org,
                                                           const float* __restrict__ dir, uint32_t n,
                                                           uint32_t nprim, int brute, uint32_t* __restrict__ out) {
  __shared__ float4 s_stack[kLaneStackArea];
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 64u + (uint32_t)lane;
  Stack stk;
  stk.idx = (uint32_t*)s_stack;
  stk.tt = (float*)s_stack + kLdsStack * 64;
  stk.spill = p.spill + (size_t)blockIdx.x * 64 + (size_t)lane;
  stk.stride = gridDim.x * 64u;
  stk.lane = lane;
  stk.sp = 0;
  const bool act = i < n;
  f3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f};
  if (act) {
    o = f3{org[3 * (size_t)i], org[3 * (size_t)i + 1], org[3 * (size_t)i + 2]};
    d = f3{dir[3 * (size_t)i], dir[3 * (size_t)i + 1], dir[3 * (size_t)i + 2]};
  }
  const Ray r = make_ray(p, o, d, p.eps_rel);
  Best b;
  b.dist = __builtin_inff();
  b.t_cut = __builtin_inff();
  b.prim = 0xffffffffu;
  b.obj = 0;
  b.u = b.v = 0.0f;
  b.t = 0.0f;
  if (brute) {
    if (act)
      for (uint32_t k = 0; k < nprim; k++) {
        const float4* t = p.tri_prim + 3 * (size_t)k;
        consider(r, t[0], t[1], t[2], b);
      }
  } else {
    LaneCount lc = {0, 0, 0, 0, 0, 0, 0, 0};
    if (act) {
      if (p.node_rf)  // the exact reflection mode's walk (rt_hip_set_exact_reflections)
        oct_closest_rf<false>(p, r, b, stk, lc);
      else
        oct_closest<false>(p, r, b, stk, lc);
    }
    if (act && lc.unproven) out[2 * (size_t)i + 1] = 0x7fc00001u;  // (never: |d| past RT_RF_DLMAX)
  }
  if (act) {
    out[2 * (size_t)i] = b.dist == __builtin_inff() ? 0xffffffffu : b.prim;
    out[2 * (size_t)i + 1] = __float_as_uint(b.dist);
  }
}

// A pixel's four samples (trace_kernel items 4t..4t+3): each sample's path
// terms summed deepest-first, acc = color_add(reflected, term)
// (cpu/raytracer.c:29-30), then acc = color_add(acc, color_mul(s, 0.25)) over
// the samples (i,j), (i,j+.5), (i+.5,j), (i+.5,j+.5) (cpu/raytracer.c:55-68);
// pixels outside the framebuffer's even-sized area are 0.  One thread per
// pixel of the rank's tile buffer.
__global__ __launch_bounds__(256) void fold_kernel(KParams p) {
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx == 0 && p.frame_check) {  // every earlier launch of the frame has ended (same stream)
    uint32_t f = 0;
    for (int x = 0; x < RT_HIT_REGIONS; x++)
      if (p.hit_count[32 * x] > p.hit_cap) f |= RT_FRAME_HITBUF;
    unsigned long long s[RT_NSTATS] = {};
    for (int set = 0; set < RT_STAT_SETS; set++)
      for (int k = 0; k < RT_NSTATS; k++) s[k] += p.stats[set * RT_STAT_STRIDE + k];
    if (s[5]) f |= RT_FRAME_DEPTH;
    if (s[6] || s[18]) f |= RT_FRAME_ZERO;
    if (s[21] || s[22] || (p.oob_count && *p.oob_count > p.oob_cap)) f |= RT_FRAME_UNPROVEN;
    if (p.list_flag && *p.list_flag) f |= RT_FRAME_LISTS;
    atomicOr(p.frame_check, (unsigned long long)f);
    atomicAdd(p.frame_check + 1, 1ull);
    atomicAdd(p.frame_check + 2, s[0]);
    atomicAdd(p.frame_check + 3, s[1]);
  }
  if (idx >= (uint32_t)p.ntiles_local * 64u) return;
  const uint32_t t = idx >> 6, lane = idx & 63u;
  int pr, pc;
  tile_pixel(p, t, (int)lane, pr, pc);
  const int ii = p.W - pc, jj = p.H - pr;
  const bool valid = pr < p.H && pc < p.W && ii >= 1 && ii <= 2 * (p.W / 2) && jj >= 1 &&
                     jj <= 2 * (p.H / 2);
  col acc = init_color(0.0f, 0.0f, 0.0f);
  for (int smp = 0; smp < 4; smp++) {
    col sc = init_color(0.0f, 0.0f, 0.0f);
    uint32_t r = p.last[((size_t)t * 4 + (size_t)smp) * 64 + lane];
    while (r != RT_NO_REC && (r >> 3) < p.hit_cap) {
      const size_t a = rec_addr(p, r);
      const float4 tm = p.hit_term[a];
      sc = color_add(sc, col{tm.x, tm.y, tm.z});
      r = p.hit_prev[a];
    }
    acc = color_add(acc, color_mul(sc, 0.25f));
  }
  if (!valid) acc = col{0.0f, 0.0f, 0.0f};
  float* o = p.out + (size_t)idx * 3;
  o[0] = acc.r;
  o[1] = acc.g;
  o[2] = acc.b;
}

// ------------------------------------------------ gpu/rt compatibility mode
// The reference's GPU renderer's own output semantics (SURVEY.md §8(f) item
// 4): the frame rendered at 3x the size with one ray per high-resolution
// pixel (gpu/rt.cpp:72-83, gpu/raytracer.cu:88-125), colours as saturating
// uint8 (gpu/colors.cu:3-49), reflections accumulated front to back for at
// most 11 queries (gpu/raytracer.cu:31-46,113-120), the light model of
// gpu/light.cu (cpu/light.c's, in uint8 colours), then a 3x3 box downscale
// (gpu/raytracer.cu:48-85).  Geometry, closest hit and shadow queries are
// cpu/rt's (gpu/hit.cu:4-123 restates cpu/hit.c) and run through the same
// walks.  uint8 channels are held as integral floats.

// init_color (gpu/colors.cu:3-20): x*255 clamped, then the (unsigned char)
// conversion truncates (a NaN converts to 0)
__device__ __forceinline__ float chan8(float x) {
  float y = x * 255.0f;
  if (y > 255.0f) y = 255.0f;
  if (y < 0.0f) y = 0.0f;
  y = __builtin_truncf(y);
  return y == y ? y : 0.0f;
}
__device__ __forceinline__ col init8(float r, float g, float b) { return col{chan8(r), chan8(g), chan8(b)}; }
// color_add: integer sum, saturated at 255
__device__ __forceinline__ col add8(col a, col b) {
  return col{fminf(a.r + b.r, 255.0f), fminf(a.g + b.g, 255.0f), fminf(a.b + b.b, 255.0f)};
}
// color_mul: init_color(float(a.r) / 255 * coef, ...)
__device__ __forceinline__ col mul8(col a, float coef) {
  return init8(a.r / 255.0f * coef, a.g / 255.0f * coef, a.b / 255.0f * coef);
}
// color_mults: init_color((a.r / 255) * (b.r / 255), ...)
__device__ __forceinline__ col mults8(col a, col b) {
  return init8((a.r / 255.0f) * (b.r / 255.0f), (a.g / 255.0f) * (b.g / 255.0f),
               (a.b / 255.0f) * (b.b / 255.0f));
}

// gpu/light.cu:12-28 (pow(cufmax(R.V, 0), ns): the f32 pow, taken as the
// correctly rounded f64 pow rounded to float, as in cpu mode)
__device__ __forceinline__ col specular8(col tmp, f3 inc_o, f3 inc_d, f3 P, f3 N, const float* m) {
  col k = init8(m[6], m[7], m[8]);
  f3 V = sub(inc_o, P);
  f3 R = sub(inc_d, scale(N, 2.0f * dot(N, inc_d)));
  R = normalize(R);
  V = normalize(V);
  float ls = spec_pow((double)dot(R, V), (double)m[9]);
  k = mul8(k, ls);
  return add8(tmp, k);
}

// gpu/light.cu:66-118, the lit branch of a directional (1) or point (2) light
__device__ __forceinline__ col light_lit8(uint32_t type, col lc, f3 lv, const float* m, f3 P, f3 N) {
  if (type == 1) {
    col tmp = mults8(lc, init8(m[3], m[4], m[5]));
    tmp = mul8(tmp, dot(scale(lv, -1.0f), N));
    return specular8(tmp, add(P, scale(lv, -10.0f)), lv, P, N, m);
  }
  f3 to_l = sub(lv, P);
  f3 Lp = scale(lv, -1.0f);
  f3 Nf = N;
  if (dot(Lp, Nf) < 0.0f) Nf = scale(Nf, -1.0f);
  float dist = length(sub(lv, P));
  col tmp = mults8(lc, init8(m[3], m[4], m[5]));
  tmp = mul8(tmp, dot(Lp, Nf) * 1.0f / dist);
  return specular8(tmp, add(P, scale(to_l, -10.0f)), to_l, P, N, m);
}

// gpu/light.cu:46-126 for the lanes with hit; converged shadow queries
template <int ACCEL, int POL>
__device__ col apply_light8(const KParams& p, bool hit, const float* m, f3 P, f3 N, Stack& s,
                            WaveCtx& w, WorkCount& wc) {
  col acc = col{0.0f, 0.0f, 0.0f};
  for (uint32_t li = 0; li < p.nlight; li++) {
    const float* L = p.light + RT_LIGHT_FLOATS_D * li;
    uint32_t type = __float_as_uint(L[0]);
    col lc = init8(L[1], L[2], L[3]);
    f3 lv = f3{L[4], L[5], L[6]};
    if (type == 0) {
      if (hit) acc = add8(acc, mults8(lc, init8(m[0], m[1], m[2])));
    } else if (type == 1 || type == 2) {
      bool sh = shadow_q<ACCEL, false, POL>(p, P, shadow_dir(type, lv, P), type, li, hit, s, w, wc);
      if (hit && !sh) acc = add8(acc, light_lit8(type, lc, lv, m, P, N));
    }
  }
  return acc;
}

// One high-resolution pixel per lane, one 8x8 tile of the 3W x 3H image per
// wave (persistent waves, one tile counter).  p.W, p.H, p.u/v/C/pos: the
// upscaled frame; p.out: 3W x 3H packed RGBA8, row-major (row = py).
template <int ACCEL, int POL>
__global__ __launch_bounds__(64, RT_MIN_WAVES) void compat_kernel(KParams p) {
  const int lane = threadIdx.x & 63;
  WorkCount wc = {};
  __shared__ float4 s_stack[ACCEL == RT_ACCEL_FLAT_D ? 1 : kStackArea];
  __shared__ float4 s_stage[ACCEL == RT_ACCEL_FLAT_D ? kStageFlat : kStageOct];
  const size_t gl = (size_t)blockIdx.x * 64 + (size_t)lane;
  Stack stk;
  stk.idx = (uint32_t*)s_stack;
  stk.tt = (float*)s_stack + kLdsStack * 64;
  stk.spill = p.spill + gl;
  stk.stride = gridDim.x * 64u;
  stk.lane = lane;
  stk.sp = 0;
  WaveCtx w;
  w.stk2 = s_stack;
  w.stkm = (uint64_t*)(s_stack + 2 * kStack2);
  w.stage = s_stage;
  w.lane = lane;
  uint32_t* img = (uint32_t*)p.out;
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(p.tile_counter, 1u);
    t = uni(t);
    if (t >= (uint32_t)p.ntiles_total) break;
    const int ty = (int)(t / (uint32_t)p.tiles_x), tx = (int)(t % (uint32_t)p.tiles_x);
    const int py = ty * 8 + (lane >> 3), px = tx * 8 + (lane & 7);
    const bool valid = py < p.H && px < p.W;
    wc.pixels += (uint32_t)__popcll(__ballot(valid));
    // gpu/raytracer.cu:97-103
    f3 o = add(add(p.C, scale(p.u, (float)(px - p.W / 2))), scale(p.v, (float)(py - p.H / 2)));
    f3 d = normalize(sub(p.pos, o));
    col color = col{0.0f, 0.0f, 0.0f};
    float nr = 1.0f;
    int max_bounce = 10;
    bool alive = valid;
    for (int depth = 0;; depth++) {  // gpu/raytracer.cu:113-120
      const uint64_t am = __ballot(alive);
      if (am == 0) break;
      wc.closest += (uint32_t)__popcll(am);
      Ray r = make_ray(p, o, d, depth == 0 ? p.eps_rel_cam : p.eps_rel);
      Best b;
      b.dist = __builtin_inff();
      b.t_cut = __builtin_inff();
      b.prim = 0xffffffffu;
      b.obj = 0;
      b.u = b.v = 0.0f;
      b.t = 0.0f;
      closest_q<ACCEL, false, POL>(p, r, alive, depth, b, stk, w, wc);
      // the camera rays' candidate lists (rt_hip_render_compat builds them for
      // this frame's sample model): the same exactness as cpu mode
      if (ACCEL != RT_ACCEL_FLAT_D && depth == 0) cand_closest<false>(p, r, alive, t, b, w, wc);
      bool hit = alive && b.dist != __builtin_inff();
      f3 N = f3{0.0f, 0.0f, 0.0f};
      wc.hits += (uint32_t)__popcll(__ballot(hit));
      bool zero = false;
      if (hit) {
        const float* nm = p.nrm + 9 * (size_t)b.prim;
        float w0 = 1.0f - b.u - b.v;
        N = add(add(scale(ld3(nm), w0), scale(ld3(nm + 3), b.u)), scale(ld3(nm + 6), b.v));
        zero = is_zero(N);
      }
      wc.zero_normal += (uint32_t)__popcll(__ballot(zero));
      hit = hit && !zero;
      const float* m = p.mat + RT_MAT_FLOATS_D * (hit ? b.obj : 0u);
      f3 P = hit ? hit_point(r, b.t) : o;
      col local = apply_light8<ACCEL, POL>(p, hit, m, P, N, stk, w, wc);  // trace(), :31-46
      if (alive) {
        if (!hit) local = col{0.0f, 0.0f, 0.0f};
        const float loc_nr = hit ? m[10] : 0.0f;
        if (hit && m[10] > 0.0f) {
          d = bounce_dir(d, N);
          o = P;
        }
        color = add8(color, mul8(local, nr));
        nr *= loc_nr;
        alive = nr > 0.01f && max_bounce-- > 0;
      }
    }
    if (valid)
      img[(size_t)py * (size_t)p.W + (size_t)px] = (uint32_t)color.r | ((uint32_t)color.g << 8) |
                                                   ((uint32_t)color.b << 16) | 0xff000000u;
  }
  flush_counts(p, wc, lane);
}

// gpu/raytracer.cu:48-85: output pixel (row R, column c) of the W x H image
// (PNG order: gpu/rt.cpp writes buffer rows top down) is the 3x3 block of
// high-resolution pixels px = 3 (W - 1 - c) .., py = 3 (H - 1 - R) .., summed
// as floats, / (255 * 9), through init_color.
__global__ __launch_bounds__(256) void downscale_kernel(const uint32_t* __restrict__ hi,
                                                        uint32_t* __restrict__ lo, int W, int H) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= W * H) return;
  const int R = idx / W, c = idx % W;
  const int px = W - 1 - c, py = H - 1 - R, HW = 3 * W;
  float r = 0.0f, g = 0.0f, b = 0.0f;
  for (int hy = 3 * py; hy < 3 * py + 3; ++hy)
    for (int hx = 3 * px; hx < 3 * px + 3; ++hx) {
      const uint32_t q = hi[(size_t)hy * HW + hx];
      r += (float)(q & 0xffu);
      g += (float)((q >> 8) & 0xffu);
      b += (float)((q >> 16) & 0xffu);
    }
  const float ali2 = 255.0f * 3.0f * 3.0f;
  col e = init8(r / ali2, g / ali2, b / ali2);
  lo[idx] = (uint32_t)e.r | ((uint32_t)e.g << 8) | ((uint32_t)e.b << 16) | 0xff000000u;
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
  uint32_t rank;
  const int tb = rt_block_side(nranks);
  const uint32_t local = rt_tile_local(col >> 3, row >> 3, (uint32_t)nranks,
                                       (uint32_t)rt_blocks_x(tiles_x, tb), (uint32_t)tb, &rank);
  int lane = ((row & 7) << 3) | (col & 7);
  const float* src = tiles + (((size_t)rank * tiles_per_rank + local) * 64 + lane) * 3;
  rgb[3 * idx + 0] = src[0];
  rgb[3 * idx + 1] = src[1];
  rgb[3 * idx + 2] = src[2];
  (void)ntiles;
}

}  // namespace rt

// ---------------------------------------------------------------- launchers
// One instantiation per (kernel, accel, work counting, policy); the default
// policy's kernels have no policy switch inside.  The work-counting pass and
// the test policies are separate kernels, so they cannot slow the default
// ones down.
// The instantiation of (kernel, accel, counting, policy).  Policies only
// differ in the walks they use: trace has no shadow queries (policy 3 =
// default there), shade has no closest-hit queries (policy 1 = default).
template <bool TRACE>
static const void* kernel_of(int accel, int count_work, int policy);

template <bool TRACE>
static const void* kernel_of(int accel, int count_work, int policy) {
  using namespace rt;
  if (accel == RT_ACCEL_FLAT_D) {
    if (TRACE)
      return count_work ? (const void*)trace_kernel<RT_ACCEL_FLAT_D, true, 0>
                        : (const void*)trace_kernel<RT_ACCEL_FLAT_D, false, 0>;
    return count_work ? (const void*)shade_kernel<RT_ACCEL_FLAT_D, true, 0>
                      : (const void*)shade_kernel<RT_ACCEL_FLAT_D, false, 0>;
  }
  if (TRACE) {
    if (policy == RT_POLICY_EXACT_REFL)
      return count_work ? (const void*)trace_kernel<RT_ACCEL_OCTREE_D, true, RT_POLICY_EXACT_REFL>
                        : (const void*)trace_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_EXACT_REFL>;
    if (policy == RT_POLICY_LANE) return (const void*)trace_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_LANE>;
    if (policy == RT_POLICY_STAGED)
      return (const void*)trace_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_STAGED>;
    return count_work ? (const void*)trace_kernel<RT_ACCEL_OCTREE_D, true, RT_POLICY_DEFAULT>
                      : (const void*)trace_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_DEFAULT>;
  }
  if (policy == RT_POLICY_STAGED) return (const void*)shade_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_STAGED>;
  if (policy == RT_POLICY_LBUF)
    return count_work ? (const void*)shade_kernel<RT_ACCEL_OCTREE_D, true, RT_POLICY_LBUF>
                      : (const void*)shade_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_LBUF>;
  if (policy == RT_POLICY_DIR_STAGED)
    return (const void*)shade_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_DIR_STAGED>;
  return count_work ? (const void*)shade_kernel<RT_ACCEL_OCTREE_D, true, RT_POLICY_DEFAULT>
                    : (const void*)shade_kernel<RT_ACCEL_OCTREE_D, false, RT_POLICY_DEFAULT>;
}

// Persistent grid of a kernel: as many one-wave workgroups as the kernel's
// registers and LDS let every CU hold (the occupancy API), so every SIMD is
// filled and no workgroup waits for a slot.
extern "C" hipError_t rt_render_grid(int trace, int accel, int count_work, int policy, int cus,
                                     int* grid) {
  const void* k = trace ? kernel_of<true>(accel, count_work, policy)
                        : kernel_of<false>(accel, count_work, policy);
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64, 0);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 32) per_cu = 32;
  *grid = per_cu * cus;
  return hipSuccess;
}

static hipError_t launch_kernel(const void* k, int grid, const KParams* p, hipStream_t stream) {
  void* args[] = {(void*)p};
  return hipLaunchKernel(k, dim3(grid), dim3(64), args, 0, stream);
}

extern "C" hipError_t rt_launch_trace(const KParams* p, int accel, int count_work, int policy,
                                      int grid, hipStream_t stream) {
  return launch_kernel(kernel_of<true>(accel, count_work, policy), grid, p, stream);
}

extern "C" hipError_t rt_launch_shade(const KParams* p, int accel, int count_work, int policy,
                                      int grid, hipStream_t stream) {
  return launch_kernel(kernel_of<false>(accel, count_work, policy), grid, p, stream);
}

extern "C" hipError_t rt_launch_shade_fixup(const KParams* p, uint32_t nprim, hipStream_t stream) {
  if (!p->oob) return hipGetLastError();
  // the batch pass holds kFixBatch queries; the per-entry pass any number
  // (the count is on the device: both are launched, each a no-op for the
  // other's case)
  hipLaunchKernelGGL(rt::oob_fix_batch_kernel, dim3(2048), dim3(256), 0, stream, *p, nprim);
  hipLaunchKernelGGL(rt::oob_fix_kernel, dim3(4096), dim3(256), 0, stream, *p, nprim);
  hipLaunchKernelGGL(rt::oob_reshade_kernel, dim3(64), dim3(64), 0, stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_launch_probe_shadow(const KParams* p, const float* org, uint32_t n, uint32_t li,
                                             uint32_t nprim, int brute, uint32_t* out, hipStream_t stream) {
  if (n == 0) return hipGetLastError();
  hipLaunchKernelGGL(rt::probe_shadow_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, *p, org, n, li, nprim,
                     brute, out);
  return hipGetLastError();
}

extern "C" hipError_t rt_launch_probe_closest(const KParams* p, const float* org, const float* dir, uint32_t n,
                                              uint32_t nprim, int brute, uint32_t* out, int grid, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t g = (n + 63) / 64;
  if (!brute && g > (uint32_t)grid) return hipErrorInvalidValue;  // the spill area holds `grid` waves
  hipLaunchKernelGGL(rt::probe_closest_kernel, dim3(g), dim3(64), 0, stream, *p, org, dir, n, nprim, brute, out);
  return hipGetLastError();
}

extern "C" hipError_t rt_launch_fold(const KParams* p, hipStream_t stream) {
  const uint32_t n = (uint32_t)p->ntiles_local * 64u;
  if (n == 0) return hipGetLastError();
  hipLaunchKernelGGL(rt::fold_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, *p);
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

extern "C" hipError_t rt_launch_compat(const KParams* p, int accel, int grid, hipStream_t stream) {
  dim3 g(grid), b(64);
  if (accel == RT_ACCEL_FLAT_D)
    hipLaunchKernelGGL((rt::compat_kernel<RT_ACCEL_FLAT_D, 0>), g, b, 0, stream, *p);
  else
    hipLaunchKernelGGL((rt::compat_kernel<RT_ACCEL_OCTREE_D, RT_POLICY_DEFAULT>), g, b, 0, stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_launch_downscale(const uint32_t* hi, uint32_t* lo, int W, int H,
                                          hipStream_t stream) {
  const int n = W * H;
  hipLaunchKernelGGL(rt::downscale_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, hi, lo, W, H);
  return hipGetLastError();
}
