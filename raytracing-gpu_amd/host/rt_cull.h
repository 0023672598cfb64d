/*
 * rt_cull.h -- octree node encoding and the conservative culling arithmetic,
 * shared verbatim by the device traversal (csrc/rt_render.hip) and its host
 * model (host/accel_probe.c), so both make the same keep/cull decision on
 * the same floats (both are built with -ffp-contract=off).
 *
 * Node (2 x float4): lo.xyz, bits(first) | hi.xyz, bits(info)
 *   leaf:     info = RT_NODE_LEAF | record count; first = first record
 *   interior: info = child count | octant mask << 8; first = first child
 *             (children stored contiguously in increasing octant order;
 *             octant bit a set = upper half along axis a)
 *
 * Culling (DESIGN.md "Conservative culling"): a box is grown by a per-ray
 * world-space slack eps that covers the float error of the reference's
 * Moller-Trumbore accept decision (cpu/hit.c:15-33, error ~ |o - v0| ulps),
 * and the slab interval by a relative slack covering the slab arithmetic.
 * A node is pruned only when its (grown) entry distance exceeds the current
 * best new_dist by more than 2 eps.
 */
#ifndef RT_CULL_H
#define RT_CULL_H

#ifdef __HIPCC__
#define RT_CULL_FN __device__ __forceinline__
#else
#include <math.h>
#include <stdint.h>
#define RT_CULL_FN static inline
#endif

#define RT_NODE_LEAF 0x80000000u
#define RT_NODE_COUNT(info) ((info) & 0xffu)
#define RT_NODE_MASK(info) (((info) >> 8) & 0xffu)
#define RT_LEAF_COUNT(info) ((info) & 0x7fffffffu)

/* 2^-21: relative slack of slab entry/exit parameters and of the prune test */
#define RT_CULL_TREL 4.76837158203125e-7f
/* 2^-22 x (|scene centre| + R): rounding of the grown box planes themselves */
#define RT_CULL_PLANE 2.384185791015625e-7f

/* eps_rel = ulps * 2^-24; (dx,dy,dz) = origin - scene centre; cmag =
 * max-norm of the scene centre; R = scene half-extent (max-norm). */
RT_CULL_FN float rt_cull_eps(float eps_rel, float dx, float dy, float dz, float cmag, float R)
{
  float m = fmaxf(fabsf(dx), fmaxf(fabsf(dy), fabsf(dz)));
  return eps_rel * (m + R) + RT_CULL_PLANE * (cmag + R) + 1e-6f;
}

/* Slab test of the ray o + t d against [lo - eps, hi + eps]; inv = 1/d
 * component-wise.  Returns the entry parameter, or +inf when the (slack-
 * widened) interval is empty or lies behind the origin. */
RT_CULL_FN float rt_box_enter(float ox, float oy, float oz, float ix, float iy, float iz,
                              float eps, float lx, float ly, float lz, float hx, float hy,
                              float hz)
{
  float tx0 = (lx - eps - ox) * ix, tx1 = (hx + eps - ox) * ix;
  float ty0 = (ly - eps - oy) * iy, ty1 = (hy + eps - oy) * iy;
  float tz0 = (lz - eps - oz) * iz, tz1 = (hz + eps - oz) * iz;
  float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
  float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  /* NaN (0 * inf on an axis-parallel ray exactly on a slab plane) makes
   * fminf/fmaxf pick the other operand: the axis is then "inside". */
  float s = RT_CULL_TREL * fminf(fmaxf(fabsf(tmin), fabsf(tmax)), 1e30f);
  if (tmax + s < fmaxf(tmin, 0.0f) - s)
    return INFINITY;
  return tmin;
}

/* 1 = the node (entry parameter t_enter) cannot hold a triangle whose
 * new_dist is <= best. */
RT_CULL_FN int rt_prune(float t_enter, float dlen, float best, float eps)
{
  return t_enter * dlen > best + best * RT_CULL_TREL + 2.0f * eps;
}

#endif
