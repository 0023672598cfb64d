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
 * well-conditioned Moller-Trumbore accept decisions (cpu/hit.c:15-33, error
 * ~ |o - v0| ulps) and the rounding of the slab test itself.  A node is
 * pruned only when its (grown) entry distance exceeds the current best
 * new_dist by more than 2 eps.
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

/* Per-ray slab constants: inv = 1/d with zero components clamped to a huge
 * finite value of the same sign (no 0 * inf NaN in the slab products; the
 * slab of an axis the ray is parallel to then reads "inside" or "never"
 * exactly as the geometry says), oh = o + eps, ol = o - eps. */
RT_CULL_FN float rt_inv(float d)
{
  float i = 1.0f / d;
  return fabsf(i) < 1e30f ? i : copysignf(1e30f, d);
}

/* Slab test of the ray o + t d against [lo - eps, hi + eps]:
 * (lo - eps - o) / d is evaluated as fma(lo, 1/d, -(oh/d)) with oh = o + eps
 * (and hi with ol = o - eps): one fused multiply-add per plane, the per-ray
 * products oh/d, ol/d being loop-invariant (hoisted out of the walks).  The
 * rounding of oh/d moves a plane by at most an ulp of |oh| along its axis,
 * the fma's own rounding is relative to t, i.e. an ulp of |t d|; eps (>= 64
 * ulps of the origin-to-scene distance plus 4 ulps of |c| + R, hence >= 2
 * ulps of |o|) covers both, so no parametric slack is needed.  fmaf is the
 * correctly rounded IEEE operation on the host (libm) and the device
 * (v_fma_f32), so the host model decides exactly like the device.  Returns 1
 * when the interval [tmin, tmax] reaches t >= 0; *tmin = entry parameter. */
RT_CULL_FN int rt_box_hit(float ohx, float ohy, float ohz, float olx, float oly, float olz,
                          float ix, float iy, float iz, float lx, float ly, float lz, float hx,
                          float hy, float hz, float *tmin_out)
{
  float tx0 = fmaf(lx, ix, -(ohx * ix)), tx1 = fmaf(hx, ix, -(olx * ix));
  float ty0 = fmaf(ly, iy, -(ohy * iy)), ty1 = fmaf(hy, iy, -(oly * iy));
  float tz0 = fmaf(lz, iz, -(ohz * iz)), tz1 = fmaf(hz, iz, -(olz * iz));
  float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
  float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  *tmin_out = tmin;
  return tmax >= fmaxf(tmin, 0.0f);
}

/* A node whose entry parameter t_enter satisfies t_enter * |d| > limit cannot
 * hold a triangle whose new_dist is <= best (limit = +inf without a best). */
RT_CULL_FN float rt_prune_limit(float best, float eps)
{
  return best + best * RT_CULL_TREL + 2.0f * eps;
}

#endif
