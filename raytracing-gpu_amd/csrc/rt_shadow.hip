// rt_shadow.hip -- exact shadow rays: per-node culling multipliers of the
// shadow walk (DESIGN.md §2 "Exact shadow rays").
//
// cpu/rt's shadow test (cpu/light.c:24-31, cpu/hit.c:93-109) is its float
// Moller-Trumbore test (cpu/hit.c:15-33) over every triangle, and for a ray
// nearly parallel to a triangle's plane that test accepts crossings outside
// the triangle (tools/mt_bound.py): a float accept implies the exact line
// crosses the plane inside the expanded triangle
//     T_D = { v0 + U e1 + V e2 : U >= -du, V >= -dv, U + V <= 1 + dw }.
// Camera rays get per-frame candidate lists for that (csrc/rt_cand.hip).
// Shadow rays come in two families fixed by the scene, not the frame:
//   * a directional light's rays all have the direction -l.v exactly
//     (cpu/light.c:53), so each triangle's grazing cosine is one number;
//   * a point light's rays (P, l.v - P) (cpu/light.c:78) all pass within a
//     few ulps of the light, which bounds the cosine from below like the eye
//     does for camera rays.
// With that cosine the bound is linear in |S| = |o - v0|, and both it and the
// walk's slack eps(o) (host/rt_cull.h, >= eps_rel (|o - c|_max + R)) grow with
// the ray origin's distance from the scene, so
//     reach(T_D beyond T) <= (mu_T - 1) eps(o)   for every origin o,
// with mu_T a per-triangle constant.  The shadow walk grows each node's box by
// mu_N eps(o) instead of eps(o), mu_N = the max of mu_T over the node's
// subtree: every crossing point the float test could accept then lies in the
// grown box of a leaf holding the triangle and of all its ancestors, and the
// walk tests the triangle -- exact by construction.  nu_N does the same for
// the crossing's parameter: a float accept with new_dist > 0.01 may sit at an
// exact parameter slightly behind the origin (by at most the distance error
// derr <= (nu_T - 1) eps(o)), so the shadow slab test accepts boxes reaching
// t >= -nu_N eps(o) / |d|.  Triangles whose bound does not close (grazing
// within the |a| error, rho >= 1/2) go to a global list every shadow ray that
// the walk finds unshadowed tests.
//
// Computed once per scene (the lights are part of the scene), on the device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rt_shadow.h"

namespace rts {

constexpr double kEps = 0x1p-24;           // float unit roundoff
constexpr double kAMin = 9.99999997e-08;   // (double)(float)1e-7, cpu/hit.c:7
constexpr double kCDot = 8.6, kCA = 7.2;   // tools/mt_bound.py C_DOT, C_A
constexpr double kDMax = 1.0 + 4.0 * kEps;

__device__ inline double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ inline double norm3(const double* a) { return sqrt(dot3(a, a)); }

// (mu, nu) of one triangle for one light at grazing cosine >= c (c in
// [0, 1]); false: the bound does not close.
__device__ inline bool mu_nu(const ShadowParams& p, double l1, double l2, double nl, double c,
                             double& mu, double& nu, double& reach_per_s) {
  const double ea = kCA * kEps * l1 * l2 * kDMax;  // E_a / |d|
  const double den = nl * c / kDMax - ea;          // a_lb / |d| (the clamp at 1e-7 cancels)
  if (!(den > 2.0 * ea) || !(den > 0.0)) return false;  // rho >= 1/2: no bound
  const double rho = ea / den;
  const double kap = kCDot * kEps / den;  // E_sh / (|S| |e2| a_lb) and E_dq / (|S| |e1| a_lb)
  const double lmax = fmax(l1, l2), ls = l1 + l2;
  // reach <= dw lmax + (du + dv)(l1 + l2), du + dv <= |S| kap (l1 + l2) / (1 - rho),
  // dw <= (4 eps + |S| kap (l1 + l2) + rho) / (1 - rho)
  reach_per_s = kap * ls * (lmax + ls) / (1.0 - rho);
  const double reach0 = (4.0 * kEps + rho) * lmax / (1.0 - rho);
  // |S| <= sqrt 3 (|o - c|_max + R) and eps(o) >= eps_rel (|o - c|_max + R) +
  // plane_eps: each term is covered by its own part of eps(o); the 1 keeps
  // the slab test's own rounding covered as before
  mu = 1.0 + (1.7320508075688774 * reach_per_s / p.eps_rel + reach0 / p.plane_eps) * (1.0 + 1e-6);
  // distance error of the float crossing parameter, t* >= t_f - derr / |d|
  const double derr_per_s = kap * l1 * l2 / (1.0 - 2.0 * rho - 4.0 * kEps);
  nu = 1.0 + 1.7320508075688774 * derr_per_s / p.eps_rel * (1.0 + 1e-6);
  return true;
}

// Per prim: the max (mu, nu) over the scene's directional and point lights,
// or the global list.
__global__ __launch_bounds__(256) void prim_kernel(ShadowParams p) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  const float* r = (const float*)(p.tri + 3 * (size_t)prim);
  const double v0[3] = {r[0], r[1], r[2]}, e1[3] = {r[3], r[4], r[5]}, e2[3] = {r[6], r[7], r[8]};
  const double l1 = norm3(e1), l2 = norm3(e2);
  const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                       e1[0] * e2[1] - e1[1] * e2[0]};
  const double nl = norm3(n);
  double mu = 1.0, nu = 1.0;
  bool global = false;
  for (uint32_t li = 0; li < p.nlight && !global; li++) {
    const float* L = p.light + 8 * li;
    const uint32_t type = __float_as_uint(L[0]);
    if (type != 1 && type != 2) continue;
    const double lv[3] = {L[4], L[5], L[6]};
    // |d| of the light's rays: -l.v itself, or l.v - o with |o - c|_max <= omax_assumed
    const double lc[3] = {lv[0] - p.c[0], lv[1] - p.c[1], lv[2] - p.c[2]};
    const double dmax = type == 1 ? norm3(lv) * kDMax
                                  : (norm3(lc) + 1.7320508075688774 * p.omax_assumed) * kDMax;
    // the float direction fl(l.v - o) = (l.v - o)(1 + delta), |delta| <= eps: its
    // line through o passes within eps |l.v - o| of the light
    const double dline = 2.0 * kEps * dmax + 1e-12;
    // |a| <= |d| (nl + e_a) kDMax: below the 1e-7 threshold for every ray of
    // this light -> never accepted
    const double ea = kCA * kEps * l1 * l2 * kDMax;
    if ((nl + ea) * kDMax * dmax < kAMin) continue;
    double c;
    if (type == 1) {
      c = nl > 0.0 ? fabs(dot3(n, lv)) / (nl * norm3(lv)) : 0.0;
    } else {
      // lines through the light (within dline): the crossing X lies within
      // reach of the triangle, |X - lv| <= vmax + reach, and the line's
      // distance from the plane at lv is >= dpl - dline
      if (!(nl > 0.0)) {
        global = true;
        break;
      }
      const double pv[3] = {lv[0] - v0[0], lv[1] - v0[1], lv[2] - v0[2]};
      const double dpl = fabs(dot3(n, pv)) / nl;
      double vmax = norm3(pv);
      for (int k = 0; k < 2; k++) {
        const double* e = k ? e2 : e1;
        const double w[3] = {pv[0] - e[0], pv[1] - e[1], pv[2] - e[2]};
        vmax = fmax(vmax, norm3(w));
      }
      c = fmax(0.0, (dpl - dline) / (vmax + p.reach_cap + dline));
    }
    double m, u, rps;
    if (!mu_nu(p, l1, l2, nl, c, m, u, rps)) {
      global = true;
      break;
    }
    // point lights: the cosine bound assumed reach <= reach_cap for origins
    // within the assumed extent (the shade kernel counts the others)
    if (type == 2 && rps * 1.7320508075688774 * (p.omax_assumed + p.R) > p.reach_cap) {
      global = true;
      break;
    }
    mu = fmax(mu, m);
    nu = fmax(nu, u);
  }
  if (global) {
    p.global[atomicAdd(p.nglobal, 1u)] = prim;
    mu = 1.0;  // tested by every shadow ray outside the walk: no growth needed
    nu = 1.0;
  }
  p.prim_mu[prim] = make_float2((float)(mu * (1.0 + 1e-6)), (float)(nu * (1.0 + 1e-6)));
}

// leaf: max over its records' prims; interior nodes start at 1
__global__ __launch_bounds__(256) void leaf_kernel(ShadowParams p) {
  const uint32_t ni = blockIdx.x * blockDim.x + threadIdx.x;
  if (ni >= p.nnode) return;
  const uint32_t first = __float_as_uint(p.node[2 * ni].w), info = __float_as_uint(p.node[2 * ni + 1].w);
  float2 m = make_float2(1.0f, 1.0f);
  if (info & 0x80000000u) {
    const uint32_t cnt = info & 0x7fffffffu;
    for (uint32_t k = 0; k < cnt; k++) {
      const float2 q = p.prim_mu[__float_as_uint(p.rec[3 * (size_t)(first + k) + 2].y)];
      m.x = fmaxf(m.x, q.x);
      m.y = fmaxf(m.y, q.y);
    }
  }
  p.node_mu[ni] = m;
}

// interior: max over its children (one level per launch, repeated tree-depth times)
__global__ __launch_bounds__(256) void up_kernel(ShadowParams p) {
  const uint32_t ni = blockIdx.x * blockDim.x + threadIdx.x;
  if (ni >= p.nnode) return;
  const uint32_t first = __float_as_uint(p.node[2 * ni].w), info = __float_as_uint(p.node[2 * ni + 1].w);
  if (info & 0x80000000u) return;
  float2 m = p.node_mu[ni];
  const uint32_t cnt = info & 0xffu;
  for (uint32_t k = 0; k < cnt; k++) {
    const float2 q = p.node_mu[first + k];
    m.x = fmaxf(m.x, q.x);
    m.y = fmaxf(m.y, q.y);
  }
  p.node_mu[ni] = m;
}

}  // namespace rts

extern "C" hipError_t rt_shadow_build(const ShadowParams* p, int depth, hipStream_t s) {
  if (p->nprim) {
    hipLaunchKernelGGL(rts::prim_kernel, dim3((p->nprim + 255) / 256), dim3(256), 0, s, *p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (!p->nnode) return hipSuccess;
  const dim3 g((p->nnode + 255) / 256), b(256);
  hipLaunchKernelGGL(rts::leaf_kernel, g, b, 0, s, *p);
  for (int k = 0; k <= depth; k++) hipLaunchKernelGGL(rts::up_kernel, g, b, 0, s, *p);
  return hipGetLastError();
}
