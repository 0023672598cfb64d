// rt_reflect.hip -- exact reflection rays: per-node bounds of the float
// Moller-Trumbore error region for the reflection walk (DESIGN.md §2
// "Reflection rays: exact by proof").
//
// A reflection ray (cpu/raytracer.c:26-29, cpu/ray.c:16-25) starts on a
// surface and may point anywhere, so no per-frame or per-light family bounds
// its cosine with a triangle's plane, as the eye does for camera rays
// (csrc/rt_cand.hip) and the lights do for shadow rays (csrc/rt_shadow.hip,
// csrc/rt_lightbuf.hip).  The bound of tools/mt_bound.py still holds for any
// ray: a float accept (cpu/hit.c:15-33) implies the exact line crosses the
// triangle's plane at X inside the expanded triangle T_D, whose reach beyond
// the triangle is
//     reach <= |S| kap ls (lmax + ls) / (1 - rho) + (4 eps + rho) lmax / (1 - rho)
//     kap = C_DOT eps / den,  rho = E_a / a_lb = ea / den,  den = a_lb / |d|,
//     ea = C_A eps l1 l2,  ls = l1 + l2,  lmax = max(l1, l2),  |S| = |o - v0|,
// for any lower bound a_lb of the exact |a| = |d| nl c (nl = |e1 x e2|, c =
// the ray's cosine with the plane).  Two lower bounds of den:
//   * the cone: c >= c_lb, the smallest cosine of the ray with any normal of
//     a node's normal cone, so den >= nl c_lb -- a per-ray, per-node bound,
//     tight where the ray meets a surface steeply;
//   * the floor: |a_f| >= 1e-7f for any accept, so den >= 1e-7f / |d| - ea
//     >= 1e-7f / RT_RF_DLMAX - ea -- ray-independent, the only bound for a
//     ray that grazes some triangle of the node.
// Per node the walk takes, per factor, the smaller of the two bounds (each is
// a valid bound of the same quantity), and with |S| <= (the L1 distance from
// the origin to the farthest point of the node's box) + (the longest edge of
// any triangle of the subtree) grows the node's box by the reach: every
// crossing the float test could accept then lies in the grown box of a leaf
// holding the triangle (every point of a triangle lies in some leaf box that
// references it) and of every ancestor, so the walk tests it.  The distance
// error bounds the pruning and the crossings behind the origin the same way:
//     t* |d| <= [t_f |d| (1 + 2 eps)(1 - rho) + |S| kd] / (1 - 2 rho),
//     kd = C_DOT eps l1 l2 / den.
// A node where neither bound closes (rho >= 1/2: a triangle the ray may lie
// in, within the rounding of a) is entered unconditionally and never pruned.
//
// Per node (3 float4, max over the subtree; every value x (1 + 1e-6)):
//   [0] axis.xyz, psi    the normal cone: |n_T . d^| >= |axis . d^| - psi for
//                        every triangle T below (psi = 1 - cos phi + sin phi,
//                        phi = the cone's half-angle; >= 2: no cone)
//   [1] K1, Ra, Kd, Dm   cone factors: reach per |S| <= K1 / (c_lb - Ra),
//                        rho <= Ra / c_lb, kd <= Kd / c_lb; Dm = longest edge
//   [2] Fr, Fr0, Fd, Frho  floor factors: reach per |S|, the constant reach,
//                        kd, rho (Frho >= 1/2: the floor does not close)
// Built on the device once per scene, when the mode is enabled.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rt_reflect.h"

namespace rtr {

constexpr double kEps = 0x1p-24;          // float unit roundoff
constexpr double kAMin = 9.99999997e-08;  // (double)(float)1e-7, cpu/hit.c:7
constexpr double kCDot = 8.6, kCA = 7.2;  // tools/mt_bound.py C_DOT, C_A
constexpr double kPi2 = 1.5707963267948966;
constexpr double kUp = 1.0 + 1e-6;        // stored values rounded up (float conversion, evaluation)

struct Acc {  // running maxima of one node's triangles
  double K1 = 0, Ra = 0, Kd = 0, Dm = 0, Fr = 0, Fr0 = 0, Fd = 0, Frho = 0;
  bool unbounded = false;
  __device__ void merge(const Acc& o) {
    K1 = fmax(K1, o.K1);
    Ra = fmax(Ra, o.Ra);
    Kd = fmax(Kd, o.Kd);
    Dm = fmax(Dm, o.Dm);
    Fr = fmax(Fr, o.Fr);
    Fr0 = fmax(Fr0, o.Fr0);
    Fd = fmax(Fd, o.Fd);
    Frho = fmax(Frho, o.Frho);
    unbounded = unbounded || o.unbounded;
  }
};

__device__ inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ inline double norm3(const double* a) { return sqrt(dot3(a, a)); }

// One triangle record's factors; false: the float test never accepts it
// (for any query with |d| <= RT_RF_DLMAX), so it bounds nothing.
__device__ inline bool tri_factors(const float4* q, Acc& a, double nh[3]) {
  const double e1[3] = {q[0].w, q[1].x, q[1].y}, e2[3] = {q[1].z, q[1].w, q[2].x};
  const double e3[3] = {e2[0] - e1[0], e2[1] - e1[1], e2[2] - e1[2]};
  const double l1 = norm3(e1), l2 = norm3(e2), l3 = norm3(e3);
  const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                       e1[0] * e2[1] - e1[1] * e2[0]};
  const double nl = norm3(n) * (1.0 + 1e-12);
  const double dlmax = (double)RT_RF_DLMAX;
  const double ea = kCA * kEps * l1 * l2;
  // |a_f| <= |a| + E_a <= |d| (nl + ea) below 1e-7f: rejected by every query
  if (dlmax * (nl + ea) * (1.0 + 1e-9) < kAMin) return false;
  const double lmax = fmax(l1, l2), ls = l1 + l2;
  a.Dm = fmax(l1, fmax(l2, l3));
  if (!(nl > 0.0)) {  // degenerate but large enough to be accepted: nothing bounds it
    a.unbounded = true;
    nh[0] = 0.0;
    nh[1] = 0.0;
    nh[2] = 1.0;
    return true;
  }
  for (int k = 0; k < 3; k++) nh[k] = n[k] / nl;
  a.K1 = kCDot * kEps * ls * (lmax + ls) / nl;
  a.Ra = ea / nl;
  a.Kd = kCDot * kEps * l1 * l2 / nl;
  const double den = kAMin / dlmax - ea;
  if (den > 2.0 * ea) {
    const double rho = ea / den;
    a.Fr = kCDot * kEps * ls * (lmax + ls) / (den * (1.0 - rho));
    a.Fr0 = (4.0 * kEps + rho) * lmax / (1.0 - rho);
    a.Fd = kCDot * kEps * l1 * l2 / den;
    a.Frho = rho;
  } else {
    a.Frho = 1.0;  // the floor does not close for this triangle
  }
  return true;
}

__device__ inline float up_f(double x) { return (float)(x * kUp); }

__device__ inline void store(const ReflParams& p, uint32_t ni, const double ax[3], double phi, bool empty,
                             const Acc& a) {
  float4* o = p.node_rf + 3 * (size_t)ni;
  double psi;
  if (empty)
    psi = 0.0;  // no triangle below bounds anything (the factors are 0)
  else if (phi >= kPi2 || a.unbounded)
    psi = 4.0;  // no cone
  else
    psi = 1.0 - cos(phi) + sin(phi) + 1e-6;  // + the float evaluation of |axis . d^| at query time
  o[0] = make_float4((float)ax[0], (float)ax[1], (float)ax[2], up_f(psi));
  o[1] = make_float4(up_f(a.K1), up_f(a.Ra), up_f(a.Kd), up_f(a.Dm));
  if (a.unbounded || a.Frho >= 0.5)
    o[2] = make_float4(__builtin_inff(), __builtin_inff(), __builtin_inff(), 1.0f);
  else
    o[2] = make_float4(up_f(a.Fr), up_f(a.Fr0), up_f(a.Fd), up_f(a.Frho));
  p.node_phi[ni] = empty ? -1.0f : (float)fmin(phi * kUp, 4.0);
}

// The angle of the float axis stored for a node (as stored) with a unit
// vector's line, in [0, pi/2], rounded up.
__device__ inline double line_angle(const double* axf, const double* u) {
  const double la = norm3(axf);
  double c = la > 0.0 ? fabs(dot3(axf, u)) / la : 0.0;
  c = fmin(1.0, c);
  return acos(c) * kUp + 1e-9;
}

__global__ __launch_bounds__(256) void leaf_kernel(ReflParams p) {
  const uint32_t ni = blockIdx.x * blockDim.x + threadIdx.x;
  if (ni >= p.nnode) return;
  const uint32_t first = __float_as_uint(p.node[2 * ni].w), info = __float_as_uint(p.node[2 * ni + 1].w);
  if (!(info & 0x80000000u)) return;
  const uint32_t cnt = info & 0x7fffffffu;
  Acc acc;
  double s[3] = {0.0, 0.0, 0.0}, ref[3] = {0.0, 0.0, 0.0};
  bool any = false, have_ref = false;
  for (uint32_t k = 0; k < cnt; k++) {  // axis: the sign-aligned sum of the unit normals
    Acc t;
    double nh[3];
    if (!tri_factors(p.rec + 3 * (size_t)(first + k), t, nh)) continue;
    any = true;
    acc.merge(t);
    if (t.unbounded) continue;
    if (!have_ref) {
      for (int a = 0; a < 3; a++) ref[a] = nh[a];
      have_ref = true;
    }
    const double sg = dot3(nh, ref) >= 0.0 ? 1.0 : -1.0;
    for (int a = 0; a < 3; a++) s[a] += sg * nh[a];
  }
  double ax[3] = {0.0, 0.0, 1.0};
  const double ls = norm3(s);
  if (ls > 1e-12)
    for (int a = 0; a < 3; a++) ax[a] = s[a] / ls;
  const double axf[3] = {(double)(float)ax[0], (double)(float)ax[1], (double)(float)ax[2]};
  double phi = 0.0;
  for (uint32_t k = 0; k < cnt && any && !acc.unbounded; k++) {  // the half-angle against the stored axis
    Acc t;
    double nh[3];
    if (!tri_factors(p.rec + 3 * (size_t)(first + k), t, nh)) continue;
    phi = fmax(phi, line_angle(axf, nh));
  }
  if (acc.unbounded) atomicAdd(p.unbounded, 1u);
  store(p, ni, axf, phi, !any, acc);
}

// interior: from the children (one level per launch, repeated depth + 1 times)
__global__ __launch_bounds__(256) void up_kernel(ReflParams p) {
  const uint32_t ni = blockIdx.x * blockDim.x + threadIdx.x;
  if (ni >= p.nnode) return;
  const uint32_t first = __float_as_uint(p.node[2 * ni].w), info = __float_as_uint(p.node[2 * ni + 1].w);
  if (info & 0x80000000u) return;
  const uint32_t cnt = info & 0xffu;
  Acc acc;
  double s[3] = {0.0, 0.0, 0.0}, ref[3] = {0.0, 0.0, 0.0};
  bool any = false, have_ref = false, nocone = false;
  for (uint32_t k = 0; k < cnt; k++) {
    const uint32_t c = first + k;
    const float phic = p.node_phi[c];
    if (phic < 0.0f) continue;  // nothing below it bounds anything
    any = true;
    const float4* o = p.node_rf + 3 * (size_t)c;
    Acc t;
    t.K1 = o[1].x;
    t.Ra = o[1].y;
    t.Kd = o[1].z;
    t.Dm = o[1].w;
    t.Fr = o[2].x;
    t.Fr0 = o[2].y;
    t.Fd = o[2].z;
    t.Frho = o[2].w;
    acc.merge(t);  // (an unbounded child: no cone, Frho = 1 -> the same for the parent)
    if (o[0].w >= 2.0f) {
      nocone = true;
      continue;
    }
    double a[3] = {o[0].x, o[0].y, o[0].z};
    const double la = norm3(a);
    if (!(la > 0.0)) {
      nocone = true;
      continue;
    }
    for (int q = 0; q < 3; q++) a[q] /= la;
    if (!have_ref) {
      for (int q = 0; q < 3; q++) ref[q] = a[q];
      have_ref = true;
    }
    const double sg = dot3(a, ref) >= 0.0 ? 1.0 : -1.0;
    for (int q = 0; q < 3; q++) s[q] += sg * a[q];
  }
  double ax[3] = {0.0, 0.0, 1.0};
  const double ls = norm3(s);
  if (ls > 1e-12)
    for (int q = 0; q < 3; q++) ax[q] = s[q] / ls;
  const double axf[3] = {(double)(float)ax[0], (double)(float)ax[1], (double)(float)ax[2]};
  double phi = nocone ? 4.0 : 0.0;
  for (uint32_t k = 0; k < cnt && any && !nocone; k++) {
    const uint32_t c = first + k;
    const float phic = p.node_phi[c];
    if (phic < 0.0f) continue;
    const float4* o = p.node_rf + 3 * (size_t)c;
    double a[3] = {o[0].x, o[0].y, o[0].z};
    const double la = norm3(a);
    for (int q = 0; q < 3; q++) a[q] /= la;
    // every line within phic of the child's axis is within angle(axis, child
    // axis) + phic of the parent's (the triangle inequality of line angles)
    phi = fmax(phi, line_angle(axf, a) + (double)phic);
  }
  store(p, ni, axf, phi, !any, acc);
}

}  // namespace rtr

extern "C" hipError_t rt_reflect_build(const ReflParams* p, int depth, hipStream_t s) {
  if (!p->nnode) return hipSuccess;
  const dim3 g((p->nnode + 255) / 256), b(256);
  hipLaunchKernelGGL(rtr::leaf_kernel, g, b, 0, s, *p);
  for (int k = 0; k <= depth; k++) hipLaunchKernelGGL(rtr::up_kernel, g, b, 0, s, *p);
  return hipGetLastError();
}
