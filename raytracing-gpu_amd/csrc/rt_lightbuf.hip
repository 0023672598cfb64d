// rt_lightbuf.hip -- light buffers for the shadow queries (rt_lightbuf.h,
// DESIGN.md §4 "Light buffers").  Built once per scene and culling slack, on
// the device: count (cells per triangle) -> scan -> emit (cell, key, prim) ->
// radix sort by (cell, key) -> cell starts.
//
// Two ways to grow a triangle's footprint (LBParams::proven):
//
// * slack (default): a triangle is listed in every cell that a shadow ray
//   passing within the walk's slack of it can start from (the float rounding
//   of the query's own cell and key computations added as margins), and
//   skipped by a query only where it lies entirely behind the ray's origin by
//   more than twice that slack.  The walk tests a triangle when the ray
//   passes within the slack of the leaf box holding it, so both find every
//   hit within the slack of a triangle -- the same exactness class ("tested,
//   not proven", DESIGN.md §2 "Shadow rays").
//
// * proven: listed wherever a shadow ray of this light can make the
//   reference's float Moller-Trumbore test (cpu/hit.c:15-33) accept the
//   triangle.  tools/mt_bound.py bounds the float test: an accept implies the
//   exact line crosses the triangle's plane inside the expanded triangle
//     T_D = { v0 + U e1 + V e2 : U >= -du, V >= -dv, U + V <= 1 + dw },
//   du, dv, dw from the rounding errors E_sh, E_dq, E_a of s.h, d.q, a and a
//   lower bound a_lb of the float |a| (>= 1e-7 for any accept).
//   - A directional light's rays all have the direction d = -l.v exactly
//     (cpu/light.c:53): the exact a = -d.n is one number per triangle, so
//     a_lb = max(1e-7, |a| - E_a) and T_D are fixed (|S| = |o - v0| bounded
//     over the origin box, componentwise).  T_D's projection along the light
//     is the footprint; the crossing X has the origin's projection, and lies
//     at most derr = |d| E_eq / |a| behind it.  No ray accepts a triangle with
//     |a| + E_a < 1e-7: such triangles are listed nowhere.
//   - A point light's rays (P, l.v - P) (cpu/light.c:78) pass within dline of
//     the light.  A ray crossing the plane at X has cosine c >= (s_L - dline)
//     / (|X - l.v| + dline) with the plane (s_L = the light's distance from
//     it), and the bound at cosine c moves X at most h(c) from the triangle;
//     so X lies within r of it only if r <= g(r) = h(c(r)).  g is convex and
//     increasing, and the smallest R with g(R) <= R (iterated from 0) bounds
//     every crossing of rays at c >= c*, provided h(c*) < r(c*) (the r at
//     which c(r) = c*).  Rays at c < c* are accepted only from origins within
//     H_o(c*) of the plane, on lines nearly parallel to it (|s_o| bounded by
//     u, v in [0, 1] and |a_f| <= |a| + E_a), which needs s_L <= H_o(c*) +
//     Dmax c* + dline: for larger s_L there are none.  Triangles whose plane
//     passes that close to the light are listed, in addition, in the band of
//     cube-map cells within asin(c* + dline / rmin_o) of the great circle of
//     the plane through the light parallel to theirs (with the key that is
//     always tested).  The cone of directions to T's ball grown by R is the
//     footprint; keys as in slack mode with derr in place of the slack.
#include <hip/hip_runtime.h>
#include <cstring>  // before rocPRIM
#include <rocprim/rocprim.hpp>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "rt_lightbuf.h"

namespace rtl {

#define RTL_FN __host__ __device__

constexpr double kEps = 0x1p-24;
constexpr double kInvSqrt3 = 0.57735026918962573;
constexpr double kSqrt3 = 1.7320508075688772;
constexpr double kAMin = 9.99999997e-08;   // (double)(float)1e-7, cpu/hit.c:7
constexpr double kCDot = 8.6, kCA = 7.2;   // tools/mt_bound.py C_DOT, C_A (Cauchy-Schwarz)
constexpr double kCW = 6.01, kCWA = 5.01;  // tools/mt_bound.py bound_cw (componentwise)
constexpr double kDMax = 1.0 + 4.0 * kEps;
constexpr uint32_t kSmallCells = 1024;  // more (or a band): counted and emitted by a workgroup
constexpr int kMaxRects = 6;
constexpr int kBlock = 256;

struct BP {
  const float4* tri;
  uint32_t nprim, kind, proven;
  double lv[3];
  double u[3], v[3], w[3];  // DIR: the float axes, as doubles
  double u0, v0, cs, inv_cs;
  uint32_t nx, ny, n;       // DIR grid / POINT face side
  double slack, s1, dmax;
  double olo[3], ohi[3];    // the origin box (LBParams::box_lo/hi)
  double d[3], dlen;        // DIR: the rays' direction -l.v (float) and its length
  double skew;              // DIR: max |u.d^|, |v.d^| (the float axes vs the exact direction)
  double rmin_o;             // POINT proven: a lower bound of |o - l.v| over shadow-ray origins
  uint32_t* count;
  uint32_t* off;
  unsigned long long* keys;
  uint32_t* vals;
  uint32_t* big;
  uint32_t* ctr;  // [0] big prims, [1] global prims, [2] never accepted, [3] band, [4] emission overflow
  uint32_t* global;
};

struct Foot {
  int n;  // rects
  uint32_t face[kMaxRects];
  int x0[kMaxRects], x1[kMaxRects], y0[kMaxRects], y1[kMaxRects];
  double key;    // whole-triangle key (ascending = tested first)
  bool global;
  bool never;    // proven: no ray of the light can make the float test accept it
  // DIR per-cell refinement: the plane's depth over a cell column
  bool plane;
  double pn_u, pn_v, pn_w, pn_d;  // n.u, n.v, n.w, n.v0 of the triangle's plane
  double m;                       // footprint margin (world units)
  double kpad;                    // behind-origin tolerance of the keys (2 slack; proven: derr)
  // per rect: the triangle's image in the rect's coordinates (DIR: u, v;
  // POINT: the face's (s, t)) and its margin there, for the cell overlap
  // test of small footprints; tri_ok = 0: bounding rect only
  bool tri_ok[kMaxRects];
  double tx[kMaxRects][3], ty[kMaxRects][3], tm[kMaxRects];
  // POINT proven: also every cell whose directions x can have |x.bn| <= bB
  // |x|_inf-scaled (the band around the great circle of the plane through
  // the light parallel to the triangle)
  bool band;
  double bn[3], bB;
};

RTL_FN inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
RTL_FN inline double norm3(const double* a) { return sqrt(dot3(a, a)); }
RTL_FN inline void cross3d(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ inline uint32_t orderable(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ inline float unorder(uint32_t b) {
  return __uint_as_float((b & 0x80000000u) ? (b & 0x7fffffffu) : ~b);
}

RTL_FN inline int clampi(double x, int hi) {
  if (!(x > 0.0)) return 0;  // NaN -> 0
  if (x >= (double)hi) return hi;
  return (int)x;
}

RTL_FN inline void foot_init(Foot& f) {
  f.n = 0;
  f.global = false;
  f.never = false;
  f.plane = false;
  f.band = false;
  f.kpad = 0.0;
  f.m = 0.0;
  for (int q = 0; q < kMaxRects; q++) f.tri_ok[q] = false;
}

// DIR: rect and image of the points P[0..2] (the triangle, or T_D) projected
// on (u, v) with margin m; the plane of the triangle for the per-cell keys
RTL_FN inline void dir_rect(const BP& p, const double P[3][3], const double* v0, const double* e1,
                                const double* e2, double m, Foot& f, double& hw) {
  double lu = 1e300, hu = -1e300, lvv = 1e300, hvv = -1e300;
  hw = -1e300;
  for (int k = 0; k < 3; k++) {
    const double a = dot3(P[k], p.u), b = dot3(P[k], p.v), c = dot3(P[k], p.w);
    lu = fmin(lu, a);
    hu = fmax(hu, a);
    lvv = fmin(lvv, b);
    hvv = fmax(hvv, b);
    hw = fmax(hw, c);
    f.tx[0][k] = a;
    f.ty[0][k] = b;
  }
  f.tri_ok[0] = true;
  f.tm[0] = m;
  f.n = 1;
  f.face[0] = 0;
  f.x0[0] = clampi(floor((lu - m - p.u0) * p.inv_cs - 0.01), (int)p.nx - 1);
  f.x1[0] = clampi(floor((hu + m - p.u0) * p.inv_cs + 0.01), (int)p.nx - 1);
  f.y0[0] = clampi(floor((lvv - m - p.v0) * p.inv_cs - 0.01), (int)p.ny - 1);
  f.y1[0] = clampi(floor((hvv + m - p.v0) * p.inv_cs + 0.01), (int)p.ny - 1);
  f.m = m;
  double n[3];
  cross3d(e1, e2, n);
  const double nl = norm3(n);
  f.pn_u = dot3(n, p.u);
  f.pn_v = dot3(n, p.v);
  f.pn_w = dot3(n, p.w);
  f.pn_d = dot3(n, v0);
  f.plane = nl > 0.0 && fabs(f.pn_w) > 0.05 * nl;
}

// POINT: the cube-map rects of the cone from the light around the ball
// (C, rb), widened by alpha, and the central projection of V grown by beta
// for the overlap test.  false: the cone is too wide (global list).
RTL_FN inline bool point_cone(const BP& p, const double V[3][3], const double C[3], double rb, double& rmin,
                                  double grow, Foot& f) {
  const double D[3] = {C[0] - p.lv[0], C[1] - p.lv[1], C[2] - p.lv[2]};
  const double dc = norm3(D);
  if (!(dc > rb * 1.001 + 1e-9)) return false;
  rmin = dc - rb;
  const double alpha = 4.0 * kSqrt3 * kEps * p.dmax / rmin + 8.0 * kEps;
  const double th = asin(fmin(1.0, rb / dc)) + alpha + 1e-12;
  if (!(th < 1.2)) return false;
  double xlo[3], xhi[3];
  for (int a = 0; a < 3; a++) {
    const double ph = acos(fmax(-1.0, fmin(1.0, D[a] / dc)));
    xlo[a] = cos(fmin(3.141592653589793, ph + th)) - 1e-12;
    xhi[a] = cos(fmax(0.0, ph - th)) + 1e-12;
  }
  const double hn = 0.5 * (double)p.n;
  for (int a = 0; a < 3; a++)
    for (int sg = 0; sg < 2; sg++) {
      double alo = sg == 0 ? xlo[a] : -xhi[a], ahi = sg == 0 ? xhi[a] : -xlo[a];
      if (ahi < kInvSqrt3 * (1.0 - 1e-9)) continue;  // the cone never reaches this face's frustum
      alo = fmax(alo, kInvSqrt3 * (1.0 - 1e-9));    // directions on the face have |x_a| >= 1/sqrt 3
      const int j = (a + 1) % 3, k = (a + 2) % 3;
      const double slo = fmin(xlo[j] / alo, xlo[j] / ahi), shi = fmax(xhi[j] / alo, xhi[j] / ahi);
      const double tlo = fmin(xlo[k] / alo, xlo[k] / ahi), thi = fmax(xhi[k] / alo, xhi[k] / ahi);
      if (slo > 1.0 + 1e-9 || shi < -1.0 - 1e-9 || tlo > 1.0 + 1e-9 || thi < -1.0 - 1e-9) continue;
      const int q = f.n++;
      f.face[q] = (uint32_t)(2 * a + sg);
      // the triangle's central projection onto the face (valid when every
      // vertex lies well on the face's side), grown by the cone's widening
      // beta (grow / rmin + alpha) through the face map's Lipschitz bound
      {
        const double beta = grow / rmin + alpha;
        const double sgn = sg == 0 ? 1.0 : -1.0;
        double xamin = 1e300, smax = 1.0;
        bool ok = true;
        for (int v = 0; v < 3 && ok; v++) {
          const double X[3] = {V[v][0] - p.lv[0], V[v][1] - p.lv[1], V[v][2] - p.lv[2]};
          const double xl = norm3(X), xa = sgn * X[a];
          ok = xl > 0.0 && xa > 1e-3 * xl;
          if (!ok) break;
          xamin = fmin(xamin, xa / xl);
          f.tx[q][v] = X[j] / xa;
          f.ty[q][v] = X[k] / xa;
          smax = fmax(smax, fmax(fabs(f.tx[q][v]), fabs(f.ty[q][v])));
        }
        if (ok && xamin > 4.0 * beta) {
          f.tri_ok[q] = true;
          f.tm[q] = 2.0 * beta * (1.0 + smax + 2.0 * beta) / (xamin - 2.0 * beta) * 1.01 + 1e-9;
        }
      }
      f.x0[q] = clampi(floor((fmax(slo, -1.0) + 1.0) * hn - 0.01), (int)p.n - 1);
      f.x1[q] = clampi(floor((fmin(shi, 1.0) + 1.0) * hn + 0.01), (int)p.n - 1);
      f.y0[q] = clampi(floor((fmax(tlo, -1.0) + 1.0) * hn - 0.01), (int)p.n - 1);
      f.y1[q] = clampi(floor((fmin(thi, 1.0) + 1.0) * hn + 0.01), (int)p.n - 1);
    }
  return true;
}

// ---- slack-grown footprints (default) ----
RTL_FN void footprint_slack(const BP& p, const double V[3][3], const double* v0, const double* e1,
                                const double* e2, Foot& f) {
  if (p.kind == RT_LB_DIR) {
    // the query's float projection of its origin is within 3 eps s1 of the
    // exact one; the triangle's points are within the slack of the ray
    const double m = p.slack + 3.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1;
    double hw;
    dir_rect(p, V, v0, e1, e2, m, f, hw);
    // skipped by a query when its deepest point, grown by the slack on both
    // sides (behind-origin tolerance of the walk) and the rounding of the
    // query's depth, lies below the origin: key = -(that bound)
    f.kpad = 2.0 * p.slack;
    f.key = -(hw + 2.0 * p.slack + 6.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1);
    return;
  }
  // POINT: the cone from the light around the triangle's bounding sphere
  // (grown by the slack), widened by the angle the rounding of the shadow
  // direction l.v - P can turn a ray's points as seen from the light
  double C[3];
  for (int a = 0; a < 3; a++) C[a] = (V[0][a] + V[1][a] + V[2][a]) / 3.0;
  double rb = 0.0;
  for (int k = 0; k < 3; k++) {
    const double d[3] = {V[k][0] - C[0], V[k][1] - C[1], V[k][2] - C[2]};
    rb = fmax(rb, norm3(d));
  }
  rb = rb * (1.0 + 1e-12) + p.slack + 1e-12;
  double rmin = 0.0;
  if (!point_cone(p, V, C, rb, rmin, p.slack, f)) {
    f.n = 0;
    f.global = true;
    return;
  }
  // a query toward the light stops once the triangle's nearest possible
  // point lies farther from the light than its origin (plus the slack)
  f.kpad = 2.0 * p.slack;
  f.key = rmin - 2.0 * p.slack - 1e-9 * p.dmax;
}

// ---- proven footprints (module comment) ----
RTL_FN void footprint_dir_proven(const BP& p, const double* v0, const double* e1, const double* e2, Foot& f) {
  const double* d = p.d;
  double n[3];
  cross3d(e1, e2, n);
  const double A = fabs(dot3(n, d));  // |a| exact: a = e1.(d x e2) = -d.n, every ray alike
  double M[3], S[3];
  for (int i = 0; i < 3; i++) S[i] = fmax(fabs(p.olo[i] - v0[i]), fabs(p.ohi[i] - v0[i]));
  double Ea = 0.0;
  for (int i = 0; i < 3; i++) {
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    M[i] = fabs(d[j]) * fabs(e2[k]) + fabs(d[k]) * fabs(e2[j]);
    Ea += fabs(e1[i]) * M[i];
  }
  const double r1 = 1.0 + 1e-6;
  Ea *= kCWA * kEps * r1;
  if (A + Ea < kAMin * (1.0 - 1e-9)) {  // |a_f| < 1e-7 for every ray: rejected (cpu/hit.c:19)
    f.never = true;
    return;
  }
  const double alb = fmax(kAMin, A - Ea);
  const double rho = Ea / alb;
  if (!(rho < 0.5)) {
    f.global = true;
    return;
  }
  const double C[3] = {v0[0] + (e1[0] + e2[0]) / 3.0, v0[1] + (e1[1] + e2[1]) / 3.0, v0[2] + (e1[2] + e2[2]) / 3.0};
  const double ud[3] = {-d[0] / p.dlen, -d[1] / p.dlen, -d[2] / p.dlen};  // from X back toward the origin
  double du = 0.0, dv = 0.0, dw = 0.0, Eeq = 0.0;
  double P[3][3];
  // T_D with |S_i| <= the box bound, then again with the origins' own bound:
  // an accepting ray's origin o = X - t d (t >= 0) lies in the box, X in T_D
  // (every step valid for every accepting ray, so each bound is)
  for (int pass = 0; pass < 3; pass++) {
    double N[3], Esh = 0.0, Edq = 0.0;
    Eeq = 0.0;
    for (int i = 0; i < 3; i++) {
      const int j = (i + 1) % 3, k = (i + 2) % 3;
      N[i] = S[j] * fabs(e1[k]) + S[k] * fabs(e1[j]);
    }
    for (int i = 0; i < 3; i++) {
      Esh += S[i] * M[i];
      Edq += fabs(d[i]) * N[i];
      Eeq += fabs(e2[i]) * N[i];
    }
    Esh *= kCW * kEps * r1;
    Edq *= kCW * kEps * r1;
    Eeq *= kCW * kEps * r1;
    du = Esh / (alb * (1.0 - rho));
    dv = Edq / (alb * (1.0 - rho));
    dw = (4.0 * kEps + (Esh + Edq) / alb + rho) / (1.0 - rho);
    // T_D's corners (U, V) = (-du, -dv), (1 + dw + dv, -dv), (-du, 1 + dw + du)
    const double cU[3] = {-du, 1.0 + dw + dv, -du}, cV[3] = {-dv, -dv, 1.0 + dw + du};
    double rX = 0.0;
    for (int k = 0; k < 3; k++) {
      double w[3];
      for (int a = 0; a < 3; a++) {
        P[k][a] = v0[a] + cU[k] * e1[a] + cV[k] * e2[a];
        w[a] = P[k][a] - C[a];
      }
      rX = fmax(rX, norm3(w));
    }
    rX = rX * (1.0 + 1e-9) + 1e-9;
    if (pass == 2) break;
    // the origin lies on the line behind X: t <= the box exit along ud
    double tex = 1e300;
    for (int a = 0; a < 3; a++) {
      if (ud[a] > 0.0) tex = fmin(tex, (p.ohi[a] - (C[a] - rX)) / ud[a]);
      if (ud[a] < 0.0) tex = fmin(tex, ((C[a] + rX) - p.olo[a]) / -ud[a]);
    }
    tex = fmax(tex, 0.0) * (1.0 + 1e-9);
    for (int i = 0; i < 3; i++)
      S[i] = fmin(S[i], (fabs(C[i] - v0[i]) + rX + tex * fabs(ud[i])) * (1.0 + 1e-9));
  }
  const double Smax = sqrt(S[0] * S[0] + S[1] * S[1] + S[2] * S[2]);
  const double ext = (1.0 + du + dv + dw) * (norm3(e1) + norm3(e2));
  // the query's float projection (3 eps s1), and X - o along d seen through
  // the float axes (|X - o| <= |S| + T_D's extent)
  const double m = 3.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1 + p.skew * (Smax + ext) * 1.01;
  double hw;
  dir_rect(p, P, v0, e1, e2, m, f, hw);
  // an accept has t* >= -E_eq / |a|: X at most derr behind the origin
  const double derr = Eeq * p.dlen / A * 1.01;
  f.kpad = derr;
  f.key = -(hw + derr + 6.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1);
}

// reach of T_D beyond T for rays at cosine c (|d| cancels), Cauchy-Schwarz
// form as csrc/rt_shadow.hip; > 1e300: no bound
RTL_FN inline double reach_at(double c, double nl, double ea, double l1, double l2, double Smax) {
  const double den = nl * c - ea;
  if (!(den > 2.0001 * ea) || !(den > 0.0)) return 1e301;
  const double rho = ea / den, kap = kCDot * kEps / den;
  const double lmax = fmax(l1, l2), ls = l1 + l2;
  return (kap * ls * (lmax + ls) * Smax / (1.0 - rho) + (4.0 * kEps + rho) * lmax / (1.0 - rho)) * (1.0 + 1e-6);
}

// |o - v0| over the origins of accepting shadow rays of a point light that
// cross T's plane within rX of T's centroid C: o lies on a line through X
// (|X - C| <= rX) passing within dline of the light, either beyond X (o = X +
// lam u, u = (X - l.v) / |X - l.v|, the crossing between o and the light) or
// beyond the light (o = l.v - mu u, the crossing past the light); every such
// o is in the origin box, so lam, mu <= the box's exit along u's cone.
RTL_FN double point_smax(const BP& p, const double* C, const double* v0, double rX, double dline, double sbox) {
  const double D[3] = {C[0] - p.lv[0], C[1] - p.lv[1], C[2] - p.lv[2]};
  const double dc = norm3(D);
  if (!(dc > 2.0 * (rX + dline) + 1e-9)) return sbox;
  // |u - c^| <= the cone's half-angle (plus the line's offset from the light)
  const double th = asin(fmin(1.0, (rX + dline) / dc)) + (rX + dline) / (dc - rX - dline) * 1e-6 + 1e-12;
  const double sp = fmin(2.0, th * 1.001);
  double lam = 1e300, mu = 1e300;
  for (int a = 0; a < 3; a++) {
    const double ulo = D[a] / dc - sp, uhi = D[a] / dc + sp;
    if (ulo > 0.0) lam = fmin(lam, (p.ohi[a] - (C[a] - rX)) / ulo);
    if (uhi < 0.0) lam = fmin(lam, ((C[a] + rX) - p.olo[a]) / -uhi);
    // beyond the light along -u
    // (from the line's point nearest the light, within dline of it)
    if (-uhi > 0.0) mu = fmin(mu, (p.ohi[a] - p.lv[a] + dline) / -uhi);
    if (-ulo < 0.0) mu = fmin(mu, (p.lv[a] + dline - p.olo[a]) / ulo);
  }
  lam = fmax(lam, 0.0);
  // mu < 0: the line beyond the light never reaches the box (no such origin)
  const double far = mu < 0.0 ? 0.0 : dc + rX + mu;
  const double ox = fmax(lam, far) + 2.0 * dline;
  double cv[3];
  for (int a = 0; a < 3; a++) cv[a] = C[a] - v0[a];
  return fmin(sbox, (norm3(cv) + rX + ox) * (1.0 + 1e-9) + 1e-9);
}

RTL_FN void footprint_point_proven(const BP& p, const double V[3][3], const double* v0, const double* e1,
                                   const double* e2, Foot& f) {
  double n[3];
  cross3d(e1, e2, n);
  const double nl = norm3(n), l1 = norm3(e1), l2 = norm3(e2);
  const double lmax = fmax(l1, l2), ls = l1 + l2;
  const double ea = kCA * kEps * l1 * l2 * kDMax;  // E_a / |d|
  const double Dmax = p.dmax;
  // |a_f| <= |d| (|n| + e_a) < 1e-7 for every ray: never accepted
  if (Dmax * (nl + ea) * kDMax < kAMin * (1.0 - 1e-9)) {
    f.never = true;
    return;
  }
  if (!(nl > 0.0)) {  // degenerate: a is rounding noise, u, v unbounded
    f.global = true;
    return;
  }
  const double nh[3] = {n[0] / nl, n[1] / nl, n[2] / nl};
  const double LV[3] = {p.lv[0] - v0[0], p.lv[1] - v0[1], p.lv[2] - v0[2]};
  const double sL = fabs(dot3(nh, LV));
  double vmax = 0.0, S[3];
  for (int k = 0; k < 3; k++) {
    const double X[3] = {V[k][0] - p.lv[0], V[k][1] - p.lv[1], V[k][2] - p.lv[2]};
    vmax = fmax(vmax, norm3(X));
  }
  double C[3];
  for (int a = 0; a < 3; a++) C[a] = (V[0][a] + V[1][a] + V[2][a]) / 3.0;
  double rc = 0.0;
  for (int k = 0; k < 3; k++) {
    const double d[3] = {V[k][0] - C[0], V[k][1] - C[1], V[k][2] - C[2]};
    rc = fmax(rc, norm3(d));
  }
  rc *= 1.0 + 1e-12;
  for (int i = 0; i < 3; i++) S[i] = fmax(fabs(p.olo[i] - v0[i]), fabs(p.ohi[i] - v0[i]));
  const double Sbox = sqrt(S[0] * S[0] + S[1] * S[1] + S[2] * S[2]) * (1.0 + 1e-9);
  const double dline = 2.0 * kSqrt3 * kEps * Dmax;  // fl(l.v - o) from o passes this close to l.v
  const double a_ = sL - dline, b_ = vmax * (1.0 + 1e-12) + dline;
  // rays crossing within r of T: cosine >= c(r) = a_ / (b_ + r); R = a point
  // past the smallest fixed point of g(r) = reach_at(c(r)) (g(R) <= R)
  auto fixed_point = [&](double Sm) {
    double r = 0.0;
    if (!(a_ > 0.0)) return 1e301;
    for (int it = 0; it < 64; it++) {
      const double g = reach_at(a_ / (b_ + r), nl, ea, l1, l2, Sm);
      if (!(g < 1e300)) return 1e301;
      if (g <= r) return r;
      r = g * (1.0 + 1e-9) + 1e-300;
    }
    return 1e301;
  };
  double Smax = Sbox;
  double R = fixed_point(Smax);
  bool band = true;
  double clo = 0.0;
  if (R < 1e300) {
    // H_o(c) + Dmax c + dline: how close to the plane the light must be for a
    // ray at cosine < c to be accepted at all (module comment); any origin
    // in the box, so the box's |S|
    auto q = [&](double c) {
      return ls / (nl * (1.0 - c)) *
                 ((nl * c + ea) * (1.0 + 4.0 * kEps) + kCDot * kEps * Sbox * lmax + c * Sbox * lmax) *
                 (1.0 + 1e-6) +
             Dmax * c * (1.0 + 4.0 * kEps) + dline;
    };
    if (q(0.0) < sL) {
      double lo = 0.0, hi = 0.5;
      if (q(hi) <= sL) {
        lo = hi;
      } else {
        for (int it = 0; it < 64; it++) {
          const double mid = 0.5 * (lo + hi);
          if (q(mid) <= sL)
            lo = mid;
          else
            hi = mid;
        }
      }
      const double cst = lo;  // q(cst) <= sL: no accepted ray below cst
      if (cst > 0.0) {
        const double rhi = a_ / cst - b_;
        const double hc = reach_at(cst, nl, ea, l1, l2, Sbox);
        if (hc < rhi) {  // rays at c >= cst cross within R (convexity of g)
          band = false;
          // every accepting ray crosses within R: its origin's |S| is bounded
          // by point_smax, and the fixed point again with that bound (each
          // step valid for every accepting ray)
          for (int it = 0; it < 2; it++) {
            Smax = point_smax(p, C, v0, rc + R, dline, Sbox);
            const double R2 = fixed_point(Smax);
            if (!(R2 < 1e300)) break;
            R = fmin(R, R2);
          }
          clo = a_ / (b_ + R);
        }
      }
    }
  }
  // the band alternative (valid for every triangle): rays at c >= cst
  // cross within reach_at(cst) of T; rays below leave origins in the band of
  // directions within asin(cst + dline / rmin_o) of the plane through the
  // light parallel to T's.  Taken when the bound above fails, or when its
  // cone would cover more cells than the band and a small cone (a plane
  // passing close to the light: R grows like 1 / s_L).
  {
    const double Dc[3] = {C[0] - p.lv[0], C[1] - p.lv[1], C[2] - p.lv[2]};
    const double dc = norm3(Dc), hn = 0.5 * (double)p.n;
    auto cone_cells = [&](double Rr) {
      if (!(dc > (rc + Rr) * 1.001)) return 1e300;
      const double th = asin(fmin(1.0, (rc + Rr) / dc)) * hn;
      return 3.2 * th * th + 4.0 * th + 1.0;
    };
    const double rmin_o = p.rmin_o;
#ifndef RT_LB_BAND_C
#define RT_LB_BAND_C 0.5  // the band's cosine split c* = RT_LB_BAND_C / n (cells of the cube map's side n)
#endif
    const double cst = fmax(RT_LB_BAND_C / (double)p.n, 8.0 * ea / nl);
    double Sb = Sbox, Rb = reach_at(cst, nl, ea, l1, l2, Sb);
    if (Rb < 1e300) {
      Sb = point_smax(p, C, v0, rc + Rb, dline, Sbox);
      Rb = fmin(Rb, reach_at(cst, nl, ea, l1, l2, Sb));
    }
    const double bs = cst * (1.0 + 1e-6) + (rmin_o > 0.0 ? dline / rmin_o : 1e300) + 4.0 * kEps;
    const bool bok = cst < 0.25 && Rb < 1e300 && bs < 0.3;
    const double band_cells = bok ? 4.0 * (double)p.n * (bs * kSqrt3 * hn * 2.0 + 3.0) + cone_cells(Rb) : 1e300;
    if (!band && !(cone_cells(R) > band_cells)) {
      // keep the cone alone
    } else if (bok) {
      band = true;
      R = Rb;
      Smax = Sb;
      clo = cst;
      f.band = true;
      for (int a = 0; a < 3; a++) f.bn[a] = nh[a];
      // a face cell holds directions x = (s, t, +-1): |x| <= sqrt 3
      f.bB = bs * kSqrt3 * (1.0 + 1e-9) + 1e-12;
    } else if (band) {
      f.global = true;
      return;
    }
  }
  const double rb = rc + R + 1e-12;
  double rmin = 0.0;
  if (!point_cone(p, V, C, rb, rmin, R, f)) {
    f.n = 0;
    f.band = false;
    f.global = true;
    return;
  }
  // an accept has t* >= -E_eq / |a|, |a| >= |d| |n| clo: X at most derr
  // behind the origin (toward the light)
  const double derr = kCDot * kEps * Smax * l1 * l2 / (nl * clo) * 1.01;
  f.kpad = derr;
  f.key = rmin - derr - 2.0 * dline - 1e-9 * p.dmax;
}

RTL_FN void footprint(const BP& p, uint32_t prim, Foot& f) {
  const float* r = (const float*)(p.tri + 3 * (size_t)prim);
  const double v0[3] = {r[0], r[1], r[2]}, e1[3] = {r[3], r[4], r[5]}, e2[3] = {r[6], r[7], r[8]};
  const double V[3][3] = {{v0[0], v0[1], v0[2]},
                          {v0[0] + e1[0], v0[1] + e1[1], v0[2] + e1[2]},
                          {v0[0] + e2[0], v0[1] + e2[1], v0[2] + e2[2]}};
  foot_init(f);
  if (!p.proven)
    footprint_slack(p, V, v0, e1, e2, f);
  else if (p.kind == RT_LB_DIR)
    footprint_dir_proven(p, v0, e1, e2, f);
  else
    footprint_point_proven(p, V, v0, e1, e2, f);
}

RTL_FN inline uint64_t foot_cells(const BP& p, const Foot& f) {
  uint64_t c = 0;
  for (int q = 0; q < f.n; q++)
    c += (uint64_t)(f.x1[q] - f.x0[q] + 1) * (uint64_t)(f.y1[q] - f.y0[q] + 1);
  return c;
}

// key of the triangle in cell (x, y) of rect q
__device__ inline float cell_key(const BP& p, const Foot& f, int x, int y) {
  double key = f.key;
  if (p.kind == RT_LB_DIR && f.plane) {
    // the plane's depth over the cell's column grown by the margin: points of
    // the triangle in the column lie on the plane, h = (n.v0 - n_u pu - n_v pv) / n_w;
    // the float axes are orthonormal within a few ulps (1e-6 s1 covers it)
    const double ua = p.u0 + x * p.cs - f.m, ub = p.u0 + (x + 1) * p.cs + f.m;
    const double va = p.v0 + y * p.cs - f.m, vb = p.v0 + (y + 1) * p.cs + f.m;
    double h = -1e300;
    const double us[2] = {ua, ub}, vs[2] = {va, vb};
    for (int i = 0; i < 2; i++)
      for (int k = 0; k < 2; k++) h = fmax(h, (f.pn_d - f.pn_u * us[i] - f.pn_v * vs[k]) / f.pn_w);
    const double kc = -(h + f.kpad + 6.0 * kEps * p.s1 * 1.01 + 1e-6 * p.s1);
    key = fmax(key, kc);  // the tighter (larger) of the two lower bounds of -depth
  }
  return __double2float_rd(key);
}

// Can the triangle's grown image in rect q reach cell (x, y)?  Separating
// axis test of the cell square (grown by the margin) against the image's edge
// lines; conservative (true when unsure: degenerate images, rect-only).
RTL_FN inline bool cell_overlaps(const BP& p, const Foot& f, int q, int x, int y) {
  if (!f.tri_ok[q]) return true;
  double ox, oy, cs;
  if (p.kind == RT_LB_DIR) {
    ox = p.u0;
    oy = p.v0;
    cs = p.cs;
  } else {
    cs = 2.0 / (double)p.n;
    ox = oy = -1.0;
  }
  // the query's own cell index is within 0.01 cells of its exact position
  // (the bounding rects' margin): the square grows by as much
  const double M = f.tm[q] + 0.01 * cs;
  const double xa = ox + x * cs - M, xb = ox + (x + 1) * cs + M;
  const double ya = oy + y * cs - M, yb = oy + (y + 1) * cs + M;
  const double* X = f.tx[q];
  const double* Y = f.ty[q];
  const double area = (X[1] - X[0]) * (Y[2] - Y[0]) - (X[2] - X[0]) * (Y[1] - Y[0]);
  const double scale = fabs(X[1] - X[0]) + fabs(X[2] - X[0]) + fabs(Y[1] - Y[0]) + fabs(Y[2] - Y[0]);
  if (!(fabs(area) > 1e-9 * scale * scale)) return true;  // (nearly) degenerate image: keep
  for (int e = 0; e < 3; e++) {
    const int a = e, b = (e + 1) % 3;
    // inward normal of edge a -> b (toward the third vertex)
    double nx = -(Y[b] - Y[a]), ny = X[b] - X[a];
    if (area < 0.0) {
      nx = -nx;
      ny = -ny;
    }
    // the square is outside when all its corners are beyond the edge line
    const double cx = nx > 0.0 ? xb : xa, cy = ny > 0.0 ? yb : ya;  // the corner farthest inward
    const double d = nx * (cx - X[a]) + ny * (cy - Y[a]);
    const double tol = 1e-9 * (fabs(nx) + fabs(ny)) * (fabs(cx) + fabs(cy) + fabs(X[a]) + fabs(Y[a]) + cs);
    if (d < -tol) return false;
  }
  return true;
}

RTL_FN inline uint32_t cell_index(const BP& p, const Foot& f, int q, int x, int y) {
  if (p.kind == RT_LB_DIR) return (uint32_t)y * p.nx + (uint32_t)x;
  return f.face[q] * p.n * p.n + (uint32_t)y * p.n + (uint32_t)x;
}

// Band row (face, y) of a POINT footprint: the columns whose cells hold a
// direction x = (s, t, sigma) (face frame: s along axis a+1, t along a+2, as
// the query maps them) with |x.bn| <= bB; false: none.  Widened by 0.02 cells
// for the query's rounding.
RTL_FN inline bool band_row(const BP& p, const Foot& f, uint32_t face, uint32_t y, int& xa, int& xb) {
  const int a = (int)(face >> 1), j = (a + 1) % 3, k = (a + 2) % 3;
  const double sigma = (face & 1) ? -1.0 : 1.0;
  const double cs = 2.0 / (double)p.n, pad = 0.02 * cs;
  const double t0 = -1.0 + y * cs - pad, t1 = -1.0 + (y + 1) * cs + pad;
  const double nj = f.bn[j], nk = f.bn[k], na = f.bn[a];
  const double g0 = nk * t0 + na * sigma, g1 = nk * t1 + na * sigma;
  const double glo = fmin(g0, g1), ghi = fmax(g0, g1);
  const double B = f.bB;
  double lo, hi;
  if (fabs(nj) < 1e-12) {
    if (glo > B + 1e-12 || ghi < -B - 1e-12) return false;
    lo = -1.0;
    hi = 1.0;
  } else {
    const double A0 = (-B - ghi) / nj, A1 = (B - glo) / nj;
    lo = fmin(A0, A1) - pad;
    hi = fmax(A0, A1) + pad;
  }
  if (lo > 1.0 || hi < -1.0) return false;
  const double hn = 0.5 * (double)p.n;
  xa = clampi(floor((fmax(lo, -1.0) + 1.0) * hn - 0.02), (int)p.n - 1);
  xb = clampi(floor((fmin(hi, 1.0) + 1.0) * hn + 0.02), (int)p.n - 1);
  return xa <= xb;
}

// A footprint as rows: each rect's rows, then (band) the 6 n rows of the cube map.
RTL_FN inline uint32_t foot_rows(const BP& p, const Foot& f) {
  uint32_t r = 0;
  for (int q = 0; q < f.n; q++) r += (uint32_t)(f.y1[q] - f.y0[q] + 1);
  if (f.band) r += 6u * p.n;
  return r;
}

// entries of row `row`; with emit, written from `at` on, never at or past
// `lim` (the prim's own range: a count/emission mismatch is flagged in
// ctr[4], not written out of bounds)
template <bool EMIT>
RTL_FN inline uint32_t row_entries(const BP& p, const Foot& f, uint32_t prim, uint32_t row, uint64_t at,
                                       uint64_t lim) {
  for (int q = 0; q < f.n; q++) {
    const uint32_t nr = (uint32_t)(f.y1[q] - f.y0[q] + 1);
    if (row >= nr) {
      row -= nr;
      continue;
    }
    const int y = f.y0[q] + (int)row;
    uint32_t c = 0;
    for (int x = f.x0[q]; x <= f.x1[q]; x++)
      if (cell_overlaps(p, f, q, x, y)) {
        if constexpr (EMIT) {
          if (at + c >= lim) {
            p.ctr[4] = 1u;
            return c;
          }
          p.keys[at + c] = ((unsigned long long)cell_index(p, f, q, x, y) << 32) | orderable(cell_key(p, f, x, y));
          p.vals[at + c] = prim;
        }
        c++;
      }
    return c;
  }
  // band rows: always tested (key -inf)
  const uint32_t face = row / p.n, y = row % p.n;
  int xa = 0, xb = -1;
  if (!band_row(p, f, face, y, xa, xb)) return 0;
  if constexpr (EMIT) {
    const uint32_t kb = orderable(-__builtin_inff());
    for (int x = xa; x <= xb; x++) {
      const uint64_t i = at + (uint64_t)(x - xa);
      if (i >= lim) {
        p.ctr[4] = 1u;
        break;
      }
      p.keys[i] = ((unsigned long long)(face * p.n * p.n + y * p.n + (uint32_t)x) << 32) | kb;
      p.vals[i] = prim;
    }
  }
  return (uint32_t)(xb - xa + 1);
}

RTL_FN inline bool foot_is_big(const BP& p, const Foot& f) { return f.band || foot_cells(p, f) > kSmallCells; }

// distance from x to the triangle (a, b, c), double: the closest point by the
// interior / edge cases
RTL_FN double pt_tri_dist(const double* x, const double* a, const double* b, const double* c) {
  double ab[3], ac[3], ax[3];
  for (int i = 0; i < 3; i++) {
    ab[i] = b[i] - a[i];
    ac[i] = c[i] - a[i];
    ax[i] = x[i] - a[i];
  }
  double n[3];
  cross3d(ab, ac, n);
  const double nn = dot3(n, n);
  if (nn > 0.0) {
    double t[3], s[3];
    cross3d(ab, ax, t);
    cross3d(ax, ac, s);
    const double v = dot3(t, n) / nn, u = dot3(s, n) / nn;
    if (u >= 0.0 && v >= 0.0 && u + v <= 1.0) return fabs(dot3(ax, n)) / sqrt(nn);
  }
  double best = 1e300;
  const double* P[3] = {a, b, c};
  for (int e = 0; e < 3; e++) {
    const double* p0 = P[e];
    const double* p1 = P[(e + 1) % 3];
    double d[3], w[3];
    for (int i = 0; i < 3; i++) {
      d[i] = p1[i] - p0[i];
      w[i] = x[i] - p0[i];
    }
    const double dd = dot3(d, d);
    double t = dd > 0.0 ? dot3(w, d) / dd : 0.0;
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double z[3] = {w[0] - t * d[0], w[1] - t * d[1], w[2] - t * d[2]};
    best = fmin(best, norm3(z));
  }
  return best;
}

// a lower bound of the distance from the light to the shadow-ray origins on
// this triangle (hit points: on it up to their float rounding, 1e-6 s1)
RTL_FN double prim_rmin(const BP& p, uint32_t prim) {
  const float* r = (const float*)(p.tri + 3 * (size_t)prim);
  const double v0[3] = {r[0], r[1], r[2]};
  const double v1[3] = {v0[0] + r[3], v0[1] + r[4], v0[2] + r[5]};
  const double v2[3] = {v0[0] + r[6], v0[1] + r[7], v0[2] + r[8]};
  const double d = pt_tri_dist(p.lv, v0, v1, v2) * (1.0 - 1e-9) - 1e-6 * p.s1;
  return d > 0.0 ? d : 0.0;
}

__global__ __launch_bounds__(256) void rmin_kernel(BP p, uint32_t* bits) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  const double dist = prim_rmin(p, prim);
  const float fd = dist > 0.0 ? __double2float_rd(dist) : 0.0f;
  atomicMin(bits, __float_as_uint(fd));  // non-negative floats order as their bits
}

__global__ __launch_bounds__(256) void count_kernel(BP p) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  Foot f;
  footprint(p, prim, f);
  uint32_t c = 0;
  if (f.never) {
    atomicAdd(p.ctr + 2, 1u);
  } else if (f.global) {
    p.global[atomicAdd(p.ctr + 1, 1u)] = prim;
  } else if (foot_is_big(p, f)) {
    p.big[atomicAdd(p.ctr, 1u)] = prim;  // counted and emitted row-wise by a workgroup
    if (f.band) atomicAdd(p.ctr + 3, 1u);
  } else {
    const uint32_t rows = foot_rows(p, f);
    for (uint32_t r = 0; r < rows; r++) c += row_entries<false>(p, f, prim, r, 0, 0);
  }
  p.count[prim] = c;  // the host checks the total against 2^31
}

__device__ inline uint32_t block_sum(uint32_t v, uint32_t* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < kBlock / 64; w++) t += red[w];
  __syncthreads();
  return t;
}

// one workgroup per big footprint: its rows over the threads
__global__ __launch_bounds__(256) void big_count_kernel(BP p) {
  __shared__ uint32_t red[kBlock / 64];
  for (uint32_t b = blockIdx.x; b < p.ctr[0]; b += gridDim.x) {
    const uint32_t prim = p.big[b];
    Foot f;
    footprint(p, prim, f);
    const uint32_t rows = foot_rows(p, f);
    uint32_t s = 0;
    for (uint32_t r = threadIdx.x; r < rows; r += kBlock) s += row_entries<false>(p, f, prim, r, 0, 0);
    const uint32_t t = block_sum(s, red);
    if (threadIdx.x == 0) p.count[prim] = t;
  }
}

__global__ __launch_bounds__(256) void emit_kernel(BP p) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  if (p.count[prim] == 0) return;
  Foot f;
  footprint(p, prim, f);
  if (f.never || f.global || foot_is_big(p, f)) return;  // big: big_emit_kernel
  uint64_t at = p.off[prim];
  const uint64_t lim = at + p.count[prim];
  const uint32_t rows = foot_rows(p, f);
  for (uint32_t r = 0; r < rows; r++) at += row_entries<true>(p, f, prim, r, at, lim);
}

// one workgroup per big footprint: 256 rows at a time, each row's entries at
// its exclusive prefix within the block
__global__ __launch_bounds__(256) void big_emit_kernel(BP p) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t b = blockIdx.x; b < p.ctr[0]; b += gridDim.x) {
    const uint32_t prim = p.big[b];
    Foot f;
    footprint(p, prim, f);
    const uint32_t rows = foot_rows(p, f);
    uint64_t base = p.off[prim];
    const uint64_t lim = base + p.count[prim];
    for (uint32_t r0 = 0; r0 < rows; r0 += kBlock) {
      const uint32_t r = r0 + threadIdx.x;
      const uint32_t c = r < rows ? row_entries<false>(p, f, prim, r, 0, 0) : 0u;
      uint32_t incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      if (lane == 63) wsum[wid] = incl;
      __syncthreads();
      uint32_t woff = 0, tot = 0;
      for (int w = 0; w < kBlock / 64; w++) {
        if (w < wid) woff += wsum[w];
        tot += wsum[w];
      }
      if (c) row_entries<true>(p, f, prim, r, base + woff + incl - c, lim);
      base += tot;
      __syncthreads();
    }
  }
}

// sorted (cell, key) pairs and prims -> per-entry records with the key in
// the prim slot
__global__ __launch_bounds__(256) void rec_kernel(const unsigned long long* keys, const uint32_t* prim,
                                                  const float4* tri, uint32_t n, float4* rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* t = tri + 3 * (size_t)prim[i];
  float4 q2 = t[2];
  q2.y = unorder((uint32_t)keys[i]);
  rec[3 * (size_t)i] = t[0];
  rec[3 * (size_t)i + 1] = t[1];
  rec[3 * (size_t)i + 2] = q2;
}

// start[c] = the first entry of a cell >= c (binary search; empty cells get
// their successor's start), c = 0 .. ncell
__global__ __launch_bounds__(256) void start_kernel(const unsigned long long* keys, uint32_t n,
                                                    uint32_t ncell, uint32_t* start) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > ncell) return;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if ((uint32_t)(keys[mid] >> 32) < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  start[c] = lo;
}

}  // namespace rtl

struct LBDevice {
  uint32_t* start = nullptr;
  uint32_t* prim = nullptr;
  float* key = nullptr;
  float4* rec = nullptr;
  uint32_t* global = nullptr;
  unsigned long long entries = 0, cells = 0, nglobal = 0, never = 0, band = 0;
};

static void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

extern "C" void rt_lightbuf_free(LBDevice* d) {
  if (!d) return;
  (void)hipFree(d->start);
  (void)hipFree(d->prim);
  (void)hipFree(d->key);
  (void)hipFree(d->rec);
  (void)hipFree(d->global);
  delete d;
}

extern "C" void rt_lightbuf_sizes(const LBDevice* d, unsigned long long* entries, unsigned long long* cells,
                                  unsigned long long* global) {
  *entries = d ? d->entries : 0;
  *cells = d ? d->cells : 0;
  *global = d ? d->nglobal : 0;
}

extern "C" void rt_lightbuf_proof_counts(const LBDevice* d, unsigned long long* never, unsigned long long* band) {
  *never = d ? d->never : 0;
  *band = d ? d->band : 0;
}

#define LB_TRY(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      snprintf(err, errlen, "%s: %s", #x, hipGetErrorString(e_));                     \
      rc = e_ == hipErrorOutOfMemory ? 1 : -1;                                        \
      goto done;                                                                      \
    }                                                                                 \
  } while (0)

// The build's parameters (shared by the device build and the host survey):
// the DIR grid's float axes and extent, the POINT cube map's side.
static int bp_setup(const LBParams* in, rtl::BP& p, RtLightBuf* out, uint64_t& ncell, char* err, size_t errlen) {
  using namespace rtl;
  std::memset(&p, 0, sizeof p);
  std::memset(out, 0, sizeof *out);
  p.tri = in->tri;
  p.nprim = in->nprim;
  p.kind = in->kind;
  p.proven = in->proven ? 1u : 0u;
  for (int a = 0; a < 3; a++) {
    p.lv[a] = in->lv[a];
    p.olo[a] = in->box_lo[a];
    p.ohi[a] = in->box_hi[a];
  }
  p.slack = in->slack;
  p.s1 = in->s1;
  p.dmax = in->dmax;
  if (in->kind == RT_LB_DIR) {
    // axes: w = normalize(-l.v) (the rays' direction), u, v completing it;
    // rounded to float once -- the build and the query use the same floats
    double w[3] = {-in->lv[0], -in->lv[1], -in->lv[2]};
    const double wl = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!(wl > 0.0)) {
      snprintf(err, errlen, "directional light with a zero vector");
      return 1;  // no grid: its queries walk (the walk takes any direction)
    }
    for (int a = 0; a < 3; a++) {
      p.d[a] = (double)(float)(-in->lv[a]);  // the rays' direction, exactly (cpu/light.c:53)
      w[a] /= wl;
    }
    p.dlen = sqrt(p.d[0] * p.d[0] + p.d[1] * p.d[1] + p.d[2] * p.d[2]);
    int m = 0;
    for (int a = 1; a < 3; a++)
      if (fabs(w[a]) < fabs(w[m])) m = a;
    double e[3] = {0, 0, 0}, u[3], v[3];
    e[m] = 1.0;
    cross3(w, e, u);
    const double ul = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (int a = 0; a < 3; a++) u[a] /= ul;
    cross3(w, u, v);
    for (int a = 0; a < 3; a++) {
      out->u[a] = (float)u[a];
      out->v[a] = (float)v[a];
      out->w[a] = (float)w[a];
      p.u[a] = out->u[a];
      p.v[a] = out->v[a];
      p.w[a] = out->w[a];
    }
    {
      double su = 0.0, sv = 0.0;
      for (int a = 0; a < 3; a++) {
        su += p.u[a] * p.d[a] / p.dlen;
        sv += p.v[a] * p.d[a] / p.dlen;
      }
      p.skew = (fmax(fabs(su), fabs(sv)) + 1e-15) * 1.01;
    }
    // grid over the projected scene box (in->lv unused beyond the axes)
    const double m0 = in->slack + 3.0 * kEps * in->s1 * 1.01 + 1e-9 * in->s1;
    double lu = 1e300, hu = -1e300, lv2 = 1e300, hv2 = -1e300;
    for (int c = 0; c < 8; c++) {
      const double X[3] = {(c & 1) ? in->box_hi[0] : in->box_lo[0], (c & 2) ? in->box_hi[1] : in->box_lo[1],
                           (c & 4) ? in->box_hi[2] : in->box_lo[2]};
      const double a = X[0] * p.u[0] + X[1] * p.u[1] + X[2] * p.u[2];
      const double b = X[0] * p.v[0] + X[1] * p.v[1] + X[2] * p.v[2];
      lu = fmin(lu, a);
      hu = fmax(hu, a);
      lv2 = fmin(lv2, b);
      hv2 = fmax(hv2, b);
    }
    lu -= 2.0 * m0;
    lv2 -= 2.0 * m0;
    hu += 2.0 * m0;
    hv2 += 2.0 * m0;
    const double A = (hu - lu) * (hv2 - lv2);
    double cs = sqrt(A / (double)(in->target_cells ? in->target_cells : 1u));
    if (!(cs > 0.0)) cs = 1.0;
    p.nx = (uint32_t)fmin(16384.0, ceil((hu - lu) / cs) + 1.0);
    p.ny = (uint32_t)fmin(16384.0, ceil((hv2 - lv2) / cs) + 1.0);
    cs = fmax(cs, fmax((hu - lu) / (p.nx - 1), (hv2 - lv2) / (p.ny - 1)));
    out->u0 = (float)lu;
    out->v0 = (float)lv2;
    out->inv_cs = (float)(1.0 / cs);
    p.u0 = out->u0;
    p.v0 = out->v0;
    p.inv_cs = out->inv_cs;  // the float the query multiplies by
    p.cs = 1.0 / p.inv_cs;
    out->nx = p.nx;
    out->ny = p.ny;
    ncell = (uint64_t)p.nx * p.ny;
  } else {
    uint32_t n = (uint32_t)ceil(sqrt((double)(in->target_cells ? in->target_cells : 6u) / 6.0));
    if (n < 1) n = 1;
    if (n > 8192) n = 8192;
    p.n = n;
    out->nx = out->ny = n;
    out->half_n = 0.5f * (float)n;
    ncell = 6ull * n * n;
  }
  out->kind = in->kind;
  out->proven = p.proven;
  for (int a = 0; a < 3; a++) {  // rounded inward: a float inside is inside the build's box
    float lo = (float)in->box_lo[a], hi = (float)in->box_hi[a];
    if ((double)lo < in->box_lo[a]) lo = std::nextafter(lo, 3.0e38f);
    if ((double)hi > in->box_hi[a]) hi = std::nextafter(hi, -3.0e38f);
    out->olo[a] = lo;
    out->ohi[a] = hi;
  }
  if (ncell >= (1ull << 31)) {
    snprintf(err, errlen, "light buffer of %llu cells", (unsigned long long)ncell);
    return 1;
  }
  return 0;
}

extern "C" int rt_lightbuf_build(const LBParams* in, RtLightBuf* out, LBDevice** devp, hipStream_t s,
                                 char* err, size_t errlen) {
  using namespace rtl;
  int rc = 0;
  BP p;
  uint64_t total = 0, ncell = 0;
  if (const int r = bp_setup(in, p, out, ncell, err, errlen)) return r;
  LBDevice* dev = new LBDevice();
  uint32_t* count = nullptr;
  uint32_t* off = nullptr;
  uint32_t* ctr = nullptr;
  uint32_t* big = nullptr;
  uint32_t* rmin = nullptr;
  unsigned long long *k0 = nullptr, *k1 = nullptr;
  uint32_t* v0 = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  uint32_t hc[5] = {0, 0, 0, 0, 0}, last_off = 0, last_cnt = 0;
  const uint32_t np = in->nprim;
  const dim3 gp((np + 255) / 256), bk(256);
  LB_TRY(hipMalloc((void**)&count, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&off, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&ctr, 5 * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&big, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->global, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->start, (ncell + 1) * sizeof(uint32_t)));
  LB_TRY(hipMemsetAsync(ctr, 0, 5 * sizeof(uint32_t), s));
  LB_TRY(hipMemsetAsync(count + np, 0, sizeof(uint32_t), s));
  p.count = count;
  p.off = off;
  p.ctr = ctr;
  p.big = big;
  p.global = dev->global;
  if (p.proven && p.kind == RT_LB_POINT) {
    // the nearest shadow-ray origin's distance from the light (band widths)
    LB_TRY(hipMalloc((void**)&rmin, sizeof(uint32_t)));
    LB_TRY(hipMemsetAsync(rmin, 0x7f, sizeof(uint32_t), s));  // 0x7f7f7f7f: a large float
    if (np) hipLaunchKernelGGL(rmin_kernel, gp, bk, 0, s, p, rmin);
    LB_TRY(hipGetLastError());
    uint32_t rb = 0;
    LB_TRY(hipMemcpyAsync(&rb, rmin, sizeof rb, hipMemcpyDeviceToHost, s));
    LB_TRY(hipStreamSynchronize(s));
    float rf;
    std::memcpy(&rf, &rb, sizeof rf);
    p.rmin_o = (double)rf;
  }
  if (np) hipLaunchKernelGGL(count_kernel, gp, bk, 0, s, p);
  LB_TRY(hipGetLastError());
  hipLaunchKernelGGL(big_count_kernel, dim3(2048), bk, 0, s, p);
  LB_TRY(hipGetLastError());
  LB_TRY(rocprim::exclusive_scan(nullptr, tb, count, off, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), s));
  LB_TRY(hipMalloc(&tmp, tb + 16));
  LB_TRY(rocprim::exclusive_scan(tmp, tb, count, off, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), s));
  LB_TRY(hipMemcpyAsync(hc, ctr, sizeof hc, hipMemcpyDeviceToHost, s));
  if (np) {
    LB_TRY(hipMemcpyAsync(&last_off, off + np - 1, sizeof last_off, hipMemcpyDeviceToHost, s));
    LB_TRY(hipMemcpyAsync(&last_cnt, count + np - 1, sizeof last_cnt, hipMemcpyDeviceToHost, s));
  }
  LB_TRY(hipStreamSynchronize(s));
  total = (uint64_t)last_off + last_cnt;  // the 32-bit scan wrapped if the true total is >= 2^32
  {
    // a wrapped scan would show as offsets going down: check the exact sum on the host side
    // through the per-prim maximum (each count <= ncell < 2^31) and np
    if ((uint64_t)np * (uint64_t)ncell >= (1ull << 32)) {
      // possible overflow: recount in 64 bits
      unsigned long long sum = 0;
      std::vector<uint32_t> hcnt(np);
      LB_TRY(hipMemcpy(hcnt.data(), count, (size_t)np * sizeof(uint32_t), hipMemcpyDeviceToHost));
      for (uint32_t i = 0; i < np; i++) sum += hcnt[i];
      total = sum;
    }
  }
  if (total >= (1ull << 31) || (in->max_entries && total > in->max_entries)) {
    snprintf(err, errlen, "light buffer of %llu entries", (unsigned long long)total);
    rc = 1;
    goto done;
  }
  dev->entries = total;
  dev->cells = ncell;
  dev->nglobal = hc[1];
  dev->never = hc[2];
  dev->band = hc[3];
  LB_TRY(hipMalloc((void**)&dev->prim, (total + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->rec, (total + 1) * 3 * sizeof(float4)));
  if (total) {
    LB_TRY(hipMalloc((void**)&k0, total * sizeof(unsigned long long)));
    LB_TRY(hipMalloc((void**)&k1, total * sizeof(unsigned long long)));
    LB_TRY(hipMalloc((void**)&v0, total * sizeof(uint32_t)));
    p.keys = k0;
    p.vals = v0;
    hipLaunchKernelGGL(emit_kernel, gp, bk, 0, s, p);
    LB_TRY(hipGetLastError());
    if (hc[0]) {
      hipLaunchKernelGGL(big_emit_kernel, dim3(hc[0] < 4096 ? hc[0] : 4096), bk, 0, s, p);
      LB_TRY(hipGetLastError());
    }
    int bits = 32;
    while ((1ull << (bits - 32)) <= ncell) bits++;
    size_t sb = 0;
    LB_TRY(rocprim::radix_sort_pairs(nullptr, sb, k0, k1, v0, dev->prim, (size_t)total, 0, bits, s));
    if (sb > tb) {
      (void)hipFree(tmp);
      tmp = nullptr;
      LB_TRY(hipMalloc(&tmp, sb + 16));
      tb = sb;
    }
    sb = tb;
    LB_TRY(rocprim::radix_sort_pairs(tmp, sb, k0, k1, v0, dev->prim, (size_t)total, 0, bits, s));
    hipLaunchKernelGGL(rec_kernel, dim3((uint32_t)((total + 255) / 256)), bk, 0, s, k1, dev->prim, p.tri,
                       (uint32_t)total, dev->rec);
    LB_TRY(hipGetLastError());
    hipLaunchKernelGGL(start_kernel, dim3((uint32_t)((ncell + 256) / 256)), bk, 0, s, k1, (uint32_t)total,
                       (uint32_t)ncell, dev->start);
    LB_TRY(hipGetLastError());
  } else {
    LB_TRY(hipMemsetAsync(dev->start, 0, (ncell + 1) * sizeof(uint32_t), s));
  }
  LB_TRY(hipMemcpyAsync(hc + 4, ctr + 4, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  LB_TRY(hipStreamSynchronize(s));
  if (hc[4]) {
    snprintf(err, errlen, "light buffer emission disagreed with its count");
    rc = -1;
    goto done;
  }
  out->start = dev->start;
  out->rec = dev->rec;
  out->global = dev->global;
  out->nglobal = hc[1];
done:
  (void)hipFree(count);
  (void)hipFree(off);
  (void)hipFree(ctr);
  (void)hipFree(big);
  (void)hipFree(rmin);
  (void)hipFree(k0);
  (void)hipFree(k1);
  (void)hipFree(v0);
  (void)hipFree(tmp);
  if (rc) {
    rt_lightbuf_free(dev);
    std::memset(out, 0, sizeof *out);
    *devp = nullptr;
  } else {
    *devp = dev;
  }
  return rc;
}

// Host survey of a build (tests, tools; no device): the same footprints,
// counted on the CPU for every stride-th prim of in->tri (HOST prim-order
// records).  out: [0] entries, [1] never accepted, [2] global, [3] band
// prims, [4] big prims, [5] prims surveyed, [6] entries in band rows,
// [7] largest per-prim count, [8] its prim, [9] entries of prims with > 1024,
// [10] entries of prims with 65..1024, [11] prims with > 64.
extern "C" int rt_lightbuf_survey_host(const LBParams* in, uint32_t stride, unsigned long long out[12], char* err,
                                       size_t errlen) {
  using namespace rtl;
  BP p;
  RtLightBuf lb;
  uint64_t ncell = 0;
  if (bp_setup(in, p, &lb, ncell, err, errlen)) return -1;
  if (p.proven && p.kind == RT_LB_POINT) {
    double m = 1e300;
    for (uint32_t i = 0; i < p.nprim; i++) m = fmin(m, prim_rmin(p, i));
    p.rmin_o = p.nprim ? (double)(float)m : 0.0;
    if (p.rmin_o > m) p.rmin_o = std::nextafter((float)m, 0.0f);  // rounded down, as the device does
  }
  for (int k = 0; k < 12; k++) out[k] = 0;
  if (!stride) stride = 1;
  for (uint32_t prim = 0; prim < p.nprim; prim += stride) {
    Foot f;
    footprint(p, prim, f);
    out[5]++;
    if (f.never) {
      out[1]++;
      continue;
    }
    if (f.global) {
      out[2]++;
      continue;
    }
    if (f.band) out[3]++;
    if (foot_is_big(p, f)) out[4]++;
    const uint32_t rows = foot_rows(p, f);
    uint64_t c = 0;
    for (uint32_t r = 0; r < rows; r++) {
      const uint32_t e = row_entries<false>(p, f, prim, r, 0, 0);
      c += e;
      if (f.band && r >= rows - 6u * p.n) out[6] += e;
    }
    out[0] += c;
    if (c > 1024) out[9] += c;
    if (c > 64 && c <= 1024) out[10] += c;
    if (c > 64) out[11]++;
    if (c > out[7]) {
      out[7] = c;
      out[8] = prim;
    }
  }
  return 0;
}
