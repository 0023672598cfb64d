// rt_cand.hip -- per-frame camera-ray candidate lists: the part of the
// closest-hit decision of camera rays that the octree's culling slack cannot
// guarantee (DESIGN.md §2 "Exact camera rays").
//
// cpu/rt tests every triangle for every ray in float (/root/reference/cpu/
// hit.c:15-33, 72-91).  For a ray nearly parallel to a triangle's plane that
// float test accepts crossings far outside the triangle, so a walk that culls
// by the exact geometry can lose the reference's winner.  The forward error
// bound of the float test (tools/mt_bound.py, checked there against the float
// test itself) says: a float accept implies the exact line crosses the
// triangle's plane inside the expanded triangle
//     T_D = { v0 + U e1 + V e2 : U >= -du, V >= -dv, U + V <= 1 + dw }
// with du, dv, dw ~ eps |o - v0| |e| / |a|, |a| = |d| |e1 x e2| |cos|.
// Camera rays all pass (within dline) through the eye, so for a triangle the
// grazing cosine of every camera ray near it is bounded below by
// (distance of the eye from the plane) / (distance to the eye); that bound
// gives T_D per triangle.  If T_D lies within the walk's slack of the
// triangle the walk finds it (the triangle is "safe"); otherwise T_D is
// projected through the eye onto the image plane (it is planar, so its
// footprint is the triangle of its projected corners), widened by the float
// deviation of camera lines, and rasterised into the 8x8 tiles of this rank.
// Triangles with an unbounded footprint (T_D reaching the eye plane) go to a
// global list every camera ray tests.  Count pass -> rocPRIM exclusive scan
// -> fill pass; the render kernel tests each tile's list after its walk with
// the reference's exact arithmetic (consider()).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>  // rocPRIM's iterators use memset

#include <rocprim/rocprim.hpp>

#include "rt_cand.h"
#include "rt_tiles.h"

namespace rtc {

constexpr double kEps = 0x1p-24;             // float unit roundoff
constexpr double kAMin = 9.99999997e-08;     // (double)(float)1e-7, cpu/hit.c:7
constexpr double kDMin = 1.0 - 4.0 * kEps;   // |normalize(.)| of a float vector
constexpr double kDMax = 1.0 + 4.0 * kEps;

#define RTC_FN __host__ __device__ __forceinline__

RTC_FN double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
RTC_FN double norm3(const double* a) { return sqrt(dot3(a, a)); }
RTC_FN double dist3(const double* a, const double* b) {
  double x = a[0] - b[0], y = a[1] - b[1], z = a[2] - b[2];
  return sqrt(x * x + y * y + z * z);
}

enum { SAFE = 0, FOOTPRINT = 1, GLOBAL = 2 };

// The camera samples a triangle can be a float-MT candidate for, as a
// superset: (projected T_D widened by dimg, if tri_ok) intersected with the
// band of lines nearly parallel to the triangle's plane, |b0 + b1 k + b2 l|
// <= hw (b = n . (pos - o(k, l)), world units); plus, for very large
// triangles whose |a| error can reach the 1e-7 threshold, the thinner band
// hw0 of the lines too parallel to bound (c_ok > 0).
struct Footprint {
  int tri_ok;
  double k[3], l[3], dimg;
  double b0, b1, b2, hw, hw0;
  float skip;  // lower bound of (float new_dist) - |pos - o| over the candidate crossings
};

// point-triangle distance (double): closest point by the edge/interior cases
RTC_FN double pt_tri_dist(const double* x, const double* a, const double* b, const double* c) {
  double ab[3], ac[3], ax[3];
  for (int i = 0; i < 3; i++) {
    ab[i] = b[i] - a[i];
    ac[i] = c[i] - a[i];
    ax[i] = x[i] - a[i];
  }
  const double n[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2],
                       ab[0] * ac[1] - ab[1] * ac[0]};
  const double nn = dot3(n, n);
  if (nn > 0.0) {  // interior: barycentrics of the projection
    double t[3] = {ab[1] * ax[2] - ab[2] * ax[1], ab[2] * ax[0] - ab[0] * ax[2],
                   ab[0] * ax[1] - ab[1] * ax[0]};
    double s[3] = {ax[1] * ac[2] - ax[2] * ac[1], ax[2] * ac[0] - ax[0] * ac[2],
                   ax[0] * ac[1] - ax[1] * ac[0]};
    const double inn = 1.0 / nn;  // (an ulp of the barycentrics: the edge cases take over)
    const double v = dot3(t, n) * inn, u = dot3(s, n) * inn;
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
    double z[3] = {w[0] - t * d[0], w[1] - t * d[1], w[2] - t * d[2]};
    best = fmin(best, norm3(z));
  }
  return best;
}

// Classify one triangle (record r: v0, e1, e2 as floats) and build its footprint.
// td (optional, FOOTPRINT only): the bounding box of T_D(cl) (lo xyz, hi xyz)
// and the distance error derr; td[6] = -1 when T_D has no bound for every
// candidate line (c_ok > 0).
RTC_FN int classify(const CandParams& p, const float* r, const float* leafbox, Footprint& fp,
                    double* td = nullptr, int* why = nullptr) {
  const double v0[3] = {r[0], r[1], r[2]}, e1[3] = {r[3], r[4], r[5]}, e2[3] = {r[6], r[7], r[8]};
  const double v1[3] = {v0[0] + e1[0], v0[1] + e1[1], v0[2] + e1[2]};
  const double v2[3] = {v0[0] + e2[0], v0[1] + e2[1], v0[2] + e2[2]};
  const double l1 = norm3(e1), l2 = norm3(e2);
  const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                       e1[0] * e2[1] - e1[1] * e2[0]};
  const double nl = norm3(n);
  double e_a = p.c_a * kEps * l1 * l2 * kDMax;
  if (nl * kDMax + e_a < kAMin) {  // |a| < 1e-7 for every ray: never accepted
    if (why) *why = 0;
    return SAFE;
  }
  const double inl = 1.0 / nl;  // (the unit normal to an ulp or two: inside every margin below)
  const double nh[3] = {n[0] * inl, n[1] * inl, n[2] * inl};
  const double pv[3] = {p.pos[0] - v0[0], p.pos[1] - v0[1], p.pos[2] - v0[2]};
  const double deye = fabs(dot3(nh, pv));
  const double smax = p.lmax + norm3(pv);  // |o - v0| <= |o - pos| + |pos - v0|
  double e_sh = p.c_dot * kEps * smax * kDMax * l2;
  double e_dq = p.c_dot * kEps * smax * kDMax * l1;
  double e_eq = p.c_dot * kEps * smax * l1 * l2;
  // lines with grazing cosine c: |a| >= a_lb(c); the bound of
  // tools/mt_bound.py needs rho = e_a / a_lb < 1/2, i.e. c >= c_ok
  const double c_ok = kAMin >= 2.0 * e_a ? 0.0 : 3.0 * e_a / (kDMin * nl);
  auto alb = [&](double c) { return fmax(kAMin, kDMin * nl * c - e_a); };
  double P[3][3];
  // T_D(c) corners; returns how far they reach beyond the triangle
  // (two divisions instead of five: the products differ from the quotients
  // by an ulp or two, far inside the bound's own slack -- its constants are
  // rounded up by 1.3 %, tools/mt_bound.py)
  auto expand = [&](double c, double& rho_o, double& a_o) {
    const double a = alb(c), ia = 1.0 / a, rho = e_a * ia, i1r = 1.0 / (1.0 - rho);
    const double du = e_sh * ia * i1r, dv = e_dq * ia * i1r;
    const double dw = (4.0 * kEps + (e_sh + e_dq) * ia + rho) * i1r;
    for (int k = 0; k < 3; k++) {
      P[0][k] = v0[k] - du * e1[k] - dv * e2[k];
      P[1][k] = v0[k] + (1.0 + dw + dv) * e1[k] - dv * e2[k];
      P[2][k] = v0[k] - du * e1[k] + (1.0 + dw + du) * e2[k];
    }
    rho_o = rho;
    a_o = a;
    return fmax(dist3(P[0], v0), fmax(dist3(P[1], v1), dist3(P[2], v2)));
  };
  // K' >= c H(c) over every c >= c_ok: with a_lb = dmin nl c - e_a, c H(c)
  // is a convex rational function of c, so its maximum is at an end point
  double rho = 0.0, a_lb = 0.0, kmax_ch;
  const double ck = fmax(c_ok, (kAMin + e_a) / (kDMin * nl));  // kink of a_lb(c)
  {
    double rr, aa;
    kmax_ch = fmax(fmin(ck, 1.0) * expand(fmin(ck, 1.0), rr, aa), expand(1.0, rr, aa));
  }
  // smallest grazing cosine of a camera line through T_D: such a line
  // passes within dline of the eye, so c >= (deye - dline) / (|X - pos| +
  // dline) with |X - pos| <= max |v - pos| + H(c), and c H(c) <= K'
  double vmax = 0.0;
  {
    const double* V[3] = {v0, v1, v2};
    for (int k = 0; k < 3; k++) vmax = fmax(vmax, dist3(V[k], p.pos));
  }
  double cl = fmax(c_ok, (deye - p.dline - kmax_ch) / (vmax + p.dline));
  double hreach = expand(cl, rho, a_lb);
  // Second round, componentwise (tools/mt_bound.py stress_cw): every
  // candidate line crosses T_D, so its direction lies in the cone from the
  // eye to T_D's bounding sphere, which bounds each |d_i| and |S_i| =
  // |o_i - v0_i| <= lmax |d_i| + |pos_i - v0_i|; the sums
  //   E_sh <= 6.01 eps sum |S_i| M_i,  M_i = |d_j| |e2_k| + |d_k| |e2_j|
  //   E_dq <= 6.01 eps sum |d_i| N_i,  N_i = |S_j| |e1_k| + |S_k| |e1_j|
  //   E_eq <= 6.01 eps sum |e2_i| N_i, E_a <= 5.01 eps sum |e1_i| M_i
  // are much smaller than their Cauchy-Schwarz versions for camera rays.
  if (c_ok == 0.0) {
    double q[3], qr = 0.0;
    for (int a = 0; a < 3; a++) q[a] = (P[0][a] + P[1][a] + P[2][a]) / 3.0;
    for (int k = 0; k < 3; k++) qr = fmax(qr, dist3(P[k], q));
    const double R = dist3(q, p.pos);
    if (R > 2.0 * (qr + p.dline)) {
      const double iR = 1.0 / R;
      const double st = (qr + p.dline) * iR * 1.42 + 8.0 * kEps;  // |d - q^| <= 2 sin(theta / 2)
      double dm[3], sm[3], ae1[3], ae2[3];
      for (int a = 0; a < 3; a++) {
        dm[a] = fmin(1.0, fabs(q[a] - p.pos[a]) * iR + st) * kDMax;
        sm[a] = ((p.lmax + p.dline) * dm[a] + fabs(pv[a]) + p.dline) * (1.0 + 1e-9);
        ae1[a] = fabs(e1[a]);
        ae2[a] = fabs(e2[a]);
      }
      double M[3], N[3];
      for (int i = 0; i < 3; i++) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        M[i] = dm[j] * ae2[k] + dm[k] * ae2[j];
        N[i] = sm[j] * ae1[k] + sm[k] * ae1[j];
      }
      const double cw = p.c_dot / 8.6 * 6.01 * kEps, ca = p.c_a / 7.2 * 5.01 * kEps;
      const double w_sh = cw * (sm[0] * M[0] + sm[1] * M[1] + sm[2] * M[2]);
      const double w_dq = cw * (dm[0] * N[0] + dm[1] * N[1] + dm[2] * N[2]);
      const double w_eq = cw * (ae2[0] * N[0] + ae2[1] * N[1] + ae2[2] * N[2]);
      const double w_a = ca * (ae1[0] * M[0] + ae1[1] * M[1] + ae1[2] * M[2]);
      if (w_sh < e_sh) e_sh = w_sh;
      if (w_dq < e_dq) e_dq = w_dq;
      if (w_eq < e_eq) e_eq = w_eq;
      if (w_a < e_a) e_a = w_a;
      double rr, aa;
      const double ck2 = fmax(c_ok, (kAMin + e_a) / (kDMin * nl));
      kmax_ch = fmax(fmin(ck2, 1.0) * expand(fmin(ck2, 1.0), rr, aa), expand(1.0, rr, aa));
      cl = fmax(cl, (deye - p.dline - kmax_ch) / (vmax + p.dline));
      hreach = expand(cl, rho, a_lb);
    }
  }
  const double rmax = fmax(dist3(P[0], p.pos), fmax(dist3(P[1], p.pos), dist3(P[2], p.pos)));
  const double derr = kDMax * e_eq / (a_lb * (1.0 - rho)) +
                      (rmax + p.lmax) * (rho + 4.0 * kEps) / (1.0 - rho) +
                      4.0 * kEps * (p.omax + rmax + p.lmax);
  // safe: every crossing point lies within the slack of the box of a leaf
  // holding the triangle (so the walk visits that leaf and tests it), and
  // the float distance error cannot push it past the walk's pruning
  if (c_ok == 0.0 && derr <= 2.0 * p.eps_avail) {
    if (hreach <= p.eps_avail) {
      if (why) *why = 1;
      return SAFE;
    }
    if (leafbox) {
      const double e = p.eps_avail;
      bool in = true;
      for (int k = 0; k < 3 && in; k++)
        for (int a = 0; a < 3 && in; a++)
          in = P[k][a] >= (double)leafbox[a] - e && P[k][a] <= (double)leafbox[4 + a] + e;
      if (in) {
        if (why) *why = 2;
        return SAFE;
      }
    }
  }
  // band: a candidate line at cosine c crosses the plane |h'| / c from a
  // point within dline of the eye, within H(c) of the triangle, so
  // c (r_T - dline) - (deye + dline) <= c H(c) <= K' (max over c >= c_ok)
  const double rT = pt_tri_dist(p.pos, v0, v1, v2);
  if (!(rT > 2.0 * p.dline + 1e-9)) return GLOBAL;
  const double c_band = fmin(1.0, (deye + p.dline + kmax_ch) / (rT - p.dline));
#ifndef RT_CAND_CMIN
#define RT_CAND_CMIN 1
#endif
#if RT_CAND_CMIN
  // cpu/hit.c:19-20 rejects |a| < 1e-7, and |a| <= kDMax nl c + e_a: no
  // line with c < c_min is accepted.  Every candidate line has c <= c_band,
  // so c_min > c_band leaves none (with c_ok > 0 the lines below c_ok are
  // unbounded and c_min < c_ok: no exit there)
  if (c_ok == 0.0 && (kAMin - e_a) > c_band * (kDMax * nl) * (1.0 + 1e-6)) {
    if (why) *why = 3;
    return SAFE;
  }
#endif
#if defined(RT_SURVEY_DUMP) && !defined(__HIP_DEVICE_COMPILE__)
  if (td) {
    td[7] = nl; td[8] = deye; td[9] = rT; td[10] = c_band; td[11] = (kAMin - e_a) / (kDMax * nl);
    td[12] = cl; td[13] = hreach; td[14] = kmax_ch; td[15] = e_a; td[16] = e_sh; td[17] = a_lb;
  }
#endif
  const double wide = p.lmax + p.dline + p.dorig;
  fp.b0 = dot3(nh, p.pos) - dot3(nh, p.C);
  fp.b1 = -dot3(nh, p.u);
  fp.b2 = -dot3(nh, p.v);
  fp.hw = c_band * wide + p.dline + p.dorig + 1e-9 * wide;
  fp.hw0 = c_ok > 0.0 ? c_ok * wide + p.dline + p.dorig + 1e-9 * wide : -1.0;
  // the projected T_D, valid when it stays on one side of the eye plane
  fp.tri_ok = 0;
  double yn[3];
  for (int k = 0; k < 3; k++) {
    const double Y[3] = {P[k][0] - p.pos[0], P[k][1] - p.pos[1], P[k][2] - p.pos[2]};
    yn[k] = dot3(Y, p.n);
  }
  const double rmin = pt_tri_dist(p.pos, P[0], P[1], P[2]);
  const double ymag = rmax + 1.0;
  if (rmin > 1e-6 && (fmin(yn[0], fmin(yn[1], yn[2])) > 1e-9 * ymag ||
                      fmax(yn[0], fmax(yn[1], yn[2])) < -1e-9 * ymag)) {
    fp.tri_ok = 1;
    for (int k = 0; k < 3; k++) {
      const double lam = p.plane / yn[k];
      double w[3];
      for (int c = 0; c < 3; c++) w[c] = p.pos[c] + lam * (P[k][c] - p.pos[c]) - p.C[c];
      const double b1 = dot3(w, p.u), b2 = dot3(w, p.v);
      fp.k[k] = p.ginv[0] * b1 + p.ginv[1] * b2;
      fp.l[k] = p.ginv[1] * b1 + p.ginv[2] * b2;
    }
    // a float camera line through X passes within dline of the eye: at the
    // image plane it lands within dline (1 + lmax / |X - pos|) of X's projection
    fp.dimg = 1.5 * p.gscale * (p.dline * (1.0 + p.lmax / rmin) + p.dorig) + 1e-3;
  }
  // depth skip: new_dist >= |pos - o| + |X - pos| - 2 dline - derr
  const double sk = c_ok > 0.0 ? -1e30 : rmin - 2.0 * p.dline - derr - 1e-6 * (p.lmax + rmax) - 1e-3;
  fp.skip = sk > 0.0 ? (float)(sk * (1.0 - 1e-6)) : -1e30f;
  if (td) {
    for (int a = 0; a < 3; a++) {
      td[a] = fmin(P[0][a], fmin(P[1][a], P[2][a]));
      td[3 + a] = fmax(P[0][a], fmax(P[1][a], P[2][a]));
    }
    td[6] = c_ok > 0.0 ? -1.0 : derr;
  }
  return FOOTPRINT;
}

// This rank's tiles in tile row ty, columns [x0, x1] (csrc/rt_tiles.h).
__host__ __device__ inline uint32_t rank_tiles(const CandParams& p, int ty, int x0, int x1) {
  if (x0 > x1) return 0u;
  return rt_rank_row_tiles(ty, x0, x1, (uint32_t)p.nranks, (uint32_t)p.rank, (uint32_t)p.blocks_x,
                           (uint32_t)p.tb, nullptr);
}

// The pixel columns (rows: row = true) whose samples' k (l) can lie in
// [a, b], clamped to the frame (empty: c0 > c1).  cpu/rt: pixel c samples
// k in [W/2 - c, W/2 - c + 1/2] (cpu/raytracer.c:55-58);
// compatibility mode: pixel c is the one sample k = c - W/2.  Clamped in
// double before the conversion (a far-off footprint gives values beyond
// int range, whose conversion the host does not saturate).
__host__ __device__ inline void pixel_range(const CandParams& p, double a, double b, int& c0, int& c1, bool row) {
  const int n = row ? p.H : p.W;
  const double h = (double)(n / 2);
  if (p.compat) {
    c0 = (int)fmin(fmax(0.0, ceil(a + h)), (double)n);
    c1 = (int)fmax(fmin((double)(n - 1), floor(b + h)), -1.0);
  } else {
    c0 = (int)fmin(fmax(0.0, ceil(h - b)), (double)n);
    c1 = (int)fmax(fmin((double)(n - 1), floor(h - a + 0.5)), -1.0);
  }
}

// Can a footprint inside the ball (q, rb) -- every candidate crossing point
// of the triangle lies in it -- reach a tile of this rank?  The ball's
// bounding box projects (through the eye, on one side of the eye plane) into
// the image rectangle spanned by its corners' projections; widened by the
// float deviation of camera lines (classify's dimg) plus 2 pixels, it gives
// the pixel rows and columns the footprint can touch, clipped to the frame.
// false = none of this rank's tiles (off-frame, or between the rank's tiles
// of an interleaved split); true whenever unsure.
RTC_FN bool rank_may_touch(const CandParams& p, const double q[3], double rb) {
  // in float (the triangles that reach here are a third of the scene): the
  // corners must lie well in front of the eye (|Y . n| >= |Y| / 20, i.e.
  // within ~87 degrees of the view axis; anything else is kept), so the
  // projection's relative rounding stays below 1e-5 and its absolute error
  // below a pixel -- covered by the 3-pixel margin
  const float dq0 = (float)(q[0] - p.pos[0]), dq1 = (float)(q[1] - p.pos[1]),
              dq2 = (float)(q[2] - p.pos[2]);
  const float rbf = (float)rb;
  const float R = sqrtf(dq0 * dq0 + dq1 * dq1 + dq2 * dq2);
  if (!(R > 2.0f * rbf + 1e-6f)) return true;
  const float n0 = (float)p.n[0], n1 = (float)p.n[1], n2 = (float)p.n[2];
  const float u0 = (float)p.u[0], u1 = (float)p.u[1], u2 = (float)p.u[2];
  const float v0 = (float)p.v[0], v1 = (float)p.v[1], v2 = (float)p.v[2];
  const float pc0 = (float)(p.pos[0] - p.C[0]), pc1 = (float)(p.pos[1] - p.C[1]),
              pc2 = (float)(p.pos[2] - p.C[2]);
  const float plane = (float)p.plane, g0 = (float)p.ginv[0], g1 = (float)p.ginv[1],
              g2 = (float)p.ginv[2];
  const float ymin = 0.05f * (R + 1.8f * rbf);
  float kmn = 1e30f, kmx = -1e30f, lmn = 1e30f, lmx = -1e30f;
  int side = 0;
  for (int c = 0; c < 8; c++) {
    const float Y0 = dq0 + ((c & 1) ? rbf : -rbf), Y1 = dq1 + ((c & 2) ? rbf : -rbf),
                Y2 = dq2 + ((c & 4) ? rbf : -rbf);
    const float yn = Y0 * n0 + Y1 * n1 + Y2 * n2;
    const int sd = yn > ymin ? 1 : (yn < -ymin ? -1 : 0);
    if (sd == 0 || (side != 0 && sd != side)) return true;
    side = sd;
    const float lam = plane / yn;
    const float w0 = pc0 + lam * Y0, w1 = pc1 + lam * Y1, w2 = pc2 + lam * Y2;
    const float b1 = w0 * u0 + w1 * u1 + w2 * u2, b2 = w0 * v0 + w1 * v1 + w2 * v2;
    const float k = g0 * b1 + g1 * b2, l = g1 * b1 + g2 * b2;
    kmn = fminf(kmn, k);
    kmx = fmaxf(kmx, k);
    lmn = fminf(lmn, l);
    lmx = fmaxf(lmx, l);
  }
  const double m = 3.0 + 1.5 * p.gscale * (p.dline * (1.0 + p.lmax / ((double)R - 2.0 * rb)) + p.dorig) +
                   1e-5 * (fabs((double)kmn) + fabs((double)kmx) + fabs((double)lmn) + fabs((double)lmx));
  kmn -= m;
  kmx += m;
  lmn -= m;
  lmx += m;
  // samples of pixel (r, c): k in [W/2 - c, W/2 - c + 1/2], l likewise (raster_rows)
  int r0, r1, c0, c1;
  pixel_range(p, (double)kmn, (double)kmx, c0, c1, false);
  pixel_range(p, (double)lmn, (double)lmx, r0, r1, true);
  if (r0 > r1 || c0 > c1) return false;  // off the frame
  const uint32_t n = (uint32_t)p.nranks, rk = (uint32_t)p.rank;
  if (n == 1) return true;
  // whole tb x tb-tile blocks per rank, block (bx, by) -> rank (bx + by) mod
  // n (csrc/rt_tiles.h): a block column range of >= n blocks meets every
  // rank in every block row; otherwise one check per block row (the residues
  // of the rows repeat with period n)
  const int bx0 = (c0 >> 3) / p.tb, bx1 = (c1 >> 3) / p.tb;
  const int by0 = (r0 >> 3) / p.tb, by1 = (r1 >> 3) / p.tb;
  if ((uint32_t)(bx1 - bx0 + 1) >= n) return true;
  const int rows = by1 - by0 + 1 < (int)n ? by1 - by0 + 1 : (int)n;
  for (int k = 0; k < rows; k++) {
    const uint32_t res = rt_row_res((uint32_t)(by0 + k), n, rk);
    const uint32_t f = (uint32_t)bx0 <= res ? res : (uint32_t)bx0 + (res + n - (uint32_t)bx0 % n) % n;
    if (f <= (uint32_t)bx1) return true;
  }
  return false;
}

enum { Q_SAFE = 0, Q_LIST = 1, Q_AWAY = 2 };

#ifndef RT_QUICK_TIGHT
#define RT_QUICK_TIGHT 1
#endif

// Fast, conservative float version of classify()'s SAFE test (no leaf box):
// every quantity is a positive magnitude computed in a few float operations,
// bounded with explicit margins, so a true result is a proof on its own.
// Most triangles of a frame take this exit.  A triangle it cannot prove safe
// whose error region provably stays off this rank's tiles (rank_may_touch)
// is Q_AWAY: its footprint would be empty here, so it is not classified.
RTC_FN int quick_class(const CandParams& p, const float* r, float* dbg = nullptr) {
  const float fe = 5.9604645e-8f;
  const float e1x = r[3], e1y = r[4], e1z = r[5], e2x = r[6], e2y = r[7], e2z = r[8];
  const float l1 = sqrtf(e1x * e1x + e1y * e1y + e1z * e1z) * 1.00001f;
  const float l2 = sqrtf(e2x * e2x + e2y * e2y + e2z * e2z) * 1.00001f;
  const float nx = e1y * e2z - e1z * e2y, ny = e1z * e2x - e1x * e2z, nz = e1x * e2y - e1y * e2x;
  const float nl = sqrtf(nx * nx + ny * ny + nz * nz);
  // |n| and its direction carry an absolute error <= 4 eps |e1| |e2|
  const float nerr = 4.0f * fe * l1 * l2;
  if (!(nl > 64.0f * nerr)) return Q_LIST;
  const float nlo = nl - nerr;
  float e_a = (float)p.c_a * fe * l1 * l2 * 1.0001f;
  const float amin = 9.99999975e-08f;
  if (amin < 2.0f * e_a) return Q_LIST;
  const float px = (float)p.pos[0] - r[0], py = (float)p.pos[1] - r[1], pz = (float)p.pos[2] - r[2];
  const float pvl = sqrtf(px * px + py * py + pz * pz) * 1.00001f + 1e-6f;
  const float deye = fabsf(nx * px + ny * py + nz * pz) / nl;
  const float deye_lb = deye - pvl * (2.0f * nerr / nlo + 8.0f * fe) - 1e-6f;
  const float smax = ((float)p.lmax + pvl) * 1.00001f;
  float e_sh = (float)p.c_dot * fe * smax * l2 * 1.0001f;
  float e_dq = (float)p.c_dot * fe * smax * l1 * 1.0001f;
  float e_eq = (float)p.c_dot * fe * smax * l1 * l2 * 1.0001f;
  const float dmin = 1.0f - 4.0f * fe;
  // H(c) <= (du + dv + dw) (l1 + l2) with a = a_lb(c).  The quotients share
  // two IEEE reciprocals (this kernel is VALU-bound, a division is ~10
  // instructions): each product adds one rounding of a positive term (rho <=
  // 1/2 above), far inside the 1.0001 margin
  auto H = [&](float c, float& a_o, float& rho_o) {
    const float a = fmaxf(amin, (dmin * nlo * c - e_a) * 0.99999f);
    const float ra = 1.0f / a;
    const float rho = e_a * ra;
    const float rom = 1.0f / (1.0f - rho);
    const float du = e_sh * ra * rom, dv = e_dq * ra * rom;
    const float dw = (4.0f * fe + (e_sh + e_dq) * ra + rho) * rom;
    a_o = a;
    rho_o = rho;
    return (du + dv + dw) * (l1 + l2) * 1.0001f;
  };
  // H with the corners' own displacements (classify's expand: |du e1 + dv
  // e2|, |(dw + dv) e1 - dv e2|, |-du e1 + (dw + du) e2|) instead of their
  // common bound (du + dv + dw)(l1 + l2), which is up to ~2x larger: the
  // crossing region's reach, whose test below decides most triangles.  The
  // vectors' rounding is absolute (cancellation), so it is bounded by 8 eps
  // of the terms' magnitudes on top of the relative margin.
  auto Ht = [&](float c, float& a_o, float& rho_o) {
    const float a = fmaxf(amin, (dmin * nlo * c - e_a) * 0.99999f);
    const float ra = 1.0f / a;
    const float rho = e_a * ra;
    const float rom = 1.0f / (1.0f - rho);
    const float du = e_sh * ra * rom, dv = e_dq * ra * rom;
    const float dw = (4.0f * fe + (e_sh + e_dq) * ra + rho) * rom;
    a_o = a;
    rho_o = rho;
    const float p1 = dw + dv, p2 = dw + du;
    const float x0 = du * e1x + dv * e2x, y0 = du * e1y + dv * e2y, z0 = du * e1z + dv * e2z;
    const float x1 = p1 * e1x - dv * e2x, y1 = p1 * e1y - dv * e2y, z1 = p1 * e1z - dv * e2z;
    const float x2 = p2 * e2x - du * e1x, y2 = p2 * e2y - du * e1y, z2 = p2 * e2z - du * e1z;
    const float m = fmaxf(x0 * x0 + y0 * y0 + z0 * z0, fmaxf(x1 * x1 + y1 * y1 + z1 * z1, x2 * x2 + y2 * y2 + z2 * z2));
    return sqrtf(m) * 1.0002f + 8.0f * fe * (p1 + p2) * (l1 + l2);
  };
  float a, rho;
  const float ck = fminf(1.0f, (amin + e_a) / (dmin * nlo) * 1.0001f);
  const float kmax_ch = fmaxf(ck * H(ck, a, rho), H(1.0f, a, rho)) * 1.0001f;
  float vmax = 0.0f;
  for (int k = 0; k < 3; k++) {
    const float ox = k == 0 ? 0.0f : (k == 1 ? e1x : e2x), oy = k == 0 ? 0.0f : (k == 1 ? e1y : e2y),
                oz = k == 0 ? 0.0f : (k == 1 ? e1z : e2z);
    const float qx = px - ox, qy = py - oy, qz = pz - oz;
    vmax = fmaxf(vmax, sqrtf(qx * qx + qy * qy + qz * qz));
  }
  vmax = vmax * 1.00002f + 1e-6f;
  float num = deye_lb - (float)p.dline - kmax_ch - 1e-5f * (deye + kmax_ch);
  if (!(num > 0.0f)) return Q_LIST;
  float cl = num / (vmax + (float)p.dline) * 0.9999f;
  float h = H(cl, a, rho);
  // componentwise second round (see classify): the candidate lines cross
  // T_D, inside the ball (centroid, max vertex distance + h) -- with the
  // common bound h, so that the cone, and the componentwise error terms from
  // it, stay above classify()'s own (its ball is around T_D's corners):
  // every verdict here is one classify() also reaches (rt_cand_survey [80])
  const float cx = (e1x + e2x) / 3.0f, cy = (e1y + e2y) / 3.0f, cz = (e1z + e2z) / 3.0f;  // - v0
  float rv = sqrtf(cx * cx + cy * cy + cz * cz);  // max vertex distance from the centroid
  rv = fmaxf(rv, sqrtf((e1x - cx) * (e1x - cx) + (e1y - cy) * (e1y - cy) + (e1z - cz) * (e1z - cz)));
  rv = fmaxf(rv, sqrtf((e2x - cx) * (e2x - cx) + (e2y - cy) * (e2y - cy) + (e2z - cz) * (e2z - cz)));
  {
    float rq = (rv + h) * 1.0001f + 1e-6f + (float)p.dline;
    const float qx = cx - px, qy = cy - py, qz = cz - pz;  // centroid - pos
    const float R = sqrtf(qx * qx + qy * qy + qz * qz) * 0.99999f;
    if (R > 2.0f * rq) {
      const float rR = 1.0f / R;  // (one more rounding per quotient, inside the 1.00001 margins)
      const float st = rq * rR * 1.42f + 8.0f * fe + 1e-6f;
      const float d0 = fminf(1.0f, fabsf(qx) * rR + st) * 1.00001f;
      const float d1 = fminf(1.0f, fabsf(qy) * rR + st) * 1.00001f;
      const float d2 = fminf(1.0f, fabsf(qz) * rR + st) * 1.00001f;
      const float L = ((float)p.lmax + (float)p.dline) * 1.00001f, dl = (float)p.dline + 1e-6f;
      const float s0 = (L * d0 + fabsf(px) + dl) * 1.00001f;
      const float s1 = (L * d1 + fabsf(py) + dl) * 1.00001f;
      const float s2 = (L * d2 + fabsf(pz) + dl) * 1.00001f;
      const float a1x = fabsf(e1x), a1y = fabsf(e1y), a1z = fabsf(e1z);
      const float a2x = fabsf(e2x), a2y = fabsf(e2y), a2z = fabsf(e2z);
      const float M0 = d1 * a2z + d2 * a2y, M1 = d2 * a2x + d0 * a2z, M2 = d0 * a2y + d1 * a2x;
      const float N0 = s1 * a1z + s2 * a1y, N1 = s2 * a1x + s0 * a1z, N2 = s0 * a1y + s1 * a1x;
      const float cw = (float)(p.c_dot / 8.6 * 6.01) * fe * 1.0001f;
      const float ca = (float)(p.c_a / 7.2 * 5.01) * fe * 1.0001f;
      e_sh = fminf(e_sh, cw * (s0 * M0 + s1 * M1 + s2 * M2));
      e_dq = fminf(e_dq, cw * (d0 * N0 + d1 * N1 + d2 * N2));
      e_eq = fminf(e_eq, cw * (a2x * N0 + a2y * N1 + a2z * N2));
      e_a = fminf(e_a, ca * (a1x * M0 + a1y * M1 + a1z * M2));
      const float ck2 = fminf(1.0f, (amin + e_a) / (dmin * nlo) * 1.0001f);
      const float k2 = fmaxf(ck2 * H(ck2, a, rho), H(1.0f, a, rho)) * 1.0001f;
      const float num2 = deye_lb - (float)p.dline - k2 - 1e-5f * (deye + k2);
      if (num2 > 0.0f) cl = fmaxf(cl, num2 / (vmax + (float)p.dline) * 0.9999f);
      h = H(cl, a, rho);
    }
  }
  if (RT_QUICK_TIGHT) h = Ht(cl, a, rho);
  const float rmax = vmax + h;
  const float derr = (e_eq / (a * (1.0f - rho)) + (rmax + (float)p.lmax) * (rho + 4.0f * fe) / (1.0f - rho) +
                      4.0f * fe * ((float)p.omax + rmax + (float)p.lmax)) * 1.0001f;
  if (dbg) {
    dbg[0] = h;
    dbg[1] = derr;
    dbg[2] = cl;
    dbg[3] = a;
  }
  if (h <= (float)p.eps_avail * 0.9999f && derr <= 2.0f * (float)p.eps_avail * 0.9999f) return Q_SAFE;
  // T_D lies in the ball (centroid, rv + h): every corner of T_D is within
  // H(cl) of its vertex.  The centroid in double from the record's floats.
  const double q[3] = {(double)r[0] + (double)cx, (double)r[1] + (double)cy, (double)r[2] + (double)cz};
  const double rb = ((double)rv + (double)h) * 1.001 + 1e-5 + 1e-6 * (fabs(q[0]) + fabs(q[1]) + fabs(q[2]));
  return rank_may_touch(p, q, rb) ? Q_LIST : Q_AWAY;
}

// Tiles of this rank whose camera samples can be candidates for the
// triangle.  Pixel (r, c) samples k in [W/2 - c, W/2 - c + 1/2], l in
// [H/2 - r, H/2 - r + 1/2] (cpu/raytracer.c:55-58 with i = W/2 - c, j = H/2 -
// r).
// Pixel rows [r0, r1] the footprint can reach; false: none.
__host__ __device__ inline bool raster_rows(const CandParams& p, const Footprint& fp, int& r0, int& r1) {
  r0 = 0;
  r1 = p.H - 1;
  if (fp.tri_ok && fp.hw0 < 0.0) {
    const double lmn = fmin(fp.l[0], fmin(fp.l[1], fp.l[2])) - fp.dimg;
    const double lmx = fmax(fp.l[0], fmax(fp.l[1], fp.l[2])) + fp.dimg;
    if (!(lmx >= p.lmin && lmn <= p.lmax_)) return false;
    pixel_range(p, lmn, lmx, r0, r1, true);
  }
  return r0 <= r1;
}

// The footprint's tiles in tile row ty (rows clipped to [r0, r1]): tile
// columns [a0, a1] and [b0, b1] (empty when a0 > a1; the second range only
// counts where it leaves the first).
__host__ __device__ inline void row_tiles(const CandParams& p, const Footprint& fp, int ty, int r0,
                                          int r1, int& a0, int& a1, int& b0, int& b1) {
  const double hh = (double)(p.H / 2);
  auto cols = [&](double a, double b, int& c0, int& c1) {  // k in [a, b] -> columns
    pixel_range(p, a, b, c0, c1, false);
  };
  // k-range of a band |b0 + b1 k + b2 l| <= hw for some l in [la, lb]
  auto band = [&](double hw, double la, double lb, double& a, double& b) {
    const double m = fmin(fp.b2 * la, fp.b2 * lb), M = fmax(fp.b2 * la, fp.b2 * lb);
    const double lo = -hw - fp.b0 - M, hi = hw - fp.b0 - m;  // b1 k in [lo, hi]
    if (fabs(fp.b1) < 1e-12) {
      if (lo <= 0.0 && hi >= 0.0) {
        a = -1e300;
        b = 1e300;
      } else {
        a = 1e300;
        b = -1e300;
      }
    } else if (fp.b1 > 0.0) {
      a = lo / fp.b1;
      b = hi / fp.b1;
    } else {
      a = hi / fp.b1;
      b = lo / fp.b1;
    }
  };
  const int ra = ty * 8 > r0 ? ty * 8 : r0, rb = ty * 8 + 7 < r1 ? ty * 8 + 7 : r1;
  // l-range of the strip's samples
  const double la = p.compat ? ra - hh : hh - rb, lb = p.compat ? rb - hh : hh - ra + 0.5;
  double a = -1e300, b = 1e300;
  if (fp.tri_ok) {  // the projected T_D cut to the (widened) strip
    const double la2 = la - fp.dimg, lb2 = lb + fp.dimg;
    double ta = 1e300, tb = -1e300;
    for (int i = 0; i < 3; i++) {
      if (fp.l[i] >= la2 && fp.l[i] <= lb2) {
        ta = fmin(ta, fp.k[i]);
        tb = fmax(tb, fp.k[i]);
      }
      const int j = (i + 1) % 3;
      const double ys[2] = {la2, lb2};
      for (int s = 0; s < 2; s++) {
        const double y = ys[s];
        if ((fp.l[i] - y) * (fp.l[j] - y) < 0.0) {
          const double t = (y - fp.l[i]) / (fp.l[j] - fp.l[i]);
          const double x = fp.k[i] + t * (fp.k[j] - fp.k[i]);
          ta = fmin(ta, x);
          tb = fmax(tb, x);
        }
      }
    }
    a = ta - fp.dimg;
    b = tb + fp.dimg;
  }
  double ba, bb;
  band(fp.hw, la, lb, ba, bb);
  a = fmax(a, ba);
  b = fmin(b, bb);
  int c0 = 1, c1 = 0, d0 = 1, d1 = 0;
  if (a <= b) cols(fmax(a, p.kmin - 1.0), fmin(b, p.kmax + 1.0), c0, c1);
  if (fp.hw0 >= 0.0) {
    band(fp.hw0, la, lb, ba, bb);
    if (ba <= bb) cols(fmax(ba, p.kmin - 1.0), fmin(bb, p.kmax + 1.0), d0, d1);
  }
  a0 = c0 <= c1 ? c0 >> 3 : 1;
  a1 = c0 <= c1 ? c1 >> 3 : 0;
  b0 = d0 <= d1 ? d0 >> 3 : 1;
  b1 = d0 <= d1 ? d1 >> 3 : 0;
}

// The footprint's tiles of this rank in tile row ty, in column order.
template <class F>
__host__ __device__ void raster_row(const CandParams& p, const Footprint& fp, int ty, int r0, int r1,
                                    F emit) {
  int a0, a1, b0, b1;
  row_tiles(p, fp, ty, r0, r1, a0, a1, b0, b1);
  auto put = [&](int tx) {
    uint32_t rk;
    const uint32_t t = rt_tile_local(tx, ty, (uint32_t)p.nranks, (uint32_t)p.blocks_x, (uint32_t)p.tb, &rk);
    if ((int)rk == p.rank) emit(t);
  };
  for (int tx = a0; tx <= a1; tx++) put(tx);
  for (int tx = b0; tx <= b1; tx++)
    if (!(tx >= a0 && tx <= a1)) put(tx);
}

// Number of tiles raster_row emits for row ty, without visiting them.
__host__ __device__ inline uint32_t count_row(const CandParams& p, const Footprint& fp, int ty, int r0,
                                              int r1) {
  int a0, a1, b0, b1;
  row_tiles(p, fp, ty, r0, r1, a0, a1, b0, b1);
  auto cnt = [&](int x0, int x1) { return rank_tiles(p, ty, x0, x1); };
  uint32_t c = cnt(a0, a1) + cnt(b0, b1);
  if (a0 <= a1 && b0 <= b1) c -= cnt(a0 > b0 ? a0 : b0, a1 < b1 ? a1 : b1);  // overlap counted once
  return c;
}

// raster_row's tiles of row ty as three disjoint column intervals, in
// emission order: x[0..1] = [a0, a1], then the parts of [b0, b1] left and
// right of it (x[2..3], x[4..5]; empty: x0 > x1); c[i] = this rank's tiles in
// interval i, f[i] = its first block column (rt_rank_row_tiles).  c[0] + c[1]
// + c[2] == count_row (the rank's tiles of a column set add up over disjoint
// parts).
__host__ __device__ inline void row_ivs(const CandParams& p, const Footprint& fp, int ty, int r0, int r1,
                                        int* x, int* f, uint32_t* c) {
  int a0, a1, b0, b1;
  row_tiles(p, fp, ty, r0, r1, a0, a1, b0, b1);
  x[0] = a0;
  x[1] = a1;
  if (a0 > a1) {
    x[2] = b0;
    x[3] = b1;
    x[4] = 1;
    x[5] = 0;
  } else {
    x[2] = b0;
    x[3] = b1 < a0 - 1 ? b1 : a0 - 1;
    x[4] = b0 > a1 + 1 ? b0 : a1 + 1;
    x[5] = b1;
  }
  for (int i = 0; i < 3; i++) {
    f[i] = 0;
    c[i] = x[2 * i] > x[2 * i + 1]
               ? 0u
               : rt_rank_row_tiles(ty, x[2 * i], x[2 * i + 1], (uint32_t)p.nranks, (uint32_t)p.rank,
                                   (uint32_t)p.blocks_x, (uint32_t)p.tb, &f[i]);
  }
}

// Tiles of this rank whose camera samples can be candidates for the
// triangle.  Pixel (r, c) samples k in [W/2 - c, W/2 - c + 1/2], l in
// [H/2 - r, H/2 - r + 1/2] (cpu/raytracer.c:55-58 with i = W/2 - c, j = H/2 -
// r).
template <class F>
__host__ __device__ void raster(const CandParams& p, const Footprint& fp, F emit) {
  int r0, r1;
  if (!raster_rows(p, fp, r0, r1)) return;
  for (int ty = r0 >> 3; ty <= (r1 >> 3); ty++) raster_row(p, fp, ty, r0, r1, emit);
}

// The number of tiles raster() emits, one step per tile row.
__host__ __device__ inline uint32_t raster_count(const CandParams& p, const Footprint& fp) {
  int r0, r1;
  if (!raster_rows(p, fp, r0, r1)) return 0;
  uint32_t n = 0;
  for (int ty = r0 >> 3; ty <= (r1 >> 3); ty++) n += count_row(p, fp, ty, r0, r1);
  return n;
}

// Per-tile refinement of a listed (prim, tile) entry.  classify() bounds the
// error region T_D once per triangle, over every camera line that can reach
// it: the smallest grazing cosine of any such line and the widest cone of
// directions.  The rays of one 8x8 tile have nearly one direction, so the
// same bound (tools/mt_bound.py, componentwise) evaluated with that tile's
// own |d_i|, |o_i - v0_i| and |a| gives a T_D of the tile's rays alone;
// false when the tile's samples, projected through the eye and widened by
// the camera lines' float deviation (classify's dimg), provably miss it (or
// no ray of the tile reaches |a| >= 1e-7).  true whenever unsure.
// The triangle's part (once per footprint; the big emission keeps it in LDS).
// With Y = P - pos for a point P = v0 + cu e1 + cv e2 of the triangle's
// plane, the homogeneous image point of P (classify's projection through the
// eye, H = (k0 yn + plane (g0 yu + g1 yv), l0 yn + plane (g1 yu + g2 yv), yn),
// yn / yu / yv = Y . n / u / v) is linear in (cu, cv): H = B0 + cu B1 + cv B2.
struct TileTri {
  double pv0[3];           // pos - v0
  double ae1[3], ae2[3];   // |e1_i|, |e2_i|
  double nl;               // |e1 x e2|
  double bcp, bcx, bcy;    // grazing offset (pos - o) . nh at tile (tx, ty): bcp - tx bcx - ty bcy
  double bw;               // its spread over a tile's rectangle
  double B[3][3];          // H of v0 - pos, e1, e2 (as points / directions)
  double ym[3];            // L1 norms of v0 - pos, e1, e2 (bounds of |Y|)
};
// The frame's part (CandParams' tile_* constants and the bound's terms).
struct TileFrame {
  double k00, l00, dk, dl, hk, hl, hd;
  double p00[3], du[3], dv[3], w[3];
  double dorig, cw, ca, gscale, dline, lmax;
};
RTC_FN void tile_frame(const CandParams& p, TileFrame& f) {
  f.k00 = p.tile_k00;
  f.l00 = p.tile_l00;
  f.dk = p.tile_dk;
  f.dl = p.tile_dl;
  f.hk = p.tile_hk;
  f.hl = p.tile_hl;
  f.hd = p.tile_hd;
  for (int a = 0; a < 3; a++) {
    f.p00[a] = p.tile_p00[a];
    f.du[a] = p.tile_du[a];
    f.dv[a] = p.tile_dv[a];
    f.w[a] = p.tile_w[a];
  }
  f.dorig = p.dorig;
  f.cw = p.c_dot / 8.6 * 6.01 * kEps;
  f.ca = p.c_a / 7.2 * 5.01 * kEps;
  f.gscale = p.gscale;
  f.dline = p.dline;
  f.lmax = p.lmax;
}
RTC_FN bool tile_tri(const CandParams& p, const float* r, TileTri& t) {
  double v0[3], e1[3], e2[3];
  for (int a = 0; a < 3; a++) {
    v0[a] = r[a];
    e1[a] = r[3 + a];
    e2[a] = r[6 + a];
    t.pv0[a] = p.pos[a] - v0[a];
    t.ae1[a] = fabs(e1[a]);
    t.ae2[a] = fabs(e2[a]);
  }
  const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  t.nl = norm3(n);
  if (!(t.nl > 0.0)) return false;
  const double inl = 1.0 / t.nl;
  const double nh[3] = {n[0] * inl, n[1] * inl, n[2] * inl};
  t.bcp = dot3(p.tile_p00, nh);
  t.bcx = dot3(p.tile_du, nh);
  t.bcy = dot3(p.tile_dv, nh);
  t.bw = fabs(dot3(p.u, nh)) * p.tile_hk + fabs(dot3(p.v, nh)) * p.tile_hl;
  const double* V[3] = {t.pv0, e1, e2};
  for (int k = 0; k < 3; k++) {
    const double sgn = k == 0 ? -1.0 : 1.0;  // v0 - pos = -(pos - v0)
    const double yn = sgn * dot3(V[k], p.n), yu = sgn * dot3(V[k], p.u), yv = sgn * dot3(V[k], p.v);
    t.B[k][0] = p.k0 * yn + p.plane * (p.ginv[0] * yu + p.ginv[1] * yv);
    t.B[k][1] = p.l0 * yn + p.plane * (p.ginv[1] * yu + p.ginv[2] * yv);
    t.B[k][2] = yn;
    t.ym[k] = fabs(V[k][0]) + fabs(V[k][1]) + fabs(V[k][2]);
  }
  return true;
}

// The tile's part.  Division-light (the big emission runs it per entry, in
// f64): the affine quantities' extremes over the tile's sample rectangle in
// closed form (|f_c| + |f_k| hk + |f_l| hl), and T_D's projection tested in
// homogeneous image coordinates (no per-corner division).
RTC_FN bool tile_keep(const TileFrame& p, const TileTri& t, int tx, int ty) {
  // the tile's sample rectangle [kc -+ hk] x [lc -+ hl] (pixel_range's
  // inverse, CandParams::tile_*), its centre o_c = C + kc u + lc v, and per
  // axis max |pos_i - o_i| and max |o_i - v0_i| over it
  // (fused multiply-adds throughout: these are bounds of our own, each
  // rounding far inside their margins, and fma is exact IEEE on host and device)
  const double dtx = (double)tx, dty = (double)ty;
  const double kc = fma(dtx, p.dk, p.k00), lc = fma(dty, p.dl, p.l00);
  double pm[3], sm[3], po[3];
  for (int a = 0; a < 3; a++) {
    po[a] = fma(-dtx, p.du[a], fma(-dty, p.dv[a], p.p00[a]));  // pos - o_c
    pm[a] = fabs(po[a]) + p.w[a];
    sm[a] = (fabs(t.pv0[a] - po[a]) + p.w[a] + p.dorig) * (1.0 + 1e-9);
  }
  // |pos - o| within the centre's +- the tile's half diagonal (hk |u| + hl |v|)
  const double rc = sqrt(fma(po[0], po[0], fma(po[1], po[1], po[2] * po[2])));
  const double rmn = rc - p.hd - p.dorig, rmx = (rc + p.hd + p.dorig) * (1.0 + 1e-9);
  if (!(rmn > 1e-6)) return true;
  const double irn = 1.0 / rmn;
  // float origins within dorig, float directions within a few eps of pos - o
  double dm[3];
  for (int a = 0; a < 3; a++) dm[a] = fmin(1.0, fma(pm[a] + p.dorig, irn, 8.0 * kEps)) * kDMax;
  double M[3], N[3];
  for (int i = 0; i < 3; i++) {
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    M[i] = fma(dm[j], t.ae2[k], dm[k] * t.ae2[j]);
    N[i] = fma(sm[j], t.ae1[k], sm[k] * t.ae1[j]);
  }
  // the componentwise bounds alone (each of them and classify's Cauchy-Schwarz
  // ones is a bound on its own; for a tile's narrow cone these are the
  // smaller)
  const double cw = p.cw, ca = p.ca;
  auto dotf = [](const double* a, const double* b) { return fma(a[0], b[0], fma(a[1], b[1], a[2] * b[2])); };
  const double e_sh = cw * dotf(sm, M);
  const double e_dq = cw * dotf(dm, N);
  const double e_a = ca * dotf(t.ae1, M);
  // grazing cosine of the tile's rays: |b| over the rectangle is in [bl, bh]
  const double bc = fma(-dtx, t.bcx, fma(-dty, t.bcy, t.bcp));
  const double bl = fmax(0.0, fabs(bc) - t.bw), bh = fabs(bc) + t.bw;
  const double cmax = fmin(1.0, fma(bh + p.dorig, irn, 8.0 * kEps));
  if (kDMax * t.nl * cmax + e_a < kAMin) return false;  // |a| < 1e-7 for every ray of the tile
  // a_lb = max(kAMin, dmin nl cmin - e_a), cmin = (bl - dorig) / rmx - 8 eps,
  // kept as the fraction num / rmx; rho = e_a / a_lb < 1/2 <=> 2 e_a < a_lb
  const double num = fma(kDMin * t.nl, bl - p.dorig - 8.0 * kEps * rmx, -e_a * rmx);
  const bool clamp = !(num > kAMin * rmx);
  if (clamp ? !(2.0 * e_a < kAMin) : !(2.0 * e_a * rmx < num)) return true;
  // 1 / (a_lb (1 - rho)) = 1 / (a_lb - e_a): du = e_sh / (a_lb - e_a), and
  // dw = (4 eps + (e_sh + e_dq) / a_lb + rho) / (1 - rho)
  //    = 4 eps / (1 - rho) + (e_sh + e_dq + e_a) / (a_lb - e_a)
  //   <= 8 eps + (e_sh + e_dq + e_a) / (a_lb - e_a)
  const double iq = clamp ? 1.0 / (kAMin - e_a) : rmx / fma(-e_a, rmx, num);
  const double du = e_sh * iq, dv = e_dq * iq;
  const double dw = fma(e_sh + e_dq + e_a, iq, 8.0 * kEps);
  // T_D's corners (cu, cv) and their homogeneous image points H_k = B0 + cu
  // B1 + cv B2 ~ (K_k, L_k, 1): classify's lam = plane / yn, without dividing
  const double cu[3] = {-du, 1.0 + dw + dv, -du}, cv[3] = {-dv, -dv, 1.0 + dw + du};
  double H[3][3], ymag = 1.0, ylo = 1e300, yhi = -1e300;
  for (int k = 0; k < 3; k++) {
    for (int c = 0; c < 3; c++) H[k][c] = fma(cu[k], t.B[1][c], fma(cv[k], t.B[2][c], t.B[0][c]));
    ymag = fmax(ymag, fma(fabs(cu[k]), t.ym[1], fma(fabs(cv[k]), t.ym[2], t.ym[0])));
    ylo = fmin(ylo, H[k][2]);
    yhi = fmax(yhi, H[k][2]);
  }
  // every corner strictly on one side of the eye plane; the nearest point of
  // T_D is then at least min |yn| from the eye
  if (!(ylo > 1e-6 * ymag || yhi < -1e-6 * ymag)) return true;
  const double sg = ylo > 0.0 ? 1.0 : -1.0, rlo = fmin(fabs(ylo), fabs(yhi));
  const double dimg = 1.5 * p.gscale * (p.dline * (1.0 + p.lmax / rlo) + p.dorig) + 1e-3;
  const double x0 = kc - p.hk - dimg, x1 = kc + p.hk + dimg;
  const double y0 = lc - p.hl - dimg, y1 = lc + p.hl + dimg;
  // separating axes: the rectangle's (K_k < x0 <=> sg H_k0 < sg x0 yn_k, ...)
  {
    bool lx = true, gx = true, ly = true, gy = true;
    for (int k = 0; k < 3; k++) {
      const double hx = sg * H[k][0], hy = sg * H[k][1], w = sg * H[k][2];  // w > 0
      const double tx0 = 1e-9 * (fabs(hx) + fabs(x0) * w), tx1 = 1e-9 * (fabs(hx) + fabs(x1) * w);
      const double ty0 = 1e-9 * (fabs(hy) + fabs(y0) * w), ty1 = 1e-9 * (fabs(hy) + fabs(y1) * w);
      lx = lx && hx < x0 * w - tx0;
      gx = gx && hx > x1 * w + tx1;
      ly = ly && hy < y0 * w - ty0;
      gy = gy && hy > y1 * w + ty1;
    }
    if (lx || gx || ly || gy) return false;
  }
  // and the triangle's edges: q = (x, y, 1) lies outside edge e -> f when
  // det[H_e; H_f; q] has the sign opposite to det[H_0; H_1; H_2] sg
  double c01[3], c12[3], c20[3];
  auto cross3 = [](const double* a, const double* b, double* c) {
    c[0] = fma(a[1], b[2], -a[2] * b[1]);
    c[1] = fma(a[2], b[0], -a[0] * b[2]);
    c[2] = fma(a[0], b[1], -a[1] * b[0]);
  };
  cross3(H[0], H[1], c01);
  cross3(H[1], H[2], c12);
  cross3(H[2], H[0], c20);
  const double orient = dotf(H[2], c01) * sg;
  if (orient == 0.0) return true;
  const double so = orient > 0.0 ? 1.0 : -1.0;
  const double* C3[3] = {c01, c12, c20};
  for (int e = 0; e < 3; e++) {
    const double cx = so * C3[e][0], cy = so * C3[e][1], cz = so * C3[e][2];
    const double mx = fmax(cx * x0, cx * x1) + fmax(cy * y0, cy * y1) + cz;  // largest over the rectangle
    const double tol = 1e-9 * (fabs(cx) * fmax(fabs(x0), fabs(x1)) + fabs(cy) * fmax(fabs(y0), fabs(y1)) + fabs(cz));
    if (mx < -tol) return false;
  }
  return true;
}

RTC_FN bool tile_keep(const CandParams& p, const float* r, int tx, int ty) {
  TileTri t;
  TileFrame f;
  tile_frame(p, f);
  return !tile_tri(p, r, t) || tile_keep(f, t, tx, ty);
}

// A footprint is "big" -- counted and emitted by one wave, its tile rows
// spread over the lanes -- when it spans more than kSmallRows tile rows or
// has more than kSmallEntries entries; the others are counted and emitted by
// one thread each.  (A thread per footprint of hundreds of entries stalled
// its whole wave: count 2.6 ms, emit 1.4 ms on C5 before the split.)
constexpr int kSmallRows = 2;
constexpr uint32_t kSmallEntries = 32;
// persistent waves of the big-footprint passes (they loop over the big list,
// whose length only the device knows before the scan)
constexpr int kBigWaves = 4096;
// Entries per big_item_kernel / refine_kernel wave: 1 << CandParams::
// chunk_shift.  One wave per footprint (big_kernel) left the chip idle behind
// a few long ones: C5's largest footprint has 53,789 entries in rows of ~200
// tiles, each lane writing its row alone, and the kernel ran at 0.42 resident
// waves per SIMD (profiles/r03w_c5/pmc_sq.json).  1024 for a whole frame; a
// build of 1/N of the work (a rank's share, a producer's slice) has 1/N of
// the items, too few to cover the latency of one, and takes smaller chunks
// (rt_hip.cpp cand_chunk_shift).
// threads per workgroup of the per-prim list passes (fast path,
// classification, small emission)
#ifndef RT_LIST_BLOCK
#define RT_LIST_BLOCK 256
#endif
// bits per radix place of the lists' sort (0: rocPRIM's tuned default, 8):
// 9 sorts C5's 17-bit tile keys in two places instead of three (lists 2.13
// -> 1.98 ms; 6 bits: 2.20; profiles/r04o_sort_bits/)
#ifndef RT_SORT_BITS
#define RT_SORT_BITS 9
#endif
#ifndef RT_SORT_MERGE_LIMIT
#define RT_SORT_MERGE_LIMIT (1u << 16)
#endif

// Pass 0: the float fast path over every prim; flags the prims it cannot
// prove safe (visits[prim] = 1), which an exclusive scan and scatter_kernel
// turn into a compact list, so the f64 classification of pass 1 runs on full
// waves instead of on the scattered third of the lanes of every wave.
// the i-th prim of the build's slice (CandParams::prim0, sl_stride)
__device__ __forceinline__ uint32_t slice_prim(const CandParams& p, uint32_t i) {
  if (p.sl_stride <= 1u) return p.prim0 + i;
  const uint32_t b = i / RT_SLICE_BLOCK;
  return (b * p.sl_stride + p.sl_rank) * RT_SLICE_BLOCK + i % RT_SLICE_BLOCK;
}

// waves per SIMD the fast path is compiled for (VGPR budget; A/B knob)
#ifndef RT_QUICK_WAVES
#define RT_QUICK_WAVES 1
#endif
__global__ __launch_bounds__(RT_LIST_BLOCK, RT_QUICK_WAVES) void quick_kernel(CandParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // index in the slice
  const uint32_t len = p.prim1 - p.prim0;
  if (i < 8u) p.ctr[i] = 0u;          // the frame's counters (count / big passes, later launches)
  if (i == 0u) p.visits[len] = 0u;    // the scan's last input
  if (i >= len) return;
  p.visits[i] = quick_class(p, (const float*)(p.tri + 3 * (size_t)slice_prim(p, i))) == Q_LIST ? 1u : 0u;
}

__global__ __launch_bounds__(256) void scatter_kernel(CandParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t len = p.prim1 - p.prim0;
  if (i > len) return;
  if (i == len) {
    p.ctr[3] = p.off[len];  // list length
    return;
  }
  if (p.visits[i]) p.list[p.off[i]] = slice_prim(p, i);
}

// The footprints whose entries are refined per tile (CandParams::refine):
// those spanning more than kSmallRows tile rows of the frame.  A property of
// the footprint alone, not of a rank's share of its tiles, so a rank's own
// lists and the triangle-parallel build (one whole-frame rank) refine the same
// entries; all of them are big footprints (the big passes emit them).
__host__ __device__ inline bool refined_rows(int r0, int r1) { return (r1 >> 3) - (r0 >> 3) + 1 > kSmallRows; }
__host__ __device__ inline bool refined_footprint(const CandParams& p, const Footprint& fp) {
  int r0, r1;
  return raster_rows(p, fp, r0, r1) && refined_rows(r0, r1);
}

// small footprint: few tile rows, counted here row by row; false: big
__host__ __device__ inline bool small_count(const CandParams& p, const Footprint& fp, uint32_t& n) {
  int r0, r1;
  n = 0;
  if (!raster_rows(p, fp, r0, r1)) return true;
  if ((r1 >> 3) - (r0 >> 3) + 1 > kSmallRows) return false;
  for (int ty = r0 >> 3; ty <= (r1 >> 3); ty++) n += count_row(p, fp, ty, r0, r1);
  return n <= kSmallEntries;
}

// A small footprint as emit_kernel needs it: its first tile row and row
// count, and per row (at most kSmallRows) row_ivs's three column intervals as
// 16-bit values -- 32 B instead of the 120 B footprint, and no f64 row
// geometry in the emission.  small_count and this form in one pass (row_ivs's
// counts add up to count_row's).  (cand_prepare keeps the footprint path for
// frames of 32,767 tile columns or more.)
__device__ __forceinline__ bool small_pack(const CandParams& p, const Footprint& fp, uint32_t& n, uint32_t* w) {
  int r0, r1;
  n = 0;
  if (!raster_rows(p, fp, r0, r1)) return true;
  const int ty0 = r0 >> 3, nr = (r1 >> 3) - ty0 + 1;
  if (nr > kSmallRows) return false;
  w[0] = (uint32_t)ty0 | ((uint32_t)nr << 16);
  for (int h = 1; h < 8; h++) w[h] = 0u;
  for (int r = 0; r < nr; r++) {
    int x[6], f[3];
    uint32_t c[3];
    row_ivs(p, fp, ty0 + r, r0, r1, x, f, c);
    n += c[0] + c[1] + c[2];
    for (int i = 0; i < 6; i++) {
      const int h = 1 + r * 3 + i / 2;  // words 1..3 row 0, 4..6 row 1
      w[h] |= ((uint32_t)x[i] & 0xffffu) << (16 * (i & 1));
    }
  }
  return n <= kSmallEntries;
}

// the classification's leaf box loaded at its start instead of at its use
// (A/B knob: lists 1.803 -> 1.816 ms at 128 VGPRs, profiles/r08_list_occupancy/)
#ifndef RT_COUNT_LEAF_AHEAD
#define RT_COUNT_LEAF_AHEAD 0
#endif
// Pass 1: classify the listed prims, keep each one's footprint and count the
// tiles of the small ones (visits[j] for list entry j; visits is zero beyond
// the list); big ones are queued for big_count_kernel.
__device__ __forceinline__ void count_one(const CandParams& p, uint32_t j) {
  const uint32_t prim = p.list[j];
  const float* rec = (const float*)(p.tri + 3 * (size_t)prim);
  uint32_t visits = 0;
  Footprint fp;
#if RT_COUNT_LEAF_AHEAD
  // the leaf box in registers from the start: its loads (prim -> leaf ->
  // box, a dependent pair) overlap the f64 bound instead of waiting at its end
  // (no leaf map: an empty box, which no corner lies in -- the same verdicts
  // as no box; one array either way keeps it in registers)
  float4 b0 = make_float4(__builtin_inff(), __builtin_inff(), __builtin_inff(), 0.0f);
  float4 b1 = make_float4(-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), 0.0f);
  if (p.prim_leaf) {
    const float4* nb = p.node + 2 * (size_t)p.prim_leaf[prim];
    b0 = nb[0];
    b1 = nb[1];
  }
  const float lbox[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const float* lb = lbox;
#else
  const float* lb = p.prim_leaf ? (const float*)(p.node + 2 * (size_t)p.prim_leaf[prim]) : nullptr;
#endif
  const int c = classify(p, rec, lb, fp);
  if (c == GLOBAL) {
    p.global[atomicAdd(p.ctr + 1, 1u)] = prim;
    p.skip[prim] = -1e30f;
  } else if (c == FOOTPRINT) {
    p.skip[prim] = fp.skip;
    uint32_t w[8];
    if (p.sfp ? small_pack(p, fp, visits, w) : small_count(p, fp, visits)) {
      if (visits) {
        if (p.store_fp) p.fp[j] = fp;
        if (p.sfp) {
          p.sfp[2 * (size_t)j] = make_uint4(w[0], w[1], w[2], w[3]);
          p.sfp[2 * (size_t)j + 1] = make_uint4(w[4], w[5], w[6], w[7]);
        }
      }
    } else {
      p.fp[j] = fp;
      if (p.sfp) p.sfp[2 * (size_t)j] = make_uint4(0xffffffffu, 0u, 0u, 0u);  // big: not emit_kernel's
      p.big[atomicAdd(p.ctr + 2, 1u)] = j;
      visits = 0;  // big_count_kernel
    }
  }
  p.visits[j] = visits;
}

#ifndef RT_COUNT_WAVES
#define RT_COUNT_WAVES 1
#endif
__global__ __launch_bounds__(RT_LIST_BLOCK, RT_COUNT_WAVES) void count_kernel(CandParams p) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < p.ctr[3]) count_one(p, j);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// exclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, int lane) {
  uint32_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  return inc - x;
}

// Pass 1b: one wave per big footprint, its tile rows over the lanes.
__global__ __launch_bounds__(64) void big_count_kernel(CandParams p) {
  const int lane = threadIdx.x;
  const uint32_t nbig = p.ctr[2];
  uint32_t witems = 0;
  for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const uint32_t j = p.big[b];
    const Footprint fp = p.fp[j];
    int r0, r1;
    uint32_t cnt = 0;
    if (raster_rows(p, fp, r0, r1))
      for (int ty = (r0 >> 3) + lane; ty <= (r1 >> 3); ty += 64) cnt += count_row(p, fp, ty, r0, r1);
    if (b < p.big_cap) p.big_lane[(size_t)b * 64 + lane] = cnt;  // big_kernel's offsets
    cnt = wave_sum(cnt);
    if (lane == 0) p.visits[j] = cnt;
    witems += (cnt + (1u << p.chunk_shift) - 1) >> p.chunk_shift;
  }
  // this wave's big_item_kernel items (one per chunk of entries of each of its
  // footprints), placed by a scan over the waves: one atomic per footprint
  // on a shared counter serialised at L2 (big_count 0.16 -> 1.5 ms on C5)
  if (lane == 0) p.wave_items[blockIdx.x] = witems;
}

// After the scan of wave_items: each big_count wave's footprints, in the same
// order, write their items from the wave's offset; past item_cap, ctr[5] = 1
// and the host emits with big_kernel instead.
__global__ __launch_bounds__(64) void item_kernel(CandParams p) {
  const int lane = threadIdx.x;
  const uint32_t nbig = p.ctr[2];
  uint32_t at = p.wave_base[blockIdx.x];
  if (blockIdx.x == 0 && lane == 0) p.ctr[4] = p.wave_base[kBigWaves];  // all items (read back with ctr[])
  for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const uint32_t ni = (p.visits[p.big[b]] + (1u << p.chunk_shift) - 1) >> p.chunk_shift;
    if (at + ni <= p.item_cap) {
      for (uint32_t c = (uint32_t)lane; c < ni; c += 64) p.items[at + c] = make_uint2(b, c);
    } else if (lane == 0) {
      p.ctr[5] = 1u;
    }
    at += ni;
  }
}

// The rank's tiles of one tile-row column interval [x0, x1] of tile row ty:
// the rank's blocks bx = f, f + n, ... of the row (csrc/rt_tiles.h), each
// contributing its columns inside the interval at consecutive local indices
// (the rank's blocks of a row are consecutive in its buffer) -- one prefix
// count per interval, no division per tile.  Returns the count written at
// keys/vals[o ..].
__device__ __forceinline__ uint32_t emit_interval(const CandParams& p, int ty, int x0, int x1,
                                                  uint32_t o, uint32_t prim, bool refine = false) {
  if (x0 > x1) return 0;
  const uint32_t n = (uint32_t)p.nranks, r = (uint32_t)p.rank;
  int f;
  const int tb = p.tb;
  const uint32_t cnt = rt_rank_row_tiles(ty, x0, x1, n, r, (uint32_t)p.blocks_x, (uint32_t)tb, &f);
  if (cnt == 0) return 0;
  const uint32_t row = (uint32_t)(ty % tb) * (uint32_t)tb;
  uint32_t blk = rt_block_local((uint32_t)f, (uint32_t)(ty / tb), n, (uint32_t)p.blocks_x, r);
  uint32_t k = 0;
  for (int bx = f; k < cnt; bx += (int)n, blk++) {
    const int a = x0 > bx * tb ? x0 : bx * tb, b = x1 < bx * tb + tb - 1 ? x1 : bx * tb + tb - 1;
    const uint32_t base = blk * (uint32_t)(tb * tb) + row;
    for (int tx = a; tx <= b; tx++, k++) {
      if (p.key_cap && o + k >= p.key_cap) {  // the buffers hold the previous frame's total
        p.ctr[7] = 1u;
        continue;
      }
      const bool keep = !refine || tile_keep(p, (const float*)(p.tri + 3 * (size_t)prim), tx, ty);
      p.keys[o + k] = keep ? base + (uint32_t)(tx - bx * tb) : p.drop_key;
      p.vals[o + k] = prim;
    }
  }
  return cnt;
}

// One tile row of a footprint (raster_row's tiles: [a0, a1] and the parts
// of [b0, b1] outside it); returns the entries written.
__device__ __forceinline__ uint32_t emit_row(const CandParams& p, const Footprint& fp, int ty, int r0,
                                             int r1, uint32_t o, uint32_t prim, bool refine = false) {
  int a0, a1, b0, b1;
  row_tiles(p, fp, ty, r0, r1, a0, a1, b0, b1);
  uint32_t k = emit_interval(p, ty, a0, a1, o, prim, refine);
  if (a0 > a1) {
    k += emit_interval(p, ty, b0, b1, o + k, prim, refine);
  } else {
    k += emit_interval(p, ty, b0, b1 < a0 - 1 ? b1 : a0 - 1, o + k, prim, refine);
    k += emit_interval(p, ty, b0 > a1 + 1 ? b0 : a1 + 1, b1, o + k, prim, refine);
  }
  return k;
}

// Pass 2 (after the scan of visits): the small footprints write their
// (tile, prim) pairs at their offsets.
__global__ __launch_bounds__(RT_LIST_BLOCK) void emit_kernel(CandParams p) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p.ctr[3]) return;
  uint32_t o = p.off[j];
  const uint32_t n = p.off[j + 1] - o;
  if (n == 0 || n > kSmallEntries) return;  // big footprints: big_kernel
  const uint32_t prim = p.list[j];
  if (p.sfp) {
    const uint4 a = p.sfp[2 * (size_t)j];
    if (a.x == 0xffffffffu) return;  // a big footprint of few entries
    const uint4 b = p.sfp[2 * (size_t)j + 1];
    const uint32_t w[7] = {a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int ty0 = (int)(a.x & 0xffffu), nr = (int)(a.x >> 16);
    for (int r = 0; r < nr; r++)
      for (int i = 0; i < 3; i++) {
        const uint32_t v = w[r * 3 + i];
        const int x0 = (int)(int16_t)(v & 0xffffu), x1 = (int)(int16_t)(v >> 16);
        o += emit_interval(p, ty0 + r, x0, x1, o, prim);
      }
    return;
  }
  const Footprint fp = p.fp[j];
  int r0, r1;
  if (!raster_rows(p, fp, r0, r1) || (r1 >> 3) - (r0 >> 3) + 1 > kSmallRows) return;
  for (int ty = r0 >> 3; ty <= (r1 >> 3); ty++) o += emit_row(p, fp, ty, r0, r1, o, prim);
}

// Pass 2b: one wave per big footprint, its tile rows over the lanes; a wave
// prefix sum of the lanes' row counts places each lane's entries.
__global__ __launch_bounds__(64) void big_kernel(CandParams p) {
  // launched only when the build expects more than item_cap items (ctr[5]):
  // read back, or -- an asynchronous build -- the same frame's earlier
  // read-back build's shape.  A shape that differs on the device (never
  // expected) means big_item_kernel was not launched: the frame is reported
  // (ctr[7] -> RT_EHITBUF, built again with a read-back), never incomplete.
  if (!p.ctr[5]) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p.ctr[7] = 1u;
    return;
  }
  const int lane = threadIdx.x;
  const uint32_t nbig = p.ctr[2];
  for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const uint32_t j = p.big[b], prim = p.list[j];
    const Footprint fp = p.fp[j];
    int r0 = 0, r1 = -1;
    const bool rows = raster_rows(p, fp, r0, r1);
    const int ty0 = r0 >> 3, ty1 = r1 >> 3;
    uint32_t cnt = 0;
    if (b < p.big_cap)
      cnt = p.big_lane[(size_t)b * 64 + lane];  // big_count_kernel's row subtotals
    else if (rows)
      for (int ty = ty0 + lane; ty <= ty1; ty += 64) cnt += count_row(p, fp, ty, r0, r1);
    uint32_t o = p.off[j] + wave_excl_scan(cnt, lane);
    const bool refine = p.refine != 0u && rows && refined_rows(r0, r1);
    if (rows)
      for (int ty = ty0 + lane; ty <= ty1; ty += 64) o += emit_row(p, fp, ty, r0, r1, o, prim, refine);
  }
}

// Column of the k-th of this rank's tiles in [x0, x1] of tile row ty (f =
// the first of the rank's block columns there, rt_rank_row_tiles): the first
// block may be cut on the left, the ones after it hold tb tiles each, n
// blocks apart.  tb is 1 or RT_TB (a power of two).
__device__ __forceinline__ int kth_rank_col(const CandParams& p, int x0, int x1, int f, uint32_t k) {
  const int tb = p.tb;
  const int s0 = x0 > f * tb ? x0 : f * tb;
  const int e0 = x1 < f * tb + tb - 1 ? x1 : f * tb + tb - 1;
  const uint32_t c0 = (uint32_t)(e0 - s0 + 1);
  if (k < c0) return s0 + (int)k;
  const uint32_t kk = k - c0, sh = (uint32_t)(__ffs(tb) - 1);
  const int m = 1 + (int)(kk >> sh);
  return (f + m * p.nranks) * tb + (int)(kk & (uint32_t)(tb - 1));
}

// Pass 2b, entry-parallel (big_count_kernel's items): the wave writes entries
// [c chunk, (c + 1) chunk) of big footprint b, lane-consecutive (coalesced
// stores).  Row by row in row-major order, each row's intervals in
// raster_row's order; the rows are taken 64 at a time -- the lanes compute
// their intervals and counts (row_ivs), a wave scan places them, and each
// entry of the chunk finds its row by binary search over the 64 prefixes in
// LDS.  Same (tile, prim) set as big_kernel; the sort orders it.
// One workgroup per item.  CHECK (an asynchronous build: its grid is the
// same frame's read-back build's) reads the item count and the over-cap flag
// on the device: an over-cap flag (ctr[5]) the launch did not expect, or a
// count the grid does not cover -- never expected -- sets ctr[7], so the
// frame is reported rather than incomplete.  (The checks cost 16-18 VGPRs -- 4 waves
// per SIMD instead of 5 -- so the read-back build's launch, whose grid is
// the exact count, goes without them; a grid-stride loop over the items held
// 118 VGPRs.)
template <bool CHECK>
__global__ __launch_bounds__(64) void big_item_kernel(CandParams p) {
  __shared__ uint32_t pre[65];
  __shared__ int rx[64][6], rf[64][3];
  __shared__ uint32_t rc[64][2];
  __shared__ int rty[64];
  const int lane = threadIdx.x;
  if (CHECK) {
    if (p.ctr[5]) {  // more items than item_cap after all: big_kernel was not launched (as big_kernel)
      if (blockIdx.x == 0 && lane == 0) p.ctr[7] = 1u;
      return;
    }
    const uint32_t n_items = p.wave_base[kBigWaves];
    if (blockIdx.x == 0 && lane == 0 && n_items > gridDim.x) p.ctr[7] = 1u;
    if (blockIdx.x >= n_items) return;
  }
  const uint2 it = p.items[blockIdx.x];
  const uint32_t j = p.big[it.x], prim = p.list[j];
  const uint32_t base = p.off[j], total = p.off[j + 1] - base;
  const uint32_t c0 = it.y << p.chunk_shift;
  uint32_t c1 = c0 + (1u << p.chunk_shift) < total ? c0 + (1u << p.chunk_shift) : total;
  if (CHECK && base + c1 > p.key_cap) {  // entries past the buffers: not written, the frame reported
    if (lane == 0) p.ctr[7] = 1u;
    c1 = p.key_cap > base ? p.key_cap - base : 0u;
  }
  const Footprint fp = p.fp[j];
  int r0, r1;
  if (!raster_rows(p, fp, r0, r1)) return;  // no entries, no items
  uint32_t g0 = 0;  // entries of the footprint before this group of rows
  for (int gy = r0 >> 3; gy <= (r1 >> 3) && g0 < c1; gy += 64) {
    const int ty = gy + lane;
    int x[6] = {1, 0, 1, 0, 1, 0}, f[3] = {0, 0, 0};
    uint32_t c[3] = {0u, 0u, 0u};
    if (ty <= (r1 >> 3)) row_ivs(p, fp, ty, r0, r1, x, f, c);
    const uint32_t n = c[0] + c[1] + c[2];
    const uint32_t ex = wave_excl_scan(n, lane);
    const uint32_t gt = __shfl(ex + n, 63, 64);
    if (g0 + gt > c0) {
      __syncthreads();  // after the previous group's readers
      pre[lane] = g0 + ex;
      if (lane == 63) pre[64] = g0 + gt;
#pragma unroll
      for (int i = 0; i < 6; i++) rx[lane][i] = x[i];
#pragma unroll
      for (int i = 0; i < 3; i++) rf[lane][i] = f[i];
      rc[lane][0] = c[0];
      rc[lane][1] = c[1];
      rty[lane] = ty;
      __syncthreads();
      const uint32_t e0 = c0 > g0 ? c0 : g0, e1 = c1 < g0 + gt ? c1 : g0 + gt;
      for (uint32_t e = e0 + (uint32_t)lane; e < e1; e += 64) {
        // the last row whose prefix is <= e (it holds e: e < pre[64], and a
        // row without entries shares its prefix with the next one)
        int r = 0;
#pragma unroll
        for (int s = 32; s > 0; s >>= 1)
          if (pre[r + s] <= e) r += s;
        uint32_t k = e - pre[r];
        int iv = 0;
        if (k >= rc[r][0]) {
          k -= rc[r][0];
          iv = 1;
          if (k >= rc[r][1]) {
            k -= rc[r][1];
            iv = 2;
          }
        }
        const int tx = kth_rank_col(p, rx[r][2 * iv], rx[r][2 * iv + 1], rf[r][iv], k);
        uint32_t rk;
        p.keys[base + e] = rt_tile_local(tx, rty[r], (uint32_t)p.nranks, (uint32_t)p.blocks_x,
                                         (uint32_t)p.tb, &rk);
        p.vals[base + e] = prim;
      }
    }
    g0 += gt;
  }
}

// The per-tile refinement (CandParams::refine) as its own pass over
// big_item_kernel's items: each wave re-reads its chunk's keys and rewrites
// the dropped ones with drop_key.  A pass of its own, with the triangle's and
// the frame's parts in LDS and re-read per entry, runs at 80 VGPRs and 6
// waves per SIMD; inside big_item_kernel the same test held 137-175 VGPRs (2-3
// waves) and the frame took 0.1 ms longer on C5 (profiles/r06e/ab.log).
__device__ __forceinline__ void refine_item(const CandParams& p, uint32_t item);

#ifndef RT_REFINE_WAVES
#define RT_REFINE_WAVES 1
#endif
template <bool CHECK>
__global__ __launch_bounds__(64, RT_REFINE_WAVES) void refine_kernel(CandParams p) {
  if (CHECK && (p.ctr[5] || blockIdx.x >= p.wave_base[kBigWaves])) return;
  refine_item(p, blockIdx.x);
}

__device__ __forceinline__ void refine_item(const CandParams& p, uint32_t item) {
  const int lane = threadIdx.x;
  const uint2 it = p.items[item];
  const uint32_t j = p.big[it.x], prim = p.list[j];
  const Footprint fp = p.fp[j];
  int r0, r1;
  if (!raster_rows(p, fp, r0, r1) || !refined_rows(r0, r1)) return;
  const uint32_t base = p.off[j], total = p.off[j + 1] - base;
  const uint32_t c0 = it.y << p.chunk_shift;
  const uint32_t c1 = c0 + (1u << p.chunk_shift) < total ? c0 + (1u << p.chunk_shift) : total;
  __shared__ TileTri tt;
  __shared__ TileFrame tf;
  __shared__ int tt_ok;
  if (lane == 0) {
    tt_ok = tile_tri(p, (const float*)(p.tri + 3 * (size_t)prim), tt) ? 1 : 0;
    tile_frame(p, tf);
  }
  __syncthreads();
  if (!tt_ok) return;
  for (uint32_t e = c0 + (uint32_t)lane; e < c1; e += 64) {
    // re-read the LDS inputs per entry instead of holding them live across
    // the loop (a compiler memory barrier; 161 -> 80 VGPRs)
    __asm__ volatile("" ::: "memory");
    if (p.key_cap && base + e >= p.key_cap) break;  // not written (ctr[7] is set)
    int tx, ty;
    rt_tile_xy(p.keys[base + e], (uint32_t)p.rank, (uint32_t)p.nranks, (uint32_t)p.blocks_x, (uint32_t)p.tb, &tx, &ty);
    if (!tile_keep(tf, tt, tx, ty)) p.keys[base + e] = p.drop_key;
  }
}

__global__ __launch_bounds__(256) void prim_leaf_kernel(const float4* node, uint32_t nnode,
                                                        const float4* tri, uint32_t* prim_leaf) {
  const uint32_t ni = blockIdx.x * blockDim.x + threadIdx.x;
  if (ni >= nnode) return;
  const uint32_t first = __float_as_uint(node[2 * ni].w), info = __float_as_uint(node[2 * ni + 1].w);
  if (!(info & 0x80000000u)) return;  // RT_NODE_LEAF
  const uint32_t cnt = info & 0x7fffffffu;
  // the smallest leaf index holding the prim (a prim referenced by several
  // leaves -- the host SAH tree duplicates -- gets the same leaf on every
  // build, so the lists do not depend on the order of these writes)
  for (uint32_t k = 0; k < cnt; k++) atomicMin(prim_leaf + __float_as_uint(tri[3 * (size_t)(first + k) + 2].y), ni);
}

// start[t] = first entry of tile t in the tile-sorted keys; start[ntiles] =
// the entries with a tile (the refinement's dropped entries, key ntiles, sort
// after them)
__global__ __launch_bounds__(256) void bounds_kernel(const uint32_t* keys, uint32_t n, uint32_t* start,
                                                     uint32_t ntiles, uint32_t* snap) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // an asynchronous build's counters ctr[0 .. 7] -> ctr[16 .. 23] for
  // rt_hip_stats, after every pass that may set its overflow flag
  if (snap && t < 8u) snap[16 + t] = snap[t];
  if (t > ntiles) return;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (keys[mid] < t)
      lo = mid + 1;
    else
      hi = mid;
  }
  start[t] = lo;
}

// per list entry: the depth-skip bound of its prim (coalesced for the render
// kernel, which would otherwise gather it right after loading the entry)
// n_dev (optional): the entries with a tile, start[ntiles] -- the ones the
// refinement dropped sort after them and are never read
__global__ __launch_bounds__(256) void entry_skip_kernel(const uint32_t* cand, const float* skip,
                                                         float* out, uint32_t n, const uint32_t* n_dev) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (!n_dev || i < *n_dev)) out[i] = skip[cand[i]];
}

// --- triangle-parallel multi-GPU lists (rt_cand.h "route") ---------------
// A whole-frame entry (scanline tile of the one-rank map) -> its rank d and
// rank-local tile l under the N-rank block map: key d << tbits | l (l <= tpr
// < 2^tbits), partitioned by d below.
__device__ __forceinline__ uint32_t route_key(uint32_t t, int tiles_x, int nranks, int blocks_x, int tb,
                                              uint32_t tbits, uint32_t drop_key) {
  if (t == drop_key) return (uint32_t)nranks << tbits;  // dropped by the refinement: after every rank's entries
  uint32_t d;
  const uint32_t l = rt_tile_local((int)(t % (uint32_t)tiles_x), (int)(t / (uint32_t)tiles_x), (uint32_t)nranks,
                                   (uint32_t)blocks_x, (uint32_t)tb, &d);
  return d << tbits | l;
}

// the slice's globals: one entry per rank, local slot tpr
__global__ __launch_bounds__(256) void route_globals_kernel(const uint32_t* global, uint32_t nglobal, int nranks,
                                                            uint32_t tpr, uint32_t tbits, uint32_t* keys,
                                                            uint32_t* vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nglobal * (uint32_t)nranks) return;
  const uint32_t d = i / nglobal, g = i % nglobal;
  keys[i] = d << tbits | tpr;
  vals[i] = global[g];
}

// Stable partition of the routed entries by destination rank, packed for
// the exchange (replaces a radix sort on the rank bits + rank_bounds + pack:
// 3 launches and a scan instead of 9; the produce step is latency-bound at
// 1/N of a frame).  Wave w owns entries [w kPartChunk, (w + 1) kPartChunk);
// part_count_kernel -> hist[d nw + w] = its entries of rank d (d <= nranks,
// nranks = dropped) -> exclusive scan (rank-major: every rank's entries in
// wave order) -> part_scatter_kernel writes each entry at its rank's running
// offset, in entry order (a per-step ballot per distinct rank), 3 words
// (local tile or tpr, prim, skip bits); start[d] = hist offset of (d, 0).
constexpr uint32_t kPartSteps = 16, kPartChunk = 64 * kPartSteps;

// (with the routing of the entries [0, nroute) fused in: route_kernel's
// key, written back for part_scatter; the globals past them come routed)
__global__ __launch_bounds__(64) void part_count_kernel(uint32_t* keys, uint32_t n, uint32_t tbits, int nranks,
                                                        uint32_t* hist, uint32_t nroute, int tiles_x, int blocks_x,
                                                        int tb, uint32_t drop_key, const uint32_t* total_dev) {
  __shared__ uint32_t cnt[257];
  const int lane = threadIdx.x;
  const uint32_t nw = gridDim.x, w = blockIdx.x;
  for (int d = lane; d <= nranks; d += 64) cnt[d] = 0u;
  __syncthreads();
  const uint32_t e0 = w * kPartChunk, e1 = e0 + kPartChunk < n ? e0 + kPartChunk : n;
  const uint32_t own = total_dev ? *total_dev : nroute;  // entries the build wrote (async: <= nroute)
  uint32_t k[kPartSteps];  // every load in flight at once (the pass is latency-bound)
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    k[t] = i < e1 ? keys[i] : 0u;
  }
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    if (i < e1 && i < nroute) {
      const uint32_t key = route_key(i < own ? k[t] : drop_key, tiles_x, nranks, blocks_x, tb, tbits, drop_key);
      keys[i] = key;
      k[t] = key;
    }
    k[t] = i < e1 ? k[t] >> tbits : 0xffffffffu;
  }
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++)
    if (k[t] != 0xffffffffu) atomicAdd(&cnt[k[t]], 1u);
  __syncthreads();
  for (int d = lane; d <= nranks; d += 64) hist[(size_t)d * nw + w] = cnt[d];
}

__global__ __launch_bounds__(64) void part_scatter_kernel(const uint32_t* keys, const uint32_t* prims,
                                                          const float* skip, uint32_t n, uint32_t tbits, int nranks,
                                                          const uint32_t* off, uint32_t* start, uint32_t* out,
                                                          const uint32_t* ctr) {
  __shared__ uint32_t base[257];
  const int lane = threadIdx.x;
  const uint32_t nw = (n + kPartChunk - 1) / kPartChunk, w = blockIdx.x;  // (one workgroup when n = 0)
  for (int d = lane; d <= nranks; d += 64) {
    base[d] = nw ? off[(size_t)d * nw + w] : 0u;
    if (w == 0) start[d] = base[d];
  }
  // the build's counters beside the starts: the host reads both in one copy
  if (w == 0 && lane < 8) start[nranks + 1 + lane] = ctr[lane];
  __syncthreads();
  const uint32_t e0 = w * kPartChunk, e1 = e0 + kPartChunk < n ? e0 + kPartChunk : n;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t kk[kPartSteps], pr[kPartSteps];
  float sk[kPartSteps];
  // the chunk's keys, prims and skip bounds in flight at once (latency-bound)
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    kk[t] = i < e1 ? keys[i] : 0xffffffffu;
    pr[t] = i < e1 ? prims[i] : 0u;
  }
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) sk[t] = kk[t] != 0xffffffffu ? skip[pr[t]] : 0.0f;
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    if (e0 + t * 64u >= e1) break;
    const bool valid = i < e1;
    const uint32_t key = kk[t];
    const uint32_t d = key >> tbits;
    uint64_t left = __ballot(valid);
    uint32_t pos = 0;
    while (left) {  // one round per distinct rank of this step's entries
      const int first = __ffsll((long long)left) - 1;
      const uint32_t dd = (uint32_t)__shfl((int)d, first, 64);
      const uint64_t m = __ballot(valid && d == dd) & left;
      // (one wave: its LDS read of base[dd] completes before its write)
      const uint32_t b = base[dd];
      if (valid && d == dd) pos = b + (uint32_t)__popcll(m & lt);
      if (lane == first) base[dd] = b + (uint32_t)__popcll(m);
      left &= ~m;
    }
    if (valid && d < (uint32_t)nranks) {
      out[3 * (size_t)pos] = key & ((1u << tbits) - 1u);
      out[3 * (size_t)pos + 1] = pr[t];
      out[3 * (size_t)pos + 2] = __float_as_uint(sk[t]);
    }
  }
}

// Stable compaction of the (key, value) entries whose key is not drop_key
// (the per-tile refinement drops ~55 % of C5's entries: the sort then runs
// over the kept ones only).  Wave w owns entries [w kPartChunk, (w + 1)
// kPartChunk): compact_count_kernel -> cnt[w] -> exclusive scan (off, off[nw]
// = the kept total) -> compact_scatter_kernel writes the kept entries in
// order at off[w] + their rank in the wave; past cap they are not written
// and ctr7 is set (the host sized cap from the same frame's earlier build).
__global__ __launch_bounds__(64) void compact_count_kernel(const uint32_t* keys, uint32_t n, uint32_t drop_key,
                                                           uint32_t* cnt, const uint32_t* n_dev) {
  const int lane = threadIdx.x;
  const uint32_t e0 = blockIdx.x * kPartChunk;
  const uint32_t m = n_dev && *n_dev < n ? *n_dev : n;  // the build's own entries (the rest: unused)
  uint32_t c = 0;
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    c += (i < m && keys[i] != drop_key) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) cnt[blockIdx.x] = c;
  if (blockIdx.x == 0 && lane == 0) cnt[gridDim.x] = 0u;  // the scan's last input
}

__global__ __launch_bounds__(64) void compact_scatter_kernel(const uint32_t* keys, const uint32_t* vals, uint32_t n,
                                                             uint32_t drop_key, const uint32_t* off, uint32_t cap,
                                                             uint32_t* keys_out, uint32_t* vals_out, uint32_t* ctr7,
                                                             const uint32_t* n_dev) {
  const int lane = threadIdx.x;
  const uint32_t e0 = blockIdx.x * kPartChunk;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t m = n_dev && *n_dev < n ? *n_dev : n;
  // fewer kept entries than cap -- never expected for the same frame -- leave
  // a tail: dropped (every workgroup a strided part of it)
  for (uint32_t i = off[gridDim.x] + blockIdx.x * 64u + (uint32_t)lane; i < cap; i += gridDim.x * 64u)
    keys_out[i] = drop_key;
  uint32_t k[kPartSteps], v[kPartSteps];
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const uint32_t i = e0 + t * 64u + (uint32_t)lane;
    k[t] = i < m ? keys[i] : drop_key;
    v[t] = i < m ? vals[i] : 0u;
  }
  uint32_t base = off[blockIdx.x];
#pragma unroll
  for (uint32_t t = 0; t < kPartSteps; t++) {
    const bool keep = k[t] != drop_key;
    const uint64_t m = __ballot(keep);
    const uint32_t pos = base + (uint32_t)__popcll(m & lt);
    if (keep) {
      if (pos < cap) {
        keys_out[pos] = k[t];
        vals_out[pos] = v[t];
      } else {
        *ctr7 = 1u;
      }
    }
    base += (uint32_t)__popcll(m);
  }
}

__global__ __launch_bounds__(256) void unpack_kernel(const uint32_t* in, uint32_t n, uint32_t ntiles, uint32_t tpr,
                                                     uint32_t* keys, uint32_t* idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t l = in[3 * (size_t)i];
  keys[i] = l >= tpr ? ntiles : l;  // the globals after every tile
  idx[i] = i;
}

__global__ __launch_bounds__(256) void gather_kernel(const uint32_t* in, const uint32_t* idx, uint32_t n,
                                                     uint32_t* cand, float* skip) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t k = 3 * (size_t)idx[j];
  cand[j] = in[k + 1];
  skip[j] = __uint_as_float(in[k + 2]);
}

// Work order of the trace kernel's tiles (longest processing time first): a
// tile's camera-candidate entries predict its cost (r = 0.89 on C5,
// tools/tile_cost.py), so tiles with more than 8x the mean go first and the
// persistent waves' last items are short ones.  flags -> exclusive scan ->
// perm: heavy tiles first, then the rest, each in their own order.
// a tile is heavy when its list is longer than 8x the mean; the mean over
// the entries with a tile (start[ntiles], read here: the host's total also
// counts the entries the refinement dropped).
// Also heavy (item_cost != NULL: the same frame rendered before on this
// context): a tile one of whose items took more than a quarter of a
// balanced wave's share of that trace (cost_sum / waves).  Long reflection
// chains cost little camera-candidate work -- C5's worst items at N = 8 are
// mirror paths through tiles of 30-60 entries -- and one of them started
// late ran past every other wave: rank 0 of 8 traced in 1.23 ms against
// 0.88-0.97 for the others with the same total clocks (tools/tile_cost.py).
__global__ __launch_bounds__(256) void heavy_flag_kernel(const uint32_t* start, uint32_t ntiles,
                                                         uint32_t* flags, const uint32_t* item_cost,
                                                         const unsigned long long* cost_sum, uint32_t waves) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  const uint32_t total = start[ntiles] - start[0];
  bool heavy = t < ntiles && (unsigned long long)(start[t + 1] - start[t]) * ntiles > 8ull * (unsigned long long)total;
  if (item_cost && t < ntiles && !heavy) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) m = item_cost[4 * (size_t)t + k] > m ? item_cost[4 * (size_t)t + k] : m;
    heavy = 4.0 * (double)m * (double)waves > (double)*cost_sum;
  }
  flags[t] = heavy ? 1u : 0u;
}

__global__ __launch_bounds__(256) void heavy_perm_kernel(const uint32_t* flags, const uint32_t* pos,
                                                         uint32_t ntiles, uint32_t* perm) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint32_t nheavy = pos[ntiles];
  perm[flags[t] ? pos[t] : nheavy + t - pos[t]] = t;
}


// Exclusive scan of in[0 .. n] (n + 1 values: out[n] = the sum of in[0 ..
// n - 1], also written to *total) with n read on the device (min(*n_dev,
// nmax); n_dev NULL: nmax) -- the classification's scan runs over the listed
// prims only, whose count the host does not know before its one
// synchronisation.  Three passes over tiles of kScanTile values: tile sums,
// one workgroup scanning them, tile-local scans through LDS (coalesced loads
// and stores).  Deterministic (integer adds).
constexpr int kScanThreads = 256, kScanPer = 16, kScanTile = kScanThreads * kScanPer;

__device__ __forceinline__ uint32_t scan_len(uint32_t nmax, const uint32_t* n_dev) {
  const uint32_t n = n_dev ? *n_dev : nmax;
  return (n < nmax ? n : nmax) + 1u;
}

// exclusive scan of one value per thread over a 256-thread block; *sum = total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* sh, uint32_t* sum) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < kScanThreads / 64; k++) {
    if (k < wv) before += sh[k];
    tot += sh[k];
  }
  __syncthreads();
  *sum = tot;
  return before + inc - x;
}

__global__ __launch_bounds__(kScanThreads) void scan_sums_kernel(const uint32_t* __restrict__ in, uint32_t nmax,
                                                                 const uint32_t* n_dev, uint32_t* bsum) {
  __shared__ uint32_t sh[kScanThreads / 64];
  const uint32_t n1 = scan_len(nmax, n_dev), base = blockIdx.x * (uint32_t)kScanTile;
  uint32_t x = 0;
  if (base < n1)
    for (int k = 0; k < kScanPer; k++) {
      const uint32_t i = base + (uint32_t)(k * kScanThreads) + threadIdx.x;
      if (i < n1) x += in[i];
    }
  uint32_t tot;
  block_excl_scan(x, sh, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// The tiles' prefix: each apply workgroup sums the tile sums before its own
// (a few thousand tiles at most: ~10 loads per thread from L2) instead of a
// one-workgroup pass over them between the two launches.
// SCATTER (the fast path's flags over the build's slice, CandParams p): the
// exclusive prefix of a flagged prim is its place in the compact list, which
// this pass writes directly (list[o] = prim), and the scan's last value is
// the list length (ctr[3]) -- no offsets array, no scatter launch.
template <bool SCATTER>
__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(const uint32_t* __restrict__ in, uint32_t* out,
                                                                  uint32_t nmax, const uint32_t* n_dev,
                                                                  const uint32_t* bsum, uint32_t* total,
                                                                  CandParams p) {
  __shared__ uint32_t v[kScanTile + kScanThreads];  // thread t's 16 values at t * 17 (no bank conflicts)
  __shared__ uint32_t sh[kScanThreads / 64];
  const uint32_t n1 = scan_len(nmax, n_dev), base = blockIdx.x * (uint32_t)kScanTile;
  if (base >= n1) return;  // uniform per block
  const int t = threadIdx.x;
  uint32_t before = 0;
  for (uint32_t b = (uint32_t)t; b < blockIdx.x; b += kScanThreads) before += bsum[b];
  uint32_t tot0;
  block_excl_scan(before, sh, &tot0);  // tot0 = the tiles before this one
  for (int k = 0; k < kScanPer; k++) {
    const uint32_t e = (uint32_t)(k * kScanThreads + t), i = base + e;
    v[e + e / kScanPer] = i < n1 ? in[i] : 0u;
  }
  __syncthreads();
  uint32_t run = 0;
  for (int k = 0; k < kScanPer; k++) run += v[t * (kScanPer + 1) + k];
  uint32_t tot;
  uint32_t pre = tot0 + block_excl_scan(run, sh, &tot);
  uint32_t flags = 0;  // SCATTER: which of this thread's values were set
  for (int k = 0; k < kScanPer; k++) {
    const uint32_t x = v[t * (kScanPer + 1) + k];
    if (SCATTER && x) flags |= 1u << k;
    v[t * (kScanPer + 1) + k] = pre;
    pre += x;
  }
  if (SCATTER) {
    // thread t's values are elements t * 16 + k of the tile: write the list
    // entries of its flagged ones (in[] holds 0 / 1)
    for (int k = 0; k < kScanPer; k++) {
      const uint32_t e = (uint32_t)(t * kScanPer + k), i = base + e;
      if (i >= n1) break;
      const uint32_t o = v[t * (kScanPer + 1) + k];
      if (i == n1 - 1u) {
        p.ctr[3] = o;  // list length (the scan's last input is 0)
      } else if ((flags >> k) & 1u) {
        p.list[o] = slice_prim(p, i);
      }
    }
    return;
  }
  __syncthreads();
  for (int k = 0; k < kScanPer; k++) {
    const uint32_t e = (uint32_t)(k * kScanThreads + t), i = base + e;
    if (i < n1) {
      const uint32_t o = v[e + e / kScanPer];
      out[i] = o;
      if (i == n1 - 1u && total) *total = o;
    }
  }
}

// Exclusive scan of in[0 .. n] (n + 1 values, out[n] = their sum) in one
// workgroup, for the short scans between list passes (the big footprints'
// items, a partition's per-wave counts, a rank's work order): one launch
// instead of rocPRIM's two.  Wave w owns a contiguous segment of the values,
// loaded and stored lane-consecutive (coalesced) in steps of 64, its lanes'
// values held in registers; a wave scan per step with a running carry, the
// 16 waves' totals combined through LDS.
constexpr uint32_t kSmallScanThreads = 1024, kSmallScanPer = 32;
constexpr uint32_t kSmallScanWaves = kSmallScanThreads / 64;
constexpr uint32_t kSmallScanMax = kSmallScanThreads * kSmallScanPer;

__global__ __launch_bounds__(kSmallScanThreads) void scan_small_kernel(const uint32_t* __restrict__ in,
                                                                       uint32_t* __restrict__ out, uint32_t n) {
  __shared__ uint32_t wsum[kSmallScanWaves];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t m = n + 1u;
  const uint32_t seg = ((m + kSmallScanWaves - 1u) / kSmallScanWaves + 63u) & ~63u;  // per wave, whole steps
  const uint32_t base = wv * seg, steps = seg / 64u;
  uint32_t v[kSmallScanPer], tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSmallScanPer; k++) {
    const uint32_t i = base + k * 64u + lane;
    v[k] = (k < steps && i < m) ? in[i] : 0u;
    tot += v[k];
  }
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if (lane == 0) wsum[wv] = tot;
  __syncthreads();
  uint32_t carry = 0;
  for (uint32_t k = 0; k < wv; k++) carry += wsum[k];
#pragma unroll
  for (uint32_t k = 0; k < kSmallScanPer; k++) {
    if (k < steps) {  // (uniform)
      uint32_t inc = v[k];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if ((int)lane >= o) inc += y;
      }
      const uint32_t i = base + k * 64u + lane;
      if (i < m) out[i] = carry + inc - v[k];
      carry += __shfl(inc, 63, 64);
    }
  }
}

}  // namespace rtc

#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" hipError_t rt_cand_prim_leaf(const float4* node, uint32_t nnode, const float4* tri,
                                        uint32_t* prim_leaf, hipStream_t s) {
  if (nnode == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::prim_leaf_kernel, dim3((nnode + 255) / 256), dim3(256), 0, s, node, nnode,
                     tri, prim_leaf);
  return hipGetLastError();
}

extern "C" int rt_cand_survey_host(const CandParams* p, const float* tri, const float* node,
                                   const uint32_t* prim_leaf, int threads,
                                   unsigned long long out[88]) {
  // out: [0] safe, [1] footprint, [2] global, [3] entries, [4 + k] prims
  // with 2^k <= entries < 2^(k+1), [20 + k] their entries (k < 16);
  // [36 + k] footprint prims whose T_D box (grown by the distance error
  // beyond the pruning margin) reaches beyond the triangle's own box by
  // g with 2^(k-8) <= g / eps_avail < 2^(k-7) (k = 0: below 2^-7; k = 15:
  // 2^7 and more, or unbounded), [52 + k] their entries
  // [71..77]: quick_class's verdicts (listed; of those classify() SAFE
  // through the leaf box, SAFE otherwise, FOOTPRINT without a tile, GLOBAL;
  // Q_SAFE; Q_AWAY); [78] / [79] listed and SAFE by the reach / steepness
  // exits; [80] Q_SAFE that classify() does not confirm
  for (int k = 0; k < 88; k++) out[k] = 0;
  if (threads < 1) threads = 1;
  std::vector<unsigned long long> part(88 * (size_t)threads, 0);
  std::vector<unsigned long long> bad((size_t)threads, 0);
  std::vector<std::thread> th;
#ifdef RT_SURVEY_DUMP
  std::vector<std::vector<double>> dump((size_t)threads);
#endif
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t]() {
      unsigned long long* o = &part[88 * (size_t)t];
      for (uint32_t i = (uint32_t)t; i < p->nprim; i += (uint32_t)threads) {
        rtc::Footprint fp;
        const float* lb = prim_leaf ? node + 8 * (size_t)prim_leaf[i] : nullptr;
        double td[18];
        const float* rec = tri + 12 * (size_t)i;
        const int c = rtc::classify(*p, rec, lb, fp, td);
        o[c]++;
        const int qc = rtc::quick_class(*p, rec);
        if (qc == rtc::Q_LIST) {
          o[71]++;
          if (c == rtc::SAFE) {
            rtc::Footprint f2;
            int why = -1;
            o[rtc::classify(*p, rec, nullptr, f2, nullptr, &why) == rtc::SAFE ? 73 : 72]++;
            if (why == 1) o[78]++;  // the error region within the slack
            if (why == 3) o[79]++;  // no candidate line steep enough to be accepted
          } else if (c == rtc::GLOBAL) {
            o[75]++;
          }
        } else {
          o[qc == rtc::Q_SAFE ? 76 : 77]++;
          if (qc == rtc::Q_SAFE && c != rtc::SAFE) {
            o[80]++;  // the fast path's proof must hold
            if (getenv("RT_SURVEY_VIOL") && o[80] <= 8) {
              float dq[4];
              rtc::quick_class(*p, rec, dq);
              rtc::Footprint f3;
              double t3[18];
              for (double& x : t3) x = -9.0;
              rtc::classify(*p, rec, nullptr, f3, t3);
              fprintf(stderr, "viol prim %u c %d: f32 h %.6g derr %.6g cl %.6g a %.6g | f64 hreach %.6g cl %.6g kmax %.6g e_a %.6g derr %.6g eps %.6g\n",
                      i, c, dq[0], dq[1], dq[2], dq[3], t3[13], t3[12], t3[14], t3[15], t3[6], p->eps_avail);
            }
          }
        }
        if (c == rtc::FOOTPRINT) {
          unsigned long long v = 0, kept = 0;
          rtc::raster(*p, fp, [&](uint32_t tl) {
            v++;
            int tx, ty;
            rt_tile_xy(tl, (uint32_t)p->rank, (uint32_t)p->nranks, (uint32_t)p->blocks_x, (uint32_t)p->tb, &tx, &ty);
            kept += rtc::tile_keep(*p, rec, tx, ty) ? 1u : 0u;
          });
          if (rtc::refined_footprint(*p, fp)) {  // the device refines these (CandParams::refine)
            o[68] += kept;
            o[69] += v;
            o[70] += kept;
          } else {
            o[68] += v;
          }
          // big_count_kernel counts rows through row_ivs (big_item_kernel's intervals)
          unsigned long long vi = 0;
          int q0, q1;
          if (rtc::raster_rows(*p, fp, q0, q1))
            for (int ty = q0 >> 3; ty <= (q1 >> 3); ty++) {
              int x[6], fb[3];
              uint32_t cn[3];
              rtc::row_ivs(*p, fp, ty, q0, q1, x, fb, cn);
              vi += cn[0] + cn[1] + cn[2];
            }
          if (v != rtc::raster_count(*p, fp) || vi != v) {
            bad[t]++;  // the device count pass must agree
#ifdef RT_SURVEY_DEBUG
            int r0, r1;
            rtc::raster_rows(*p, fp, r0, r1);
            for (int ty = r0 >> 3; ty <= (r1 >> 3); ty++) {
              unsigned long long vr = 0;
              rtc::raster_row(*p, fp, ty, r0, r1, [&](uint32_t) { vr++; });
              int a0, a1, b0, b1;
              rtc::row_tiles(*p, fp, ty, r0, r1, a0, a1, b0, b1);
              if (vr != rtc::count_row(*p, fp, ty, r0, r1))
                fprintf(stderr, "prim %u ty %d iter %llu count %u a %d..%d b %d..%d\n", i, ty, vr,
                        rtc::count_row(*p, fp, ty, r0, r1), a0, a1, b0, b1);
            }
#endif
          }
          o[3] += v;
          if (!v && qc == rtc::Q_LIST) o[74]++;
          int k = 0;
          while (k < 15 && (2ull << k) <= v) k++;
          if (v) {
            o[4 + k]++;
            o[20 + k] += v;
          }
          double g = 1e300;
          if (td[6] >= 0.0) {
            g = fmax(0.0, td[6] - 2.0 * p->eps_avail);
            for (int a = 0; a < 3; a++) {
              const double lo = fmin((double)rec[a], fmin((double)rec[a] + rec[3 + a], (double)rec[a] + rec[6 + a]));
              const double hi = fmax((double)rec[a], fmax((double)rec[a] + rec[3 + a], (double)rec[a] + rec[6 + a]));
              g = fmax(g, fmax(lo - td[a], td[3 + a] - hi) + fmax(0.0, td[6] - 2.0 * p->eps_avail));
            }
          }
          int kg = 0;
          while (kg < 15 && g >= p->eps_avail * std::ldexp(1.0, kg - 7)) kg++;
          o[36 + kg]++;
          o[52 + kg] += v;
#ifdef RT_SURVEY_DUMP
          dump[t].push_back((double)i);
          dump[t].push_back((double)v);
          for (int q = 7; q < 18; q++) dump[t].push_back(td[q]);
#endif
        }
      }
    });
  for (auto& x : th) x.join();
#ifdef RT_SURVEY_DUMP
  if (const char* fn = getenv("RT_SURVEY_DUMP_FILE")) {
    FILE* fo = fopen(fn, "wb");
    for (auto& d : dump) fwrite(d.data(), sizeof(double), d.size(), fo);
    fclose(fo);
  }
#endif
  for (int k = 0; k < 88; k++) {
    out[k] = 0;
    for (int t = 0; t < threads; t++) out[k] += part[88 * (size_t)t + k];
  }
  unsigned long long nbad = 0;
  for (int t = 0; t < threads; t++) nbad += bad[t];
  return nbad ? -1 : 0;
}

// Host sample of the per-tile refinement (tests: tests/test_exact.py checks
// each dropped entry against the reference's float test on every camera
// sample of its tile): every stride-th (prim, tile) entry of a refined
// footprint (rtc::refined_footprint; no leaf boxes), 4 words each: prim, tx,
// ty, kept.  Returns the entries written (at most cap); *total = all sampled.
extern "C" size_t rt_cand_refine_sample_host(const CandParams* p, const float* tri, uint32_t stride,
                                             uint32_t* out, size_t cap, size_t* total) {
  const int threads = 8;
  std::vector<std::vector<uint32_t>> part(threads);
  std::vector<std::thread> th;
  if (stride < 1) stride = 1;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t]() {
      for (uint32_t i = (uint32_t)t; i < p->nprim; i += (uint32_t)threads) {
        rtc::Footprint fp;
        const float* rec = tri + 12 * (size_t)i;
        if (rtc::classify(*p, rec, nullptr, fp) != rtc::FOOTPRINT || !rtc::refined_footprint(*p, fp)) continue;
        uint64_t k = 0;
        rtc::raster(*p, fp, [&](uint32_t tl) {
          if (((uint64_t)i * 7919u + k++) % stride != 0) return;
          int tx, ty;
          rt_tile_xy(tl, (uint32_t)p->rank, (uint32_t)p->nranks, (uint32_t)p->blocks_x, (uint32_t)p->tb, &tx, &ty);
          const uint32_t e[4] = {i, (uint32_t)tx, (uint32_t)ty, rtc::tile_keep(*p, rec, tx, ty) ? 1u : 0u};
          part[t].insert(part[t].end(), e, e + 4);
        });
      }
    });
  for (auto& x : th) x.join();
  size_t n = 0, all = 0;
  for (auto& v : part) {
    all += v.size() / 4;
    for (size_t j = 0; j + 4 <= v.size() && n < cap; j += 4, n++) std::memcpy(out + 4 * n, &v[j], 16);
  }
  *total = all;
  return n;
}

// Host check of the device-built lists of one frame (tests): every prim the
// float fast path listed is re-classified on the host (same code, so the
// same f64 bits; the safe ones have no tiles), every kept footprint compared
// bit for bit, and every tile's list equal, as a multiset, to the tiles the
// host raster gives the listed footprints.  out: [0] listed prims, [1] entries,
// [2] footprint mismatches, [3] tile-list mismatches (tiles), [4] globals,
// [5] fast-path filter violations, [6] prims the rank/frame filter dropped.
extern "C" int rt_cand_verify_host(const CandParams* p, const float* tri, const float* node,
                                   const uint32_t* prim_leaf, const uint32_t* list, uint32_t nlist,
                                   const void* fp_dev, const uint32_t* start, const uint32_t* cand,
                                   uint32_t ntiles, unsigned long long out[7]) {
  for (int k = 0; k < 7; k++) out[k] = 0;
  out[0] = nlist;
  out[1] = start[ntiles];
  const rtc::Footprint* fpd = (const rtc::Footprint*)fp_dev;
  // host threads: the process's share (OMP_NUM_THREADS on the GPU box), at
  // most 64 -- C5 re-classifies ~10^7 prims in f64
  int threads = (int)std::thread::hardware_concurrency();
  if (const char* e = std::getenv("OMP_NUM_THREADS"))
    if (std::atoi(e) > 0) threads = std::atoi(e);
  threads = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  std::vector<std::vector<uint64_t>> pairs(threads);  // (tile << 32 | prim) the host raster gives
  std::vector<unsigned long long> cnt(7 * (size_t)threads, 0);
  auto leafbox = [&](uint32_t prim) { return prim_leaf ? node + 8 * (size_t)prim_leaf[prim] : nullptr; };
  std::vector<unsigned char> listed(p->nprim + 1, 0);
  for (uint32_t j = 0; j < nlist; j++) listed[list[j]] = 1;
  std::vector<std::thread> th;
  for (int ti = 0; ti < threads; ti++)
    th.emplace_back([&, ti]() {
      unsigned long long* o = &cnt[7 * (size_t)ti];
      // every prim the fast path listed: re-classified, its footprint
      // compared with the device's bit for bit, its tiles collected
      for (uint32_t j = (uint32_t)ti; j < nlist; j += (uint32_t)threads) {
        const uint32_t prim = list[j];
        rtc::Footprint fp;
        std::memset(&fp, 0, sizeof fp);
        const int c = rtc::classify(*p, tri + 12 * (size_t)prim, leafbox(prim), fp);
        if (c == rtc::GLOBAL) {
          o[4]++;
          continue;
        }
        if (c != rtc::FOOTPRINT) continue;  // safe after all (leaf box): no tiles
        // a tall footprint's tiles (rtc::refined_footprint) refined per tile when p->refine
        const bool refine = p->refine && rtc::refined_footprint(*p, fp);
        const float* rec = tri + 12 * (size_t)prim;
        uint32_t n = 0;
        rtc::raster(*p, fp, [&](uint32_t t) {
          int tx, ty;
          rt_tile_xy(t, (uint32_t)p->rank, (uint32_t)p->nranks, (uint32_t)p->blocks_x, (uint32_t)p->tb, &tx, &ty);
          if (t < ntiles && (!refine || rtc::tile_keep(*p, rec, tx, ty))) pairs[ti].push_back((uint64_t)t << 32 | prim);
          n++;
        });
        if (n == 0) continue;  // the device keeps no footprint without tiles
        const rtc::Footprint& d = fpd[j];
        // (k, l, dimg are only set -- and only read -- with tri_ok)
        bool same = d.tri_ok == fp.tri_ok && d.b0 == fp.b0 && d.b1 == fp.b1 && d.b2 == fp.b2 &&
                    d.hw == fp.hw && d.hw0 == fp.hw0 && d.skip == fp.skip;
        if (same && fp.tri_ok) same = d.dimg == fp.dimg;
        for (int k = 0; k < 3 && same && fp.tri_ok; k++) same = d.k[k] == fp.k[k] && d.l[k] == fp.l[k];
        if (!same) o[2]++;
      }
      // prims the fast path did not list: proven safe, or their footprint has
      // no tile of this rank (the rank/frame filter must never drop a needed one)
      const uint32_t chunk = (p->nprim + (uint32_t)threads - 1) / (uint32_t)threads;
      const uint32_t b = (uint32_t)ti * chunk, e = b + chunk < p->nprim ? b + chunk : p->nprim;
      for (uint32_t prim = b; prim < e; prim++) {
        const int qc = rtc::quick_class(*p, tri + 12 * (size_t)prim);
        if (listed[prim]) {
          if (qc != rtc::Q_LIST) o[5]++;
          continue;
        }
        if (qc == rtc::Q_LIST) {  // the device should have listed it
          o[5]++;
          continue;
        }
        // Q_SAFE: the float fast path's proof checked against the f64 one --
        // a prim it calls safe must have no tile here by classify() either;
        // Q_AWAY: the rank/frame filter's drop, likewise
        rtc::Footprint fp;
        const int c = rtc::classify(*p, tri + 12 * (size_t)prim, leafbox(prim), fp);
        if (c == rtc::GLOBAL || (c == rtc::FOOTPRINT && rtc::raster_count(*p, fp) != 0)) o[5]++;
        if (qc != rtc::Q_SAFE) o[6]++;
      }
    });
  for (auto& x : th) x.join();
  for (int ti = 0; ti < threads; ti++)
    for (int k = 2; k < 7; k++) out[k] += cnt[7 * (size_t)ti + k];
  // every tile's list as a multiset: the host pairs sorted (tile, prim)
  // against each tile's sorted device entries
  size_t np = 0;
  for (auto& v : pairs) np += v.size();
  std::vector<uint64_t> want;
  want.reserve(np);
  for (auto& v : pairs) {
    want.insert(want.end(), v.begin(), v.end());
    std::vector<uint64_t>().swap(v);
  }
  std::sort(want.begin(), want.end());
  size_t w = 0;
  std::vector<uint32_t> got;
  for (uint32_t t = 0; t < ntiles; t++) {
    got.assign(cand + start[t], cand + start[t + 1]);
    std::sort(got.begin(), got.end());
    bool same = true;
    size_t k = 0;
    for (; w < want.size() && (uint32_t)(want[w] >> 32) == t; w++, k++)
      same = same && k < got.size() && got[k] == (uint32_t)want[w];
    if (!same || k != got.size()) out[3]++;
  }
  return 0;
}

extern "C" size_t rt_cand_footprint_bytes(void) { return sizeof(rtc::Footprint); }

extern "C" hipError_t rt_cand_quick(const CandParams* p, hipStream_t s) {
  const uint32_t len = p->prim1 - p->prim0;
  if (len == 0) {  // no quick_kernel to zero the counters and the scan's last input
    hipError_t e = hipMemsetAsync(p->ctr, 0, 8 * sizeof(uint32_t), s);
    return e != hipSuccess ? e : hipMemsetAsync(p->visits, 0, sizeof(uint32_t), s);
  }
  hipLaunchKernelGGL(rtc::quick_kernel, dim3((len + RT_LIST_BLOCK - 1) / RT_LIST_BLOCK), dim3(RT_LIST_BLOCK), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_scatter(const CandParams* p, hipStream_t s) {
  const uint32_t len = p->prim1 - p->prim0;
  hipLaunchKernelGGL(rtc::scatter_kernel, dim3((len + 1 + 255) / 256), dim3(256), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_count(const CandParams* p, hipStream_t s) {
  const uint32_t len = p->prim1 - p->prim0;  // the list holds prims of the slice only
  if (len == 0) return hipSuccess;
  // sized for the worst case; threads beyond the list's length exit at once
  hipLaunchKernelGGL(rtc::count_kernel, dim3((len + RT_LIST_BLOCK - 1) / RT_LIST_BLOCK), dim3(RT_LIST_BLOCK), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_big_count(const CandParams* p, hipStream_t s) {
  if (p->nprim == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::big_count_kernel, dim3(rtc::kBigWaves), dim3(64), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_emit(const CandParams* p, hipStream_t s) {
  const uint32_t len = p->prim1 - p->prim0;
  if (len == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::emit_kernel, dim3((len + RT_LIST_BLOCK - 1) / RT_LIST_BLOCK), dim3(RT_LIST_BLOCK), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_big(const CandParams* p, uint32_t nbig, hipStream_t s) {
  if (nbig == 0) return hipSuccess;
  const uint32_t g = nbig < (uint32_t)rtc::kBigWaves ? nbig : (uint32_t)rtc::kBigWaves;
  hipLaunchKernelGGL(rtc::big_kernel, dim3(g), dim3(64), 0, s, *p);
  return hipGetLastError();
}

extern "C" uint32_t rt_cand_big_waves(void) { return (uint32_t)rtc::kBigWaves; }

extern "C" hipError_t rt_cand_items(const CandParams* p, hipStream_t s) {
  hipLaunchKernelGGL(rtc::item_kernel, dim3(rtc::kBigWaves), dim3(64), 0, s, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_big_items(const CandParams* p, uint32_t nitems, int check, hipStream_t s) {
  // nitems: the items read back (check = 0), or the same frame's read-back
  // build's (check = 1: an asynchronous build; the kernels compare on the device)
  if (nitems == 0) return hipSuccess;
  if (check) {
    hipLaunchKernelGGL(rtc::big_item_kernel<true>, dim3(nitems), dim3(64), 0, s, *p);
    if (p->refine) hipLaunchKernelGGL(rtc::refine_kernel<true>, dim3(nitems), dim3(64), 0, s, *p);
  } else {
    hipLaunchKernelGGL(rtc::big_item_kernel<false>, dim3(nitems), dim3(64), 0, s, *p);
    if (p->refine) hipLaunchKernelGGL(rtc::refine_kernel<false>, dim3(nitems), dim3(64), 0, s, *p);
  }
  return hipGetLastError();
}

// entries [ctr[6], n) of keys (the buffers' unused tail in an asynchronous
// build, sized from the previous frame) get `key`: they sort after every tile
__global__ __launch_bounds__(256) void fill_tail_kernel(uint32_t* keys, const uint32_t* total, uint32_t n,
                                                        uint32_t key) {
  for (uint32_t i = *total + blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) keys[i] = key;
}

extern "C" hipError_t rt_cand_fill_tail(uint32_t* keys, const uint32_t* total_dev, uint32_t n, uint32_t key,
                                        hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_tail_kernel, dim3(1024), dim3(256), 0, s, keys, total_dev, n, key);
  return hipGetLastError();
}

extern "C" uint32_t rt_cand_scan_dev_tiles(uint32_t nmax) {
  return (nmax + 1u + (uint32_t)rtc::kScanTile - 1u) / (uint32_t)rtc::kScanTile;
}

extern "C" hipError_t rt_cand_scan_dev(const uint32_t* in, uint32_t* out, uint32_t nmax, const uint32_t* n_dev,
                                       uint32_t* total, uint32_t* bsum, hipStream_t s) {
  const uint32_t nb = rt_cand_scan_dev_tiles(nmax);
  hipLaunchKernelGGL(rtc::scan_sums_kernel, dim3(nb), dim3(rtc::kScanThreads), 0, s, in, nmax, n_dev, bsum);
  CandParams none;
  memset(&none, 0, sizeof none);
  hipLaunchKernelGGL(rtc::scan_apply_kernel<false>, dim3(nb), dim3(rtc::kScanThreads), 0, s, in, out, nmax, n_dev,
                     (const uint32_t*)bsum, total, none);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_scan_scatter(const CandParams* p, uint32_t* bsum, hipStream_t s) {
  const uint32_t len = p->prim1 - p->prim0;
  const uint32_t nb = rt_cand_scan_dev_tiles(len);
  hipLaunchKernelGGL(rtc::scan_sums_kernel, dim3(nb), dim3(rtc::kScanThreads), 0, s, p->visits, len,
                     (const uint32_t*)nullptr, bsum);
  hipLaunchKernelGGL(rtc::scan_apply_kernel<true>, dim3(nb), dim3(rtc::kScanThreads), 0, s,
                     (const uint32_t*)p->visits, (uint32_t*)nullptr, len, (const uint32_t*)nullptr,
                     (const uint32_t*)bsum, (uint32_t*)nullptr, *p);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_scan(const uint32_t* in, uint32_t* out, uint32_t n, void* temp,
                                   size_t* temp_bytes, hipStream_t s) {
  if ((size_t)n + 1 <= rtc::kSmallScanMax) {  // one workgroup, no temporary storage
    if (!temp) {
      *temp_bytes = 0;
      return hipSuccess;
    }
    hipLaunchKernelGGL(rtc::scan_small_kernel, dim3(1), dim3(rtc::kSmallScanThreads), 0, s, in, out, n);
    return hipGetLastError();
  }
  return rocprim::exclusive_scan(temp, *temp_bytes, in, out, 0u, (size_t)n + 1,
                                 rocprim::plus<uint32_t>(), s);
}

extern "C" hipError_t rt_cand_sort(uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_in,
                                   uint32_t* vals_out, uint32_t n, int begin_bit, int end_bit, void* temp,
                                   size_t* temp_bytes, hipStream_t s) {
#if RT_SORT_BITS
  // digits of RT_SORT_BITS bits per onesweep place (rocPRIM's gfx950 u32/u32
  // tuning otherwise: 8 bits, so C5's 17-bit tile keys take three places)
  // onesweep from RT_SORT_MERGE_LIMIT items up (rocPRIM's default switches
  // at 2^20: a consume of ~1 M entries at N = 8 went through 9 merge passes,
  // 0.14 ms)
  using cfg = rocprim::radix_sort_config<
      rocprim::default_config, rocprim::default_config,
      rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>,
                                          RT_SORT_BITS, rocprim::block_radix_rank_algorithm::match>,
      RT_SORT_MERGE_LIMIT>;
  return rocprim::radix_sort_pairs<cfg>(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out, (size_t)n,
                                        begin_bit, end_bit, s);
#else
  return rocprim::radix_sort_pairs(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                   (size_t)n, begin_bit, end_bit, s);
#endif
}

extern "C" hipError_t rt_cand_entry_skip(const uint32_t* cand, const float* skip, float* out,
                                         uint32_t n, const uint32_t* n_dev, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::entry_skip_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cand, skip,
                     out, n, n_dev);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_bounds(const uint32_t* keys, uint32_t n, uint32_t* start,
                                     uint32_t ntiles, uint32_t* snap, hipStream_t s) {
  hipLaunchKernelGGL(rtc::bounds_kernel, dim3((ntiles + 1 + 255) / 256), dim3(256), 0, s, keys, n,
                     start, ntiles, snap);
  return hipGetLastError();
}


extern "C" hipError_t rt_cand_route_globals(const uint32_t* global, uint32_t nglobal, int nranks, uint32_t tpr,
                                            uint32_t tbits, uint32_t* keys, uint32_t* vals, hipStream_t s) {
  const uint32_t n = nglobal * (uint32_t)nranks;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::route_globals_kernel, dim3((n + 255) / 256), dim3(256), 0, s, global, nglobal, nranks,
                     tpr, tbits, keys, vals);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_compact(const uint32_t* keys, const uint32_t* vals, uint32_t n, const uint32_t* n_dev,
                                      uint32_t drop_key, uint32_t cap, uint32_t* cnt, uint32_t* off, void* tmp,
                                      size_t* tmp_bytes, uint32_t* keys_out, uint32_t* vals_out, uint32_t* ctr7,
                                      hipStream_t s) {
  const uint32_t nw = rt_cand_part_waves(n);
  if (!tmp) return rt_cand_scan(cnt, off, nw, nullptr, tmp_bytes, s);
  if (nw == 0) return hipErrorInvalidValue;  // (the host compacts only a build with entries)
  hipLaunchKernelGGL(rtc::compact_count_kernel, dim3(nw), dim3(64), 0, s, keys, n, drop_key, cnt, n_dev);
  hipError_t e = rt_cand_scan(cnt, off, nw, tmp, tmp_bytes, s);  // off[nw] = the kept entries
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rtc::compact_scatter_kernel, dim3(nw), dim3(64), 0, s, keys, vals, n, drop_key, off, cap,
                     keys_out, vals_out, ctr7, n_dev);
  return hipGetLastError();
}

extern "C" uint32_t rt_cand_part_waves(uint32_t n) {
  return (n + rtc::kPartChunk - 1) / rtc::kPartChunk;
}

extern "C" hipError_t rt_cand_part_count(uint32_t* keys, uint32_t n, uint32_t tbits, int nranks, uint32_t* hist,
                                         uint32_t nroute, int tiles_x, int blocks_x, int tb, uint32_t drop_key,
                                         const uint32_t* total_dev, hipStream_t s) {
  const uint32_t nw = rt_cand_part_waves(n);
  if (nw == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::part_count_kernel, dim3(nw), dim3(64), 0, s, keys, n, tbits, nranks, hist, nroute,
                     tiles_x, blocks_x, tb, drop_key, total_dev);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_part_scatter(const uint32_t* keys, const uint32_t* prims, const float* skip,
                                           uint32_t n, uint32_t tbits, int nranks, const uint32_t* off,
                                           uint32_t* start, uint32_t* out, const uint32_t* ctr, hipStream_t s) {
  const uint32_t nw = rt_cand_part_waves(n);
  hipLaunchKernelGGL(rtc::part_scatter_kernel, dim3(nw ? nw : 1u), dim3(64), 0, s, keys, prims, skip, n, tbits,
                     nranks, off, start, out, ctr);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_unpack(const uint32_t* in, uint32_t n, uint32_t ntiles, uint32_t tpr, uint32_t* keys,
                                     uint32_t* idx, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::unpack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, ntiles, tpr, keys, idx);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_gather(const uint32_t* in, const uint32_t* idx, uint32_t n, uint32_t* cand,
                                     float* skip, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rtc::gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, idx, n, cand, skip);
  return hipGetLastError();
}

extern "C" hipError_t rt_cand_order(const uint32_t* start, uint32_t ntiles, uint32_t total,
                                    uint32_t* flags, uint32_t* pos, uint32_t* perm, const uint32_t* item_cost,
                                    const unsigned long long* cost_sum, uint32_t waves, void* tmp,
                                    size_t* tmp_bytes, hipStream_t s) {
  if (!tmp) return rt_cand_scan(flags, pos, ntiles, nullptr, tmp_bytes, s);
  const dim3 b(256), g((ntiles + 1 + 255) / 256);
  (void)total;
  hipLaunchKernelGGL(rtc::heavy_flag_kernel, g, b, 0, s, start, ntiles, flags, item_cost, cost_sum, waves);
  hipError_t e = rt_cand_scan(flags, pos, ntiles, tmp, tmp_bytes, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rtc::heavy_perm_kernel, g, b, 0, s, flags, pos, ntiles, perm);
  return hipGetLastError();
}
