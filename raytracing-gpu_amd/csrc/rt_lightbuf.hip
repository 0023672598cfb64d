// rt_lightbuf.hip -- light buffers for the shadow queries (rt_lightbuf.h,
// DESIGN.md §4 "Light buffers").  Built once per scene and culling slack, on
// the device: count (cells per triangle) -> scan -> emit (cell, key, prim) ->
// radix sort by (cell, key) -> cell starts.
//
// Conservative by construction, relative to the octree walk it replaces: a
// triangle is listed in every cell that a shadow ray passing within the walk's
// slack of it can start from (the float rounding of the query's own cell and
// key computations added as margins), and skipped by a query only where it
// lies entirely behind the ray's origin by more than twice that slack.  The
// walk tests a triangle when the ray passes within the slack of the leaf box
// holding it, so both find every hit within the slack of a triangle -- the same
// exactness class (DESIGN.md §2 "Shadow rays").
#include <hip/hip_runtime.h>
#include <cstring>  // before rocPRIM
#include <rocprim/rocprim.hpp>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "rt_lightbuf.h"

namespace rtl {

constexpr double kEps = 0x1p-24;
constexpr double kInvSqrt3 = 0.57735026918962573;
constexpr uint32_t kSmallCells = 1024;  // more: emitted by a workgroup
constexpr int kMaxRects = 6;

struct BP {
  const float4* tri;
  uint32_t nprim, kind;
  double lv[3];
  double u[3], v[3], w[3];  // DIR: the float axes, as doubles
  double u0, v0, cs, inv_cs;
  uint32_t nx, ny, n;       // DIR grid / POINT face side
  double slack, s1, dmax;
  uint32_t* count;
  uint32_t* off;
  unsigned long long* keys;
  uint32_t* vals;
  uint32_t* big;
  uint32_t* ctr;  // [0] big prims, [1] global prims
  uint32_t* global;
};

struct Foot {
  int n;  // rects
  uint32_t face[kMaxRects];
  int x0[kMaxRects], x1[kMaxRects], y0[kMaxRects], y1[kMaxRects];
  double key;    // whole-triangle key (ascending = tested first)
  bool global;
  // DIR per-cell refinement: the plane's depth over a cell column
  bool plane;
  double pn_u, pn_v, pn_w, pn_d;  // n.u, n.v, n.w, n.v0 of the triangle's plane
  double m;                       // footprint margin (world units)
  // per rect: the triangle's image in the rect's coordinates (DIR: u, v;
  // POINT: the face's (s, t)) and its margin there, for the cell overlap
  // test of small footprints; tri_ok = 0: bounding rect only
  bool tri_ok[kMaxRects];
  double tx[kMaxRects][3], ty[kMaxRects][3], tm[kMaxRects];
};

__device__ inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ inline uint32_t orderable(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ inline float unorder(uint32_t b) {
  return __uint_as_float((b & 0x80000000u) ? (b & 0x7fffffffu) : ~b);
}

__device__ inline int clampi(double x, int hi) {
  if (!(x > 0.0)) return 0;  // NaN -> 0
  if (x >= (double)hi) return hi;
  return (int)x;
}

__device__ void footprint(const BP& p, uint32_t prim, Foot& f) {
  const float* r = (const float*)(p.tri + 3 * (size_t)prim);
  const double v0[3] = {r[0], r[1], r[2]}, e1[3] = {r[3], r[4], r[5]}, e2[3] = {r[6], r[7], r[8]};
  const double V[3][3] = {{v0[0], v0[1], v0[2]},
                          {v0[0] + e1[0], v0[1] + e1[1], v0[2] + e1[2]},
                          {v0[0] + e2[0], v0[1] + e2[1], v0[2] + e2[2]}};
  f.n = 0;
  f.global = false;
  f.plane = false;
  for (int q = 0; q < kMaxRects; q++) f.tri_ok[q] = false;
  if (p.kind == RT_LB_DIR) {
    // the query's float projection of its origin is within 3 eps s1 of the
    // exact one; the triangle's points are within the slack of the ray
    const double m = p.slack + 3.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1;
    double lu = 1e300, hu = -1e300, lvv = 1e300, hvv = -1e300, hw = -1e300;
    for (int k = 0; k < 3; k++) {
      const double a = dot3(V[k], p.u), b = dot3(V[k], p.v), c = dot3(V[k], p.w);
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
    // skipped by a query when its deepest point, grown by the slack on both
    // sides (behind-origin tolerance of the walk) and the rounding of the
    // query's depth, lies below the origin: key = -(that bound)
    f.key = -(hw + 2.0 * p.slack + 6.0 * kEps * p.s1 * 1.01 + 1e-9 * p.s1);
    f.m = m;
    const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                         e1[0] * e2[1] - e1[1] * e2[0]};
    const double nl = sqrt(dot3(n, n));
    f.pn_u = dot3(n, p.u);
    f.pn_v = dot3(n, p.v);
    f.pn_w = dot3(n, p.w);
    f.pn_d = dot3(n, v0);
    f.plane = nl > 0.0 && fabs(f.pn_w) > 0.05 * nl;
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
    rb = fmax(rb, sqrt(dot3(d, d)));
  }
  rb = rb * (1.0 + 1e-12) + p.slack + 1e-12;
  const double D[3] = {C[0] - p.lv[0], C[1] - p.lv[1], C[2] - p.lv[2]};
  const double dc = sqrt(dot3(D, D));
  if (!(dc > rb * 1.001 + 1e-9)) {
    f.global = true;
    return;
  }
  const double rmin = dc - rb;
  const double alpha = 4.0 * 1.7320508075688772 * kEps * p.dmax / rmin + 8.0 * kEps;
  const double th = asin(fmin(1.0, rb / dc)) + alpha + 1e-12;
  if (!(th < 1.2)) {
    f.global = true;
    return;
  }
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
      // beta (slack / rmin + alpha) through the face map's Lipschitz bound
      {
        const double beta = p.slack / rmin + alpha;
        const double sgn = sg == 0 ? 1.0 : -1.0;
        double xamin = 1e300, smax = 1.0;
        bool ok = true;
        for (int v = 0; v < 3 && ok; v++) {
          const double X[3] = {V[v][0] - p.lv[0], V[v][1] - p.lv[1], V[v][2] - p.lv[2]};
          const double xl = sqrt(dot3(X, X)), xa = sgn * X[a];
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
  // a query toward the light stops once the triangle's nearest possible
  // point lies farther from the light than its origin (plus the slack)
  f.key = rmin - 2.0 * p.slack - 1e-9 * p.dmax;
}

__device__ inline uint64_t foot_cells(const BP& p, const Foot& f) {
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
    const double kc = -(h + 2.0 * p.slack + 6.0 * kEps * p.s1 * 1.01 + 1e-6 * p.s1);
    key = fmax(key, kc);  // the tighter (larger) of the two lower bounds of -depth
  }
  return __double2float_rd(key);
}

// Can the triangle's grown image in rect q reach cell (x, y)?  Separating
// axis test of the cell square (grown by the margin) against the image's edge
// lines; conservative (true when unsure: degenerate images, rect-only).
__device__ inline bool cell_overlaps(const BP& p, const Foot& f, int q, int x, int y) {
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

__device__ inline uint32_t cell_index(const BP& p, const Foot& f, int q, int x, int y) {
  if (p.kind == RT_LB_DIR) return (uint32_t)y * p.nx + (uint32_t)x;
  return f.face[q] * p.n * p.n + (uint32_t)y * p.n + (uint32_t)x;
}

__global__ __launch_bounds__(256) void count_kernel(BP p) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  Foot f;
  footprint(p, prim, f);
  uint64_t c = 0;
  if (f.global) {
    p.global[atomicAdd(p.ctr + 1, 1u)] = prim;
  } else {
    c = foot_cells(p, f);
    if (c > kSmallCells) {
      p.big[atomicAdd(p.ctr, 1u)] = prim;  // emitted rect-wise by a workgroup
    } else {
      c = 0;  // small: only the cells the grown image overlaps
      for (int q = 0; q < f.n; q++)
        for (int y = f.y0[q]; y <= f.y1[q]; y++)
          for (int x = f.x0[q]; x <= f.x1[q]; x++) c += cell_overlaps(p, f, q, x, y) ? 1u : 0u;
    }
  }
  p.count[prim] = (uint32_t)c;  // the host checks the total against 2^32
}

__device__ inline void emit_cell(const BP& p, const Foot& f, uint32_t prim, uint64_t i, uint64_t at) {
  int q = 0;
  for (;; q++) {
    const uint64_t rc = (uint64_t)(f.x1[q] - f.x0[q] + 1) * (uint64_t)(f.y1[q] - f.y0[q] + 1);
    if (i < rc) break;
    i -= rc;
  }
  const uint32_t wq = (uint32_t)(f.x1[q] - f.x0[q] + 1);
  const int x = f.x0[q] + (int)(i % wq), y = f.y0[q] + (int)(i / wq);
  const uint32_t cell = cell_index(p, f, q, x, y);
  p.keys[at] = ((unsigned long long)cell << 32) | orderable(cell_key(p, f, x, y));
  p.vals[at] = prim;
}

__global__ __launch_bounds__(256) void emit_kernel(BP p) {
  const uint32_t prim = blockIdx.x * blockDim.x + threadIdx.x;
  if (prim >= p.nprim) return;
  const uint32_t c = p.count[prim];
  if (c == 0) return;
  Foot f;
  footprint(p, prim, f);
  if (foot_cells(p, f) > kSmallCells) return;  // big: emit_big_kernel
  uint64_t at = p.off[prim];
  for (int q = 0; q < f.n; q++)
    for (int y = f.y0[q]; y <= f.y1[q]; y++)
      for (int x = f.x0[q]; x <= f.x1[q]; x++)
        if (cell_overlaps(p, f, q, x, y)) {
          p.keys[at] = ((unsigned long long)cell_index(p, f, q, x, y) << 32) | orderable(cell_key(p, f, x, y));
          p.vals[at] = prim;
          at++;
        }
}

// one workgroup per big footprint (ground planes, triangles near a point light)
__global__ __launch_bounds__(256) void emit_big_kernel(BP p) {
  for (uint32_t b = blockIdx.x; b < p.ctr[0]; b += gridDim.x) {
    const uint32_t prim = p.big[b];
    Foot f;
    footprint(p, prim, f);
    const uint32_t c = p.count[prim];
    const uint64_t o = p.off[prim];
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) emit_cell(p, f, prim, i, o + i);
  }
}

// sorted (cell, key) pairs -> per-entry keys
__global__ __launch_bounds__(256) void key_kernel(const unsigned long long* keys, uint32_t n, float* key) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key[i] = unorder((uint32_t)keys[i]);
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
  uint32_t* global = nullptr;
  unsigned long long entries = 0, cells = 0, nglobal = 0;
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
  (void)hipFree(d->global);
  delete d;
}

extern "C" void rt_lightbuf_sizes(const LBDevice* d, unsigned long long* entries, unsigned long long* cells,
                                  unsigned long long* global) {
  *entries = d ? d->entries : 0;
  *cells = d ? d->cells : 0;
  *global = d ? d->nglobal : 0;
}

#define LB_TRY(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      snprintf(err, errlen, "%s: %s", #x, hipGetErrorString(e_));                     \
      rc = -1;                                                                        \
      goto done;                                                                      \
    }                                                                                 \
  } while (0)

extern "C" int rt_lightbuf_build(const LBParams* in, RtLightBuf* out, LBDevice** devp, hipStream_t s,
                                 char* err, size_t errlen) {
  using namespace rtl;
  int rc = 0;
  BP p;
  std::memset(&p, 0, sizeof p);
  std::memset(out, 0, sizeof *out);
  LBDevice* dev = new LBDevice();
  uint32_t* count = nullptr;
  uint32_t* off = nullptr;
  uint32_t* ctr = nullptr;
  uint32_t* big = nullptr;
  unsigned long long *k0 = nullptr, *k1 = nullptr;
  uint32_t* v0 = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  uint32_t hc[2] = {0, 0}, last_off = 0, last_cnt = 0;
  uint64_t total = 0, ncell = 0;
  const uint32_t np = in->nprim;
  p.tri = in->tri;
  p.nprim = np;
  p.kind = in->kind;
  for (int a = 0; a < 3; a++) p.lv[a] = in->lv[a];
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
      delete dev;
      return -1;
    }
    for (int a = 0; a < 3; a++) w[a] /= wl;
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
  if (ncell >= (1ull << 31)) {
    snprintf(err, errlen, "light buffer of %llu cells", (unsigned long long)ncell);
    delete dev;
    return -1;
  }
  LB_TRY(hipMalloc((void**)&count, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&off, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&ctr, 2 * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&big, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->global, ((size_t)np + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->start, (ncell + 1) * sizeof(uint32_t)));
  LB_TRY(hipMemsetAsync(ctr, 0, 2 * sizeof(uint32_t), s));
  LB_TRY(hipMemsetAsync(count + np, 0, sizeof(uint32_t), s));
  p.count = count;
  p.off = off;
  p.ctr = ctr;
  p.big = big;
  p.global = dev->global;
  if (np) hipLaunchKernelGGL(count_kernel, dim3((np + 255) / 256), dim3(256), 0, s, p);
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
  if (total >= (1ull << 31)) {
    snprintf(err, errlen, "light buffer of %llu entries", (unsigned long long)total);
    rc = -1;
    goto done;
  }
  dev->entries = total;
  dev->cells = ncell;
  dev->nglobal = hc[1];
  LB_TRY(hipMalloc((void**)&dev->prim, (total + 1) * sizeof(uint32_t)));
  LB_TRY(hipMalloc((void**)&dev->key, (total + 1) * sizeof(float)));
  if (total) {
    LB_TRY(hipMalloc((void**)&k0, total * sizeof(unsigned long long)));
    LB_TRY(hipMalloc((void**)&k1, total * sizeof(unsigned long long)));
    LB_TRY(hipMalloc((void**)&v0, total * sizeof(uint32_t)));
    p.keys = k0;
    p.vals = v0;
    hipLaunchKernelGGL(emit_kernel, dim3((np + 255) / 256), dim3(256), 0, s, p);
    LB_TRY(hipGetLastError());
    if (hc[0]) {
      hipLaunchKernelGGL(emit_big_kernel, dim3(hc[0] < 4096 ? hc[0] : 4096), dim3(256), 0, s, p);
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
    hipLaunchKernelGGL(key_kernel, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, k1,
                       (uint32_t)total, dev->key);
    LB_TRY(hipGetLastError());
    hipLaunchKernelGGL(start_kernel, dim3((uint32_t)((ncell + 256) / 256)), dim3(256), 0, s, k1,
                       (uint32_t)total, (uint32_t)ncell, dev->start);
    LB_TRY(hipGetLastError());
  } else {
    LB_TRY(hipMemsetAsync(dev->start, 0, (ncell + 1) * sizeof(uint32_t), s));
  }
  LB_TRY(hipStreamSynchronize(s));
  out->start = dev->start;
  out->prim = dev->prim;
  out->key = dev->key;
  out->global = dev->global;
  out->nglobal = hc[1];
done:
  (void)hipFree(count);
  (void)hipFree(off);
  (void)hipFree(ctr);
  (void)hipFree(big);
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
