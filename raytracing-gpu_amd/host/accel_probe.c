/*
 * accel_probe.c -- host-side model of the device octree traversal.
 *
 * Used (1) to tune the octree build without a GPU: average node visits and
 * triangle tests per camera-ray closest-hit query on a pixel sample, and (2) to
 * cross-check conservative culling: every sampled query's winner (new_dist,
 * prim) is compared with the brute-force winner over all triangles (the
 * reference's collide(), cpu/hit.c:72-91).  The traversal mirrors
 * csrc/rt_render.hip oct_closest(): same slab test with the same per-ray
 * slack, same front-to-back order, same pruning rule.  Not on the render path.
 */
#define _GNU_SOURCE
#include <float.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rt_cull.h"
#include "rt_internal.h"

typedef struct { float dist; uint32_t prim; rt_vec3 pt; } winner;

/* the device walk's box test and prune rule (csrc/rt_render.hip box_enter,
 * rt_prune), on the shared rt_cull.h arithmetic */
static float probe_box_enter(rt_vec3 o, rt_vec3 inv, float eps, float lx, float ly, float lz,
                             float hx, float hy, float hz)
{
  float t;
  int hit = rt_box_hit(o.x + eps, o.y + eps, o.z + eps, o.x - eps, o.y - eps, o.z - eps, inv.x,
                       inv.y, inv.z, lx, ly, lz, hx, hy, hz, &t);
  return hit ? t : INFINITY;
}

static int rt_prune(float t_enter, float dlen, float best, float eps)
{
  return t_enter * dlen > rt_prune_limit(best, eps);
}

static int mt_exact(rt_vec3 o, rt_vec3 d, const float *r, float *t, float *u, float *v)
{
  const float eps = 0.0000001f;
  rt_vec3 v0 = { r[0], r[1], r[2] }, e1 = { r[3], r[4], r[5] }, e2 = { r[6], r[7], r[8] };
  rt_vec3 h = rt_v_cross(d, e2);
  float a = e1.x * h.x + e1.y * h.y + e1.z * h.z;
  if (a > -eps && a < eps)
    return 0;
  float f = 1 / a;
  rt_vec3 s = rt_v_sub(o, v0);
  *u = f * (s.x * h.x + s.y * h.y + s.z * h.z);
  if (*u < 0.0 || *u > 1.0)
    return 0;
  rt_vec3 q = rt_v_cross(s, e1);
  *v = f * (d.x * q.x + d.y * q.y + d.z * q.z);
  if (*v < 0.0 || *u + *v > 1.0)
    return 0;
  *t = f * (e2.x * q.x + e2.y * q.y + e2.z * q.z);
  return *t > eps;
}

static void consider(rt_vec3 o, rt_vec3 d, rt_vec3 nd, float dlen, const float *r, winner *w)
{
  float t, u, v;
  if (!mt_exact(o, d, r, &t, &u, &v))
    return;
  rt_vec3 out = rt_v_add(o, rt_v_scale(nd, t * dlen));
  float nd_ = rt_v_length(rt_v_sub(out, o));
  if (!(nd_ > 0.01))
    return;
  uint32_t prim;
  memcpy(&prim, &r[9], 4);
  if (nd_ < w->dist || (nd_ == w->dist && prim < w->prim))
  {
    w->dist = nd_;
    w->prim = prim;
    w->pt = out;
  }
}

/* any-hit walk of a shadow ray (mirrors oct_any in csrc/rt_render.hip) */
static int probe_any(const rt_flat_scene *f, rt_vec3 o, rt_vec3 d, float eps, uint32_t *stk,
                     unsigned long long *nodes, unsigned long long *tris)
{
  float dlen = rt_v_length(d);
  rt_vec3 nd = { d.x / dlen, d.y / dlen, d.z / dlen };
  rt_vec3 inv = { rt_inv(d.x), rt_inv(d.y), rt_inv(d.z) };
  uint32_t dm = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
  const float *rn = f->node;
  int sp = 0;
  if (probe_box_enter(o, inv, eps,rn[0], rn[1], rn[2], rn[4], rn[5],
                   rn[6]) != INFINITY)
    stk[sp++] = 0;
  while (sp > 0)
  {
    const float *nd_ = f->node + RT_NODE_FLOATS * stk[--sp];
    uint32_t first, info;
    memcpy(&first, &nd_[3], 4);
    memcpy(&info, &nd_[7], 4);
    (*nodes)++;
    if (info & RT_NODE_LEAF)
    {
      for (uint32_t q = 0; q < RT_LEAF_COUNT(info); q++)
      {
        winner w = { INFINITY, 0xffffffffu, { 0, 0, 0 } };
        (*tris)++;
        consider(o, d, nd, dlen, f->tri + RT_TRI_FLOATS * (size_t)(first + q), &w);
        if (w.prim != 0xffffffffu)
          return 1;
      }
      continue;
    }
    uint32_t mask = RT_NODE_MASK(info);
    for (int j = 7; j >= 0; --j)
    {
      uint32_t oc = (uint32_t)j ^ dm;
      if (!(mask & (1u << oc)))
        continue;
      uint32_t ci = first + (uint32_t)__builtin_popcount(mask & ((1u << oc) - 1u));
      const float *cn = f->node + RT_NODE_FLOATS * (size_t)ci;
      if (probe_box_enter(o, inv, eps,cn[0], cn[1], cn[2], cn[4], cn[5],
                       cn[6]) != INFINITY && sp < 4096)
        stk[sp++] = ci;
    }
  }
  return 0;
}

/* ---- mismatch diagnostics (RT_PROBE_TRACE) ---- */

/* does the line o + t d (t >= 0) hit box [lo - e, hi + e]?  (double) */
static int dbox_hit(const double o[3], const double d[3], const float *nd, double e)
{
  double t0 = 0, t1 = INFINITY;
  for (int a = 0; a < 3; a++)
  {
    double lo = nd[a] - e, hi = nd[4 + a] + e;
    if (d[a] == 0)
    {
      if (o[a] < lo || o[a] > hi)
        return 0;
      continue;
    }
    double ta = (lo - o[a]) / d[a], tb = (hi - o[a]) / d[a];
    if (ta > tb)
    {
      double x = ta;
      ta = tb;
      tb = x;
    }
    if (ta > t0) t0 = ta;
    if (tb < t1) t1 = tb;
  }
  return t0 <= t1;
}

/* smallest growth e (bisection) for which the ray hits the node box */
static double needed_eps(const double o[3], const double d[3], const float *nd)
{
  if (dbox_hit(o, d, nd, 0))
    return 0;
  double lo = 0, hi = 1e-6;
  while (!dbox_hit(o, d, nd, hi) && hi < 1e6)
    hi *= 2;
  for (int k = 0; k < 60; k++)
  {
    double m = 0.5 * (lo + hi);
    if (dbox_hit(o, d, nd, m))
      hi = m;
    else
      lo = m;
  }
  return hi;
}

static void trace_mismatch(const rt_flat_scene *f, const rt_flat_scene *flat, rt_vec3 o, rt_vec3 d,
                           float eps, winner wb, winner w, int row, int col)
{
  const float *r = flat->tri + RT_TRI_FLOATS * (size_t)wb.prim;
  double od[3] = { o.x, o.y, o.z }, dd[3] = { d.x, d.y, d.z };
  double v0[3] = { r[0], r[1], r[2] }, e1[3] = { r[3], r[4], r[5] }, e2[3] = { r[6], r[7], r[8] };
  double h[3] = { dd[1] * e2[2] - dd[2] * e2[1], dd[2] * e2[0] - dd[0] * e2[2],
                  dd[0] * e2[1] - dd[1] * e2[0] };
  double a = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
  double sv[3] = { od[0] - v0[0], od[1] - v0[1], od[2] - v0[2] };
  double u = (sv[0] * h[0] + sv[1] * h[1] + sv[2] * h[2]) / a;
  double q[3] = { sv[1] * e1[2] - sv[2] * e1[1], sv[2] * e1[0] - sv[0] * e1[2],
                  sv[0] * e1[1] - sv[1] * e1[0] };
  double v = (dd[0] * q[0] + dd[1] * q[1] + dd[2] * q[2]) / a;
  double n[3] = { e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                  e1[0] * e2[1] - e1[1] * e2[0] };
  double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  double dl = sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
  double cosn = fabs(dd[0] * n[0] + dd[1] * n[1] + dd[2] * n[2]) / (nl * dl);
  double l1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
  double l2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
  fprintf(stderr,
          "probe mismatch px (%d,%d): brute prim %u dist %.9g, octree prim %u dist %.9g; eps %.3g\n"
          "  winner exact-double u %.3g v %.3g 1-u-v %.3g  cos(ray,normal) %.3g |e1| %.3g |e2| %.3g\n",
          row, col, wb.prim, wb.dist, w.prim, w.dist, eps, u, v, 1 - u - v, cosn, l1, l2);
  /* every leaf holding the winner: how much growth would its box need? */
  for (size_t ni = 0; ni < f->nnode; ni++)
  {
    const float *nd = f->node + RT_NODE_FLOATS * ni;
    uint32_t first, info;
    memcpy(&first, &nd[3], 4);
    memcpy(&info, &nd[7], 4);
    if (!(info & RT_NODE_LEAF))
      continue;
    for (uint32_t k = 0; k < RT_LEAF_COUNT(info); k++)
    {
      uint32_t prim;
      memcpy(&prim, &f->tri[RT_TRI_FLOATS * (size_t)(first + k) + 9], 4);
      if (prim == wb.prim)
        fprintf(stderr, "  leaf %zu box [%g %g %g]-[%g %g %g] needs eps %.3g\n", ni, nd[0], nd[1],
                nd[2], nd[4], nd[5], nd[6], needed_eps(od, dd, nd));
    }
  }
}

/* Probe statistics (host-only diagnostic; see rt_hip.h). */
int rt_accel_probe(const rt_scene *s, int accel, int sample_stride, int check,
                   rt_accel_probe_result *res)
{
  if (!s || !res || sample_stride < 1)
    return rt_set_error(RT_EINVAL, "bad argument");
  memset(res, 0, sizeof *res);
  rt_flat_scene f;
  int rc = rt_flatten(s, accel, &f);
  if (rc)
    return rc;
  rt_flat_scene flat;
  memset(&flat, 0, sizeof flat);
  rc = check ? rt_flatten(s, RT_ACCEL_FLAT, &flat) : RT_OK;
  if (rc)
  {
    rt_flat_free(&f);
    return rc;
  }
  rt_frame fr;
  rc = rt_frame_from_camera(&s->camera, &fr);
  float sc[3], sr = 0;
  for (int a = 0; a < 3; a++)
  {
    sc[a] = 0.5f * (f.scene_lo[a] + f.scene_hi[a]);
    sr = fmaxf(sr, 0.5f * (f.scene_hi[a] - f.scene_lo[a]));
  }
  const char *er = getenv("RT_PROBE_EPS_ULPS");
  const float eps_rel = (er ? (float)atof(er) : 64.0f) * 5.9604645e-8f;
  float cmag = fmaxf(fabsf(sc[0]), fmaxf(fabsf(sc[1]), fabsf(sc[2])));
  int W = fr.width, H = fr.height;
  uint32_t *stk = malloc(4096 * sizeof(uint32_t));
  float *stt = malloc(4096 * sizeof(float));
  if (!stk || !stt)
    rc = rt_set_error(RT_ENOMEM, "probe");
  /* RT_PROBE_PIXELS="r,c;r,c;..." probes exactly those pixels */
  const char *plist = getenv("RT_PROBE_PIXELS");
  for (long p = 0; !rc && (plist ? *plist != 0 : p < (long)W * H); p += sample_stride)
  {
    int row = (int)(p / W), col = (int)(p % W);
    if (plist)
    {
      char *end;
      row = (int)strtol(plist, &end, 10);
      col = (int)strtol(end + 1, &end, 10);
      plist = *end ? end + 1 : end;
      if (row < 0 || row >= H || col < 0 || col >= W)
        continue;
    }
    int i = (W - col) - W / 2, j = (H - row) - H / 2;
    if (W - col < 1 || W - col > 2 * (W / 2) || H - row < 1 || H - row > 2 * (H / 2))
      continue;
    for (int sk = 0; sk < 2; sk++)
      for (int sl = 0; sl < 2; sl++)
      {
        float k = (float)i + 0.5f * (float)sk, l = (float)j + 0.5f * (float)sl;
        rt_vec3 o = rt_v_add(rt_v_add(fr.C, rt_v_scale(fr.u, k)), rt_v_scale(fr.v, l));
        rt_vec3 d = rt_v_normalize(rt_v_sub(fr.position, o));
        float dlen = rt_v_length(d);
        rt_vec3 nd = { d.x / dlen, d.y / dlen, d.z / dlen };
        res->queries++;
        /* brute force winner */
        winner wb = { INFINITY, 0xffffffffu, { 0, 0, 0 } };
        for (size_t r = 0; r < flat.nrec; r++)
          consider(o, d, nd, dlen, flat.tri + RT_TRI_FLOATS * r, &wb);
        winner w = { INFINITY, 0xffffffffu, { 0, 0, 0 } };
        unsigned long long tests_before = res->tri_tests;
        if (f.nnode == 0)
        {
          for (size_t r = 0; r < f.nrec; r++)
            consider(o, d, nd, dlen, f.tri + RT_TRI_FLOATS * r, &w);
          res->tri_tests += f.nrec;
        }
        else
        {
          rt_vec3 inv = { rt_inv(d.x), rt_inv(d.y), rt_inv(d.z) };
          uint32_t dm = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
          float eps = rt_cull_eps(eps_rel, o.x - sc[0], o.y - sc[1], o.z - sc[2], cmag, sr);
          int sp = 0;
          const float *rn = f.node;
          float t0 = probe_box_enter(o, inv, eps,rn[0], rn[1], rn[2],
                                  rn[4], rn[5], rn[6]);
          if (t0 != INFINITY)
          {
            stk[0] = 0;
            stt[0] = t0;
            sp = 1;
          }
          while (sp > 0)
          {
            --sp;
            uint32_t ni = stk[sp];
            float tn = stt[sp];
            if (w.dist != INFINITY && rt_prune(tn, dlen, w.dist, eps))
              continue;
            const float *nd_ = f.node + RT_NODE_FLOATS * ni;
            uint32_t first, info;
            memcpy(&first, &nd_[3], 4);
            memcpy(&info, &nd_[7], 4);
            res->node_visits++;
            if (info & RT_NODE_LEAF)
            {
              uint32_t cnt = RT_LEAF_COUNT(info);
              for (uint32_t q = 0; q < cnt; q++)
                consider(o, d, nd, dlen, f.tri + RT_TRI_FLOATS * (size_t)(first + q), &w);
              res->tri_tests += cnt;
            }
            else
            {
              /* same far-to-near octant push order as csrc/rt_render.hip */
              uint32_t mask = RT_NODE_MASK(info);
              for (int j = 7; j >= 0; --j)
              {
                uint32_t oc = (uint32_t)j ^ dm;
                if (!(mask & (1u << oc)))
                  continue;
                uint32_t ci = first + (uint32_t)__builtin_popcount(mask & ((1u << oc) - 1u));
                const float *cn = f.node + RT_NODE_FLOATS * (size_t)ci;
                float tc = probe_box_enter(o, inv, eps,cn[0], cn[1],
                                        cn[2], cn[4], cn[5], cn[6]);
                if (tc == INFINITY)
                  continue;
                if (w.dist != INFINITY && rt_prune(tc, dlen, w.dist, eps))
                  continue;
                if (sp < 4096)
                {
                  stk[sp] = ci;
                  stt[sp] = tc;
                  sp++;
                }
              }
              if (sp > (int)res->max_stack)
                res->max_stack = (unsigned long long)sp;
            }
          }
        }
        if (getenv("RT_PROBE_TRACE") && res->tri_tests - tests_before > 5000)
          fprintf(stderr, "probe: pixel (%d,%d) sample %d%d: %llu tri tests, hit %u d=(%g,%g,%g)\n", row,
                  col, sk, sl, res->tri_tests - tests_before, w.prim, d.x, d.y, d.z);
        if (check && (w.prim != wb.prim || (w.dist != wb.dist && !(isnan(w.dist) && isnan(wb.dist)))))
        {
          res->mismatches++;
          if (getenv("RT_PROBE_TRACE"))
            trace_mismatch(&f, &flat, o, d,
                           rt_cull_eps(eps_rel, o.x - sc[0], o.y - sc[1], o.z - sc[2], cmag, sr),
                           wb, w, row, col);
        }
        if (w.prim != 0xffffffffu)
        {
          res->hits++;
          /* shadow rays of the hit, as apply_light (cpu/light.c:51-90) casts them */
          for (size_t li = 0; f.nnode && li < f.nlight; li++)
          {
            const float *L = f.light + RT_LIGHT_FLOATS * li;
            uint32_t type;
            memcpy(&type, &L[0], 4);
            rt_vec3 lv = { L[4], L[5], L[6] }, sd;
            if (type == 1)
              sd = rt_v_scale(lv, -1.0f);
            else if (type == 2)
              sd = rt_v_sub(lv, w.pt);
            else
              continue;
            float seps = rt_cull_eps(eps_rel, w.pt.x - sc[0], w.pt.y - sc[1], w.pt.z - sc[2], cmag, sr);
            res->shadow_queries++;
            res->shadow_hits += (unsigned long long)probe_any(&f, w.pt, sd, seps, stk,
                                                              &res->shadow_node_visits,
                                                              &res->shadow_tri_tests);
          }
        }
      }
  }
  free(stk);
  free(stt);
  rt_flat_free(&f);
  rt_flat_free(&flat);
  return rc;
}
