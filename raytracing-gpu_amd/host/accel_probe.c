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

#include "rt_internal.h"

typedef struct { float dist; uint32_t prim; } winner;

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
  }
}

static float box_enter(rt_vec3 o, rt_vec3 inv, float eps, const float *nd)
{
  float tx0 = (nd[0] - eps - o.x) * inv.x, tx1 = (nd[4] + eps - o.x) * inv.x;
  float ty0 = (nd[1] - eps - o.y) * inv.y, ty1 = (nd[5] + eps - o.y) * inv.y;
  float tz0 = (nd[2] - eps - o.z) * inv.z, tz1 = (nd[6] + eps - o.z) * inv.z;
  float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
  float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  float slack = 1e-5f * fminf(fmaxf(fabsf(tmin), fabsf(tmax)), 1e30f);  // finite even for +-inf slabs
  if (tmax + slack < fmaxf(tmin, 0.0f) - slack)
    return INFINITY;
  return tmin;
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
  const float eps_rel = (er ? (float)atof(er) : 256.0f) * 5.9604645e-8f, eps_abs = 1e-6f;
  int W = fr.width, H = fr.height;
  uint32_t *stk = malloc(4096 * sizeof(uint32_t));
  float *stt = malloc(4096 * sizeof(float));
  if (!stk || !stt)
    rc = rt_set_error(RT_ENOMEM, "probe");
  for (long p = 0; !rc && p < (long)W * H; p += sample_stride)
  {
    int row = (int)(p / W), col = (int)(p % W);
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
        winner wb = { INFINITY, 0xffffffffu };
        for (size_t r = 0; r < flat.nrec; r++)
          consider(o, d, nd, dlen, flat.tri + RT_TRI_FLOATS * r, &wb);
        winner w = { INFINITY, 0xffffffffu };
        unsigned long long tests_before = res->tri_tests;
        if (f.nnode == 0)
        {
          for (size_t r = 0; r < f.nrec; r++)
            consider(o, d, nd, dlen, f.tri + RT_TRI_FLOATS * r, &w);
          res->tri_tests += f.nrec;
        }
        else
        {
          rt_vec3 inv = { 1.0f / d.x, 1.0f / d.y, 1.0f / d.z };
          float m = fmaxf(fabsf(o.x - sc[0]), fmaxf(fabsf(o.y - sc[1]), fabsf(o.z - sc[2])));
          float eps = eps_rel * (m + sr) + eps_abs;
          int sp = 0;
          float t0 = box_enter(o, inv, eps, f.node);
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
            if (w.dist != INFINITY && tn * dlen > w.dist + w.dist * 1e-5f + 2.0f * eps)
              continue;
            const float *nd_ = f.node + RT_NODE_FLOATS * ni;
            uint32_t first, cnt;
            memcpy(&first, &nd_[3], 4);
            memcpy(&cnt, &nd_[7], 4);
            res->node_visits++;
            if (cnt & RT_LEAF_FLAG)
            {
              cnt &= ~RT_LEAF_FLAG;
              for (uint32_t q = 0; q < cnt; q++)
                consider(o, d, nd, dlen, f.tri + RT_TRI_FLOATS * (size_t)(first + q), &w);
              res->tri_tests += cnt;
            }
            else
            {
              uint32_t ci[8];
              float ct[8];
              int nh = 0;
              for (uint32_t c = 0; c < cnt; c++)
              {
                float tc = box_enter(o, inv, eps, f.node + RT_NODE_FLOATS * (size_t)(first + c));
                if (tc == INFINITY)
                  continue;
                if (w.dist != INFINITY && tc * dlen > w.dist + w.dist * 1e-5f + 2.0f * eps)
                  continue;
                int q = nh++;
                while (q > 0 && ct[q - 1] < tc)
                {
                  ct[q] = ct[q - 1];
                  ci[q] = ci[q - 1];
                  --q;
                }
                ct[q] = tc;
                ci[q] = first + c;
              }
              for (int q = 0; q < nh && sp < 4096; q++)
              {
                stk[sp] = ci[q];
                stt[sp] = ct[q];
                sp++;
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
          res->mismatches++;
        if (w.prim != 0xffffffffu)
          res->hits++;
      }
  }
  free(stk);
  free(stt);
  rt_flat_free(&f);
  rt_flat_free(&flat);
  return rc;
}
