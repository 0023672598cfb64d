/*
 * diag.c -- TEST/DIAGNOSTIC INFRASTRUCTURE ONLY (never linked by the product).
 *
 * Per-pixel query trace of the oracle: replays one pixel of cpu/rt
 * (/root/reference/cpu/raytracer.c:54-71, trace :19-34, apply_light
 * cpu/light.c:33-100) with brute-force collide/collide_dist exactly as
 * rt_oracle.c does, and records every query with the triangle that decided
 * it and that triangle's conditioning:
 *
 *   closest query  deciding triangle = the winner (cpu/hit.c:72-91)
 *   shadow query   deciding triangle = among every accepting triangle
 *                  (cpu/hit.c:93-109), the one the exact ray comes closest to
 *
 * "need" = the growth of that triangle's axis-aligned box that the exact
 * (double) ray o + t d, t >= 0, needs to touch it: 0 for a geometric hit, and
 * > 0 for the reference's float "garbage" accepts of grazing rays (DESIGN.md
 * §2).  Octree culling with slack eps can only lose a decision whose need
 * exceeds eps.  Built as a unity build over rt_oracle.c (_build/liboracle_diag.so).
 */
#include "rt_oracle.c"

struct or_diag_query {
  int kind;   /* 0 camera closest, 1 reflection closest, 2 directional shadow, 3 point shadow */
  int depth;  /* bounce depth of the path (camera = 0) */
  int sample; /* 0..3 in cpu order */
  int result; /* closest: 1 hit; shadow: 1 shadowed */
  float o[3], d[3];
  int obj, tri;   /* deciding triangle (-1 if none) */
  float dist;     /* new_dist of the deciding triangle */
  int naccept;    /* triangles accepted (new_dist > 0.01) */
  double u, v;    /* exact-double barycentrics of the deciding triangle */
  double cosn;    /* |d . n| / (|d| |n|) */
  double need;    /* box growth the exact ray needs to touch it (0 = real hit) */
  double S;       /* |o - v0| */
  double inplane; /* distance of the exact plane crossing v0 + u e1 + v e2 from the triangle */
  double shape;   /* (|e1| + |e2|)^2 / |e1 x e2| */
  double kbary;   /* smallest k with u >= -k au, v >= -k av, u + v <= 1 + k (au + av),
                     au = eps_f |o - v0| |e2| / (|e1 x e2| cos), av likewise with |e1| */
};

struct diag_ctx {
  struct or_diag_query *q;
  int n, max;
  int sample;
};

static int dbox(const double o[3], const double d[3], const double lo[3], const double hi[3], double e)
{
  double t0 = 0, t1 = INFINITY;
  for (int a = 0; a < 3; a++)
  {
    double l = lo[a] - e, h = hi[a] + e;
    if (d[a] == 0)
    {
      if (o[a] < l || o[a] > h)
        return 0;
      continue;
    }
    double ta = (l - o[a]) / d[a], tb = (h - o[a]) / d[a];
    if (ta > tb)
    {
      double x = ta;
      ta = tb;
      tb = x;
    }
    if (ta > t0)
      t0 = ta;
    if (tb < t1)
      t1 = tb;
  }
  return t0 <= t1;
}

static double need_growth(ray r, const struct or_triangle *t)
{
  double o[3] = { r.origin.x, r.origin.y, r.origin.z }, d[3] = { r.direction.x, r.direction.y, r.direction.z };
  double lo[3], hi[3];
  const float *v = &t->vertex[0].x;
  for (int a = 0; a < 3; a++)
  {
    lo[a] = fmin(v[a], fmin(v[3 + a], v[6 + a]));
    hi[a] = fmax(v[a], fmax(v[3 + a], v[6 + a]));
  }
  if (dbox(o, d, lo, hi, 0))
    return 0;
  double a = 0, b = 1e-9;
  while (!dbox(o, d, lo, hi, b) && b < 1e9)
    b *= 2;
  for (int k = 0; k < 80; k++)
  {
    double m = 0.5 * (a + b);
    if (dbox(o, d, lo, hi, m))
      b = m;
    else
      a = m;
  }
  return b;
}

static void conditioning(ray r, const struct or_triangle *t, struct or_diag_query *q)
{
  double d[3] = { r.direction.x, r.direction.y, r.direction.z };
  const float *vx = &t->vertex[0].x;
  double v0[3] = { vx[0], vx[1], vx[2] };
  double e1[3], e2[3], s[3];
  for (int a = 0; a < 3; a++)
  {
    e1[a] = (double)vx[3 + a] - v0[a];
    e2[a] = (double)vx[6 + a] - v0[a];
  }
  s[0] = r.origin.x - v0[0];
  s[1] = r.origin.y - v0[1];
  s[2] = r.origin.z - v0[2];
  double h[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
  double a = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
  double qv[3] = { s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0] };
  q->u = (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]) / a;
  q->v = (d[0] * qv[0] + d[1] * qv[1] + d[2] * qv[2]) / a;
  double n[3] = { e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0] };
  double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  double dl = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  q->cosn = fabs(d[0] * n[0] + d[1] * n[1] + d[2] * n[2]) / (nl * dl);
  q->S = sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
  q->need = need_growth(r, t);
  double l1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
  double l2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
  q->shape = (l1 + l2) * (l1 + l2) / nl;
  {
    double ef = 5.9604644775390625e-8 * q->S / (nl * q->cosn);
    double au = ef * l2, av = ef * l1, k = 0;
    if (-q->u / au > k) k = -q->u / au;
    if (-q->v / av > k) k = -q->v / av;
    if ((q->u + q->v - 1) / (au + av) > k) k = (q->u + q->v - 1) / (au + av);
    q->kbary = k;
  }
  /* closest point of the triangle to X, over the triangle's barycentric
   * domain (u, v >= 0, u + v <= 1): a small convex QP, solved by checking the
   * interior and the three edges */
  double X[3], best = INFINITY;
  for (int k = 0; k < 3; k++)
    X[k] = v0[k] + q->u * e1[k] + q->v * e2[k];
  if (q->u >= 0 && q->v >= 0 && q->u + q->v <= 1)
    best = 0;
  const double P[3][3] = { { v0[0], v0[1], v0[2] },
                           { v0[0] + e1[0], v0[1] + e1[1], v0[2] + e1[2] },
                           { v0[0] + e2[0], v0[1] + e2[1], v0[2] + e2[2] } };
  for (int ed = 0; ed < 3 && best > 0; ed++)
  {
    const double *A0 = P[ed], *B0 = P[(ed + 1) % 3];
    double ab[3] = { B0[0] - A0[0], B0[1] - A0[1], B0[2] - A0[2] };
    double ax[3] = { X[0] - A0[0], X[1] - A0[1], X[2] - A0[2] };
    double tt = (ab[0] * ax[0] + ab[1] * ax[1] + ab[2] * ax[2]) / (ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2]);
    tt = tt < 0 ? 0 : (tt > 1 ? 1 : tt);
    double dd = 0;
    for (int k = 0; k < 3; k++)
    {
      double z = ax[k] - tt * ab[k];
      dd += z * z;
    }
    if (sqrt(dd) < best)
      best = sqrt(dd);
  }
  q->inplane = best;
}

static struct or_diag_query *diag_new(struct diag_ctx *c, int kind, int depth, ray r)
{
  static struct or_diag_query sink;
  struct or_diag_query *q = c->n < c->max ? &c->q[c->n] : &sink;
  c->n++;
  memset(q, 0, sizeof *q);
  q->kind = kind;
  q->depth = depth;
  q->sample = c->sample;
  q->o[0] = r.origin.x;
  q->o[1] = r.origin.y;
  q->o[2] = r.origin.z;
  q->d[0] = r.direction.x;
  q->d[1] = r.direction.y;
  q->d[2] = r.direction.z;
  q->obj = q->tri = -1;
  return q;
}

/* closest hit with the winner's (object, triangle): cpu/hit.c:46-91 */
static ray diag_collide(const struct or_scene *scene, ray r, int *oi, struct or_diag_query *q)
{
  float best = 0;
  ray ret = { { 0, 0, 0 }, { 0, 0, 0 } };
  for (size_t i = 0; i < scene->object_count; i++)
  {
    const struct or_object *obj = &scene->objects[i];
    float ob = 0;
    int oti = -1;
    ray cand = { { 0, 0, 0 }, { 0, 0, 0 } };
    for (size_t k = 0; k < obj->triangle_count; k++)
    {
      vec3 out, normal;
      if (!intersect(r, &obj->triangles[k], &out, &normal))
        continue;
      float d = v_length(v_sub(out, r.origin));
      if (!(d > 0.01))
        continue;
      q->naccept++;
      if (d < ob || ob == 0)
      {
        ob = d;
        oti = (int)k;
        cand.origin = out;
        cand.direction = normal;
      }
    }
    if (oti < 0 || v_is_zero(cand.direction))
      continue;
    if (ob < best || best == 0)
    {
      best = ob;
      ret = cand;
      *oi = (int)i;
      q->obj = (int)i;
      q->tri = oti;
    }
  }
  if (q->obj >= 0)
  {
    q->result = 1;
    q->dist = best;
    conditioning(r, &scene->objects[q->obj].triangles[q->tri], q);
  }
  return ret;
}

/* shadow query: every accepting triangle, the least garbage one decides */
static int diag_shadowed(const struct or_scene *scene, ray r, struct or_diag_query *q)
{
  double bestneed = INFINITY;
  for (size_t i = 0; i < scene->object_count; i++)
  {
    const struct or_object *obj = &scene->objects[i];
    for (size_t k = 0; k < obj->triangle_count; k++)
    {
      vec3 out, normal;
      if (!intersect(r, &obj->triangles[k], &out, &normal))
        continue;
      float d = v_length(v_sub(out, r.origin));
      if (!(d > 0.01))
        continue;
      q->naccept++;
      struct or_diag_query tmp;
      conditioning(r, &obj->triangles[k], &tmp);
      if (tmp.need < bestneed)
      {
        bestneed = tmp.need;
        q->obj = (int)i;
        q->tri = (int)k;
        q->dist = d;
        q->u = tmp.u;
        q->v = tmp.v;
        q->cosn = tmp.cosn;
        q->need = tmp.need;
        q->S = tmp.S;
        q->inplane = tmp.inplane;
        q->shape = tmp.shape;
        q->kbary = tmp.kbary;
      }
    }
  }
  q->result = q->naccept > 0;
  return q->result;
}

static color diag_shade(const struct or_scene *scene, const struct or_object *obj, ray hit, int depth,
                        struct diag_ctx *c)
{
  color acc = oracle_init_color(0, 0, 0);
  for (size_t i = 0; i < scene->light_count; i++)
  {
    const struct or_light *l = &scene->lights[i];
    if (l->type == OR_AMBIENT)
    {
      color t = oracle_color_mul2(oracle_init_color(l->r, l->g, l->b),
                                  oracle_init_color(obj->ka.x, obj->ka.y, obj->ka.z));
      acc = oracle_color_add(acc, t);
    }
    else if (l->type == OR_DIRECTIONAL)
    {
      ray sr = { hit.origin, v_scale(l->v, -1) };
      if (diag_shadowed(scene, sr, diag_new(c, 2, depth, sr)))
        continue;
      vec3 L = v_scale(l->v, -1);
      color t = oracle_color_mul2(oracle_init_color(l->r, l->g, l->b),
                                  oracle_init_color(obj->kd.x, obj->kd.y, obj->kd.z));
      t = oracle_color_mul(t, v_dot(L, hit.direction));
      ray inc = { v_add(hit.origin, v_scale(l->v, -10)), l->v };
      specular(&t, inc, hit, obj);
      acc = oracle_color_add(acc, t);
    }
    else if (l->type == OR_POINT)
    {
      vec3 L = v_scale(l->v, -1);
      vec3 N = hit.direction;
      if (v_dot(L, N) < 0)
        N = v_scale(N, -1);
      vec3 to_light = v_sub(l->v, hit.origin);
      float dist = v_length(v_sub(l->v, hit.origin));
      ray sr = { hit.origin, to_light };
      if (diag_shadowed(scene, sr, diag_new(c, 3, depth, sr)))
        continue;
      color t = oracle_color_mul2(oracle_init_color(l->r, l->g, l->b),
                                  oracle_init_color(obj->kd.x, obj->kd.y, obj->kd.z));
      t = oracle_color_mul(t, v_dot(L, N) * 1 / dist);
      ray inc = { v_add(hit.origin, v_scale(to_light, -10)), to_light };
      specular(&t, inc, hit, obj);
      acc = oracle_color_add(acc, t);
    }
  }
  return acc;
}

static color diag_trace(const struct or_scene *scene, ray r, float coef, int depth, struct diag_ctx *c)
{
  if (coef < 0.01)
    return oracle_init_color(0, 0, 0);
  int oi = -1;
  ray hit = diag_collide(scene, r, &oi, diag_new(c, depth ? 1 : 0, depth, r));
  if (v_is_zero(hit.direction))
    return oracle_init_color(0, 0, 0);
  const struct or_object *obj = &scene->objects[oi];
  color local = diag_shade(scene, obj, hit, depth, c);
  color refl = diag_trace(scene, bounce(r, hit), obj->nr * coef, depth + 1, c);
  return oracle_color_add(refl, oracle_color_mul(local, coef));
}

/* Returns the number of queries of the pixel (records beyond max are
 * dropped); rgb receives the pixel's colour (== oracle_render's). */
int oracle_diag_pixel(const struct or_scene *scene, int row, int col, struct or_diag_query *out,
                      int max, float rgb[3])
{
  vec3 u, v, C;
  oracle_camera_frame(scene, &u, &v, &C);
  int W = scene->camera.width, H = scene->camera.height;
  int ii = W - col, jj = H - row;
  struct diag_ctx c = { out, 0, max, 0 };
  color acc = { 0, 0, 0 };
  if (!(ii < 1 || ii > 2 * (W / 2) || jj < 1 || jj > 2 * (H / 2)))
  {
    int i = ii - W / 2, j = jj - H / 2;
    acc = oracle_init_color(0, 0, 0);
    for (float k = i; k < i + 1; k += 0.5)
      for (float l = j; l < j + 1; l += 0.5)
      {
        vec3 point = v_add(v_add(C, v_scale(u, k)), v_scale(v, l));
        ray r = { point, v_normalize(v_sub(scene->camera.position, point)) };
        color s = diag_trace(scene, r, 1, 0, &c);
        acc = oracle_color_add(acc, oracle_color_mul(s, 0.25));
        c.sample++;
      }
  }
  rgb[0] = acc.r;
  rgb[1] = acc.g;
  rgb[2] = acc.b;
  return c.n;
}
