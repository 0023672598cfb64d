/*
 * scene_obj.c -- Wavefront .obj loader / writer (host C).
 *
 * New code: the reference has no .obj reader; its
 * object blocks live inside .svati (cpu/parse_obj.c:42-92).  Mapping:
 *   - a new object starts at every `o`, `g` or `usemtl` line (once the
 *     current one holds triangles);
 *   - `f` faces (v, v/vt, v//vn, v/vt/vn, negative = relative) are fan-
 *     triangulated in corner order; triangle t of an object is its t-th
 *     fan triangle, corner k its k-th vertex (the order rt_scene_write_svati
 *     preserves through the reference's LIFO stack);
 *   - a face without vn gets its geometric normal on all corners;
 *   - materials: `mtllib` (newmtl Ka Kd Ks Ns Ni d, plus the non-standard
 *     `Nr` reflectivity), or inline `#rt Ka|Kd|Ks|Ns|Ni|Nr|d ...` comments
 *     written by rt_scene_write_obj; defaults are cpu/parse_obj.c:3-20.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"
#include "rt_par_write.h"
#include "rt_lex.h"

void rt_object_defaults(rt_object *o);
int rt_scene_push_object(rt_scene *s, const rt_object *o, size_t *cap);

typedef struct { rt_vec3 *a; size_t n, cap; } vbuf;
typedef struct { rt_triangle *a; size_t n, cap; } tbuf;

static int vpush(vbuf *b, rt_vec3 x)
{
  if (b->n == b->cap)
  {
    size_t nc = b->cap ? 2 * b->cap : 1024;
    rt_vec3 *na = realloc(b->a, nc * sizeof *na);
    if (!na)
      return rt_set_error(RT_ENOMEM, "obj vertices");
    b->a = na;
    b->cap = nc;
  }
  b->a[b->n++] = x;
  return RT_OK;
}

static int tpush(tbuf *b, const rt_triangle *t)
{
  if (b->n == b->cap)
  {
    size_t nc = b->cap ? 2 * b->cap : 256;
    rt_triangle *na = realloc(b->a, nc * sizeof *na);
    if (!na)
      return rt_set_error(RT_ENOMEM, "obj triangles");
    b->a = na;
    b->cap = nc;
  }
  b->a[b->n++] = *t;
  return RT_OK;
}

typedef struct {
  char name[128];
  rt_object mat;   /* material fields only */
} mtl_entry;

typedef struct { mtl_entry *a; size_t n; } mtl_lib;

static void line_span(rt_lex *lx, const char **s, const char **e)
{
  while (lx->p < lx->end && (*lx->p == ' ' || *lx->p == '\t'))
    lx->p++;
  *s = lx->p;
  rt_lex_skip_line(lx);
  *e = lx->p;
  while (*e > *s && rt_lex_space((*e)[-1]))
    (*e)--;
}

/* material keyword on the rest of a line; returns 1 if consumed */
static int material_key(rt_lex *lx, const char *t, size_t n, rt_object *m)
{
  rt_vec3 *vp = NULL;
  float *fp = NULL;
  if (RT_TOK_IS(t, n, "Ka")) vp = &m->ka;
  else if (RT_TOK_IS(t, n, "Kd")) vp = &m->kd;
  else if (RT_TOK_IS(t, n, "Ks")) vp = &m->ks;
  else if (RT_TOK_IS(t, n, "Ns")) fp = &m->ns;
  else if (RT_TOK_IS(t, n, "Ni")) fp = &m->ni;
  else if (RT_TOK_IS(t, n, "Nr")) fp = &m->nr;
  else if (RT_TOK_IS(t, n, "d")) fp = &m->d;
  else
    return 0;
  if (vp)
  {
    if (rt_lex_float(lx, &vp->x) || rt_lex_float(lx, &vp->y) || rt_lex_float(lx, &vp->z))
      return -1;
  }
  else if (rt_lex_float(lx, fp))
    return -1;
  return 1;
}

static int load_mtl(const char *path, mtl_lib *lib)
{
  rt_lex lx;
  int rc = rt_lex_open(path, &lx);
  if (rc)
    return rc;
  mtl_entry *cur = NULL;
  const char *t;
  size_t n;
  while (!rc && rt_lex_token(&lx, &t, &n))
  {
    if (RT_TOK_IS(t, n, "newmtl"))
    {
      const char *s, *e;
      line_span(&lx, &s, &e);
      mtl_entry *na = realloc(lib->a, (lib->n + 1) * sizeof *na);
      if (!na)
      {
        rc = rt_set_error(RT_ENOMEM, "mtl");
        break;
      }
      lib->a = na;
      cur = &lib->a[lib->n++];
      memset(cur, 0, sizeof *cur);
      size_t len = (size_t)(e - s) < sizeof cur->name - 1 ? (size_t)(e - s) : sizeof cur->name - 1;
      memcpy(cur->name, s, len);
      rt_object_defaults(&cur->mat);
      continue;
    }
    int k = cur ? material_key(&lx, t, n, &cur->mat) : 0;
    if (k < 0)
      rc = rt_set_error(RT_EPARSE, "%s: bad material value", path);
    else if (k == 0)
      rt_lex_skip_line(&lx);
  }
  rt_lex_close(&lx);
  return rc;
}

static int resolve(long idx, size_t n, size_t *out)
{
  if (idx > 0 && (size_t)idx <= n)
    *out = (size_t)idx - 1;
  else if (idx < 0 && (size_t)(-idx) <= n)
    *out = n - (size_t)(-idx);
  else
    return -1;
  return 0;
}

typedef struct {
  rt_scene *s;
  size_t obj_cap;
  tbuf tris;
  rt_object mat;
} obj_state;

static int flush_object(obj_state *st)
{
  if (st->tris.n == 0)
    return RT_OK;
  rt_object o = st->mat;
  o.triangles = realloc(st->tris.a, st->tris.n * sizeof *o.triangles);
  if (!o.triangles)
    return rt_set_error(RT_ENOMEM, "obj object");
  o.triangle_count = (unsigned)st->tris.n;
  st->tris.a = NULL;
  st->tris.n = st->tris.cap = 0;
  return rt_scene_push_object(st->s, &o, &st->obj_cap);
}

int rt_scene_append_obj(rt_scene *s, const char *path)
{
  rt_lex lx;
  int rc = rt_lex_open(path, &lx);
  if (rc)
    return rc;
  obj_state st;
  memset(&st, 0, sizeof st);
  st.s = s;
  st.obj_cap = s->object_count;
  rt_object_defaults(&st.mat);
  vbuf vs = { 0 }, vns = { 0 };
  rt_prescan ps;
  rt_prescan_build(&lx, &ps);
  mtl_lib lib = { 0 };
  const char *t;
  size_t n;
  while (!rc && rt_lex_token(&lx, &t, &n))
  {
    if (RT_TOK_IS(t, n, "v") || RT_TOK_IS(t, n, "vn"))
    {
      rt_vec3 x;
      float f[3];
      int pre = rt_prescan_take(&ps, &lx, t, f);
      if (pre)
        x.x = f[0], x.y = f[1], x.z = f[2];
      if (!pre && (rt_lex_float(&lx, &x.x) || rt_lex_float(&lx, &x.y) || rt_lex_float(&lx, &x.z)))
        rc = rt_set_error(RT_EPARSE, "%s: bad %.*s near byte %td", path, (int)n, t, lx.p - lx.buf);
      else
        rc = vpush(n == 1 ? &vs : &vns, x);
      rt_lex_skip_line(&lx); /* optional w */
    }
    else if (RT_TOK_IS(t, n, "f"))
    {
      size_t cv[64], cn[64];
      int has_n[64];
      int nc = 0;
      const char *s0, *e0;
      line_span(&lx, &s0, &e0);
      const char *p = s0;
      while (p < e0 && !rc)
      {
        while (p < e0 && (*p == ' ' || *p == '\t'))
          p++;
        if (p >= e0)
          break;
        if (nc == 64)
        {
          rc = rt_set_error(RT_EPARSE, "%s: face with more than 64 corners", path);
          break;
        }
        char *q;
        long vi = strtol(p, &q, 10), ni = 0;
        if (q == p || resolve(vi, vs.n, &cv[nc]))
        {
          rc = rt_set_error(RT_EPARSE, "%s: bad face index near byte %td", path, p - lx.buf);
          break;
        }
        p = q;
        has_n[nc] = 0;
        if (p < e0 && *p == '/')
        {
          p++;
          if (p < e0 && *p != '/')
            strtol(p, &q, 10), p = q; /* texture index: ignored */
          if (p < e0 && *p == '/')
          {
            p++;
            ni = strtol(p, &q, 10);
            if (q == p || resolve(ni, vns.n, &cn[nc]))
            {
              rc = rt_set_error(RT_EPARSE, "%s: bad normal index", path);
              break;
            }
            p = q;
            has_n[nc] = 1;
          }
        }
        nc++;
      }
      for (int k = 2; !rc && k < nc; k++)
      {
        int c[3] = { 0, k - 1, k };
        rt_triangle tri;
        for (int m = 0; m < 3; m++)
          tri.vertex[m] = vs.a[cv[c[m]]];
        if (has_n[0] && has_n[k - 1] && has_n[k])
          for (int m = 0; m < 3; m++)
            tri.normal[m] = vns.a[cn[c[m]]];
        else
        {
          rt_vec3 g = rt_v_cross(rt_v_sub(tri.vertex[1], tri.vertex[0]),
                                 rt_v_sub(tri.vertex[2], tri.vertex[0]));
          for (int m = 0; m < 3; m++)
            tri.normal[m] = g;
        }
        rc = tpush(&st.tris, &tri);
      }
    }
    else if (RT_TOK_IS(t, n, "o") || RT_TOK_IS(t, n, "g"))
    {
      rt_lex_skip_line(&lx);
      rc = flush_object(&st);
    }
    else if (RT_TOK_IS(t, n, "usemtl"))
    {
      const char *s0, *e0;
      line_span(&lx, &s0, &e0);
      rc = flush_object(&st);
      for (size_t i = 0; !rc && i < lib.n; i++)
        if (strlen(lib.a[i].name) == (size_t)(e0 - s0) && !memcmp(lib.a[i].name, s0, (size_t)(e0 - s0)))
          st.mat = lib.a[i].mat;
    }
    else if (RT_TOK_IS(t, n, "mtllib"))
    {
      const char *s0, *e0;
      line_span(&lx, &s0, &e0);
      char full[4096];
      const char *slash = strrchr(path, '/');
      size_t dl = slash ? (size_t)(slash - path + 1) : 0;
      size_t nl = (size_t)(e0 - s0);
      if (dl + nl + 1 > sizeof full)
        rc = rt_set_error(RT_EPARSE, "%s: mtllib path too long", path);
      else
      {
        memcpy(full, path, dl);
        memcpy(full + dl, s0, nl);
        full[dl + nl] = 0;
        rc = load_mtl(full, &lib);
      }
    }
    else if (RT_TOK_IS(t, n, "#rt"))
    {
      const char *k;
      size_t kn;
      if (rt_lex_token(&lx, &k, &kn))
      {
        if (st.tris.n)
          rc = flush_object(&st);
        if (!rc && material_key(&lx, k, kn, &st.mat) < 0)
          rc = rt_set_error(RT_EPARSE, "%s: bad #rt material", path);
      }
      rt_lex_skip_line(&lx);
    }
    else
      rt_lex_skip_line(&lx); /* comments, vt, s, l, ... */
  }
  if (!rc)
    rc = flush_object(&st);
  free(st.tris.a);
  free(vs.a);
  free(vns.a);
  free(lib.a);
  rt_prescan_free(&ps);
  rt_lex_close(&lx);
  return rc;
}

int rt_scene_load_obj(const char *path, rt_scene **out)
{
  if (!path || !out)
    return rt_set_error(RT_EINVAL, "null argument");
  rt_scene *s = calloc(1, sizeof *s);
  if (!s)
    return rt_set_error(RT_ENOMEM, "scene");
  int rc = rt_scene_append_obj(s, path);
  if (rc)
  {
    rt_scene_free(s);
    return rc;
  }
  *out = s;
  return RT_OK;
}

typedef struct {
  const rt_scene *s;
  const size_t *base; /* first vertex index (1-based) of each object */
} obj_ctx;

/* unit 0 of an object: its `o` line and #rt material block; then 3t `v`
 * lines, 3t `vn` lines and t `f` lines (t triangles) */
static size_t obj_unit(const void *ctx_, size_t oi, size_t j, char *p)
{
  const obj_ctx *ctx = ctx_;
  const rt_object *o = &ctx->s->objects[oi];
  const size_t nv = 3 * (size_t)o->triangle_count;
  if (j == 0)
    return (size_t)snprintf(p, RT_UNIT_MAX,
                            "o object%zu\n#rt Ka %.9g %.9g %.9g\n#rt Kd %.9g %.9g %.9g\n"
                            "#rt Ks %.9g %.9g %.9g\n#rt Ns %.9g\n#rt Ni %.9g\n#rt Nr %.9g\n"
                            "#rt d %.9g\n",
                            oi, (double)o->ka.x, (double)o->ka.y, (double)o->ka.z, (double)o->kd.x,
                            (double)o->kd.y, (double)o->kd.z, (double)o->ks.x, (double)o->ks.y,
                            (double)o->ks.z, (double)o->ns, (double)o->ni, (double)o->nr,
                            (double)o->d);
  j--;
  if (j < 2 * nv)
  {
    const int normal = j >= nv;
    const size_t m = normal ? j - nv : j;
    const rt_vec3 v = normal ? o->triangles[m / 3].normal[m % 3] : o->triangles[m / 3].vertex[m % 3];
    return (size_t)snprintf(p, RT_UNIT_MAX, "%s %.9g %.9g %.9g\n", normal ? "vn" : "v",
                            (double)v.x, (double)v.y, (double)v.z);
  }
  const size_t a = ctx->base[oi] + 3 * (j - 2 * nv);
  return (size_t)snprintf(p, RT_UNIT_MAX, "f %zu//%zu %zu//%zu %zu//%zu\n", a, a, a + 1, a + 1,
                          a + 2, a + 2);
}

int rt_scene_write_obj(const rt_scene *s, const char *path)
{
  FILE *f = fopen(path, "w");
  if (!f)
    return rt_set_error(RT_EIO, "%s: %s", path, strerror(errno));
  size_t *units = malloc((2 * s->object_count + 1) * sizeof *units);
  if (!units)
  {
    fclose(f);
    return rt_set_error(RT_ENOMEM, "writer");
  }
  size_t *base = units + s->object_count;
  size_t b = 1;
  for (size_t i = 0; i < s->object_count; i++)
  {
    units[i] = 1 + 7 * (size_t)s->objects[i].triangle_count;
    base[i] = b;
    b += 3 * (size_t)s->objects[i].triangle_count;
  }
  obj_ctx ctx = { s, base };
  int rc = rt_par_write(f, &ctx, s->object_count, units, obj_unit);
  free(units);
  if (fclose(f) != 0 && !rc)
    rc = rt_set_error(RT_EIO, "%s: write failed", path);
  return rc;
}
