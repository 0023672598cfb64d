/*
 * scene_svati.c -- .svati loader and writer (host C).
 *
 * Same grammar and same results as the reference parser:
 *   top level  cpu/parser.c:62-116   camera / a_light / d_light / p_light / object / #
 *   object     cpu/parse_obj.c:42-92 count, then Ka Kd Ks Ns Ni Nr d v vn until
 *                                    2*count v/vn lines have been read
 *   ordering   cpu/parse_obj.c:29-40,83-88 + cpu/stack.c:23-47: vertices and
 *              normals go on LIFO stacks, triangles pop them, so triangle t,
 *              corner k is the object's (N-1-3t-k)-th v line (same for vn)
 *   defaults   cpu/parse_obj.c:3-20  ka=kd=ks=0, ns=0, ni=1, nr=0, d=1
 *   numbers    fscanf %f / %d / %u  ==  strtof / strtol / strtoul (both round
 *              correctly), so every float is bit-identical.
 * Instead of fscanf on a FILE the whole file is read once and scanned with a
 * cursor (the reference's token loop is the bottleneck for large scenes,
 * SURVEY.md §8f item 1).
 * Extension: `objfile <path>` appends the objects of a Wavefront .obj.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"
#include "rt_lex.h"
#include "rt_par_write.h"

int rt_lex_open(const char *path, rt_lex *lx)
{
  memset(lx, 0, sizeof *lx);
  FILE *f = fopen(path, "rb");
  if (!f) /* the reference's text: errx(1, "%s\n", strerror(errno)) (cpu/parser.c:70-71) */
    return rt_set_error(RT_EIO, "%s", strerror(errno));
  if (fseek(f, 0, SEEK_END) != 0)
  {
    fclose(f);
    return rt_set_error(RT_EIO, "%s: cannot seek", path);
  }
  long size = ftell(f);
  rewind(f);
  char *buf = malloc((size_t)size + 1);
  if (!buf)
  {
    fclose(f);
    return rt_set_error(RT_ENOMEM, "%s: %ld bytes", path, size);
  }
  if (size > 0 && fread(buf, 1, (size_t)size, f) != (size_t)size)
  {
    free(buf);
    fclose(f);
    return rt_set_error(RT_EIO, "%s: short read", path);
  }
  fclose(f);
  buf[size] = 0;
  lx->buf = buf;
  lx->p = buf;
  lx->end = buf + size;
  lx->path = path;
  return RT_OK;
}

void rt_lex_close(rt_lex *lx)
{
  free(lx->buf);
  lx->buf = NULL;
}

/* ---- growable arrays ---- */

static int grow(void **ptr, size_t *cap, size_t need, size_t elem)
{
  if (need <= *cap)
    return RT_OK;
  size_t nc = *cap ? *cap : 16;
  while (nc < need)
    nc *= 2;
  void *np = realloc(*ptr, nc * elem);
  if (!np)
    return rt_set_error(RT_ENOMEM, "realloc %zu x %zu", nc, elem);
  *ptr = np;
  *cap = nc;
  return RT_OK;
}

typedef struct { rt_vec3 *a; size_t n, cap; } vecbuf;

static int vb_push(vecbuf *b, rt_vec3 x)
{
  int rc = grow((void **)&b->a, &b->cap, b->n + 1, sizeof *b->a);
  if (rc)
    return rc;
  b->a[b->n++] = x;
  return RT_OK;
}

int rt_scene_push_object(rt_scene *s, const rt_object *o, size_t *cap)
{
  int rc = grow((void **)&s->objects, cap, s->object_count + 1, sizeof *s->objects);
  if (rc)
    return rc;
  s->objects[s->object_count++] = *o;
  return RT_OK;
}

static int push_light(rt_scene *s, rt_light l)
{
  rt_light *nl = realloc(s->lights, (s->light_count + 1) * sizeof *nl);
  if (!nl)
    return rt_set_error(RT_ENOMEM, "lights");
  s->lights = nl;
  s->lights[s->light_count++] = l;
  return RT_OK;
}

void rt_object_defaults(rt_object *o)
{
  memset(o, 0, sizeof *o);
  o->ni = 1; /* cpu/parse_obj.c:16-18 */
  o->d = 1;
}

static int lex_num(rt_lex *lx, float *x)
{
  return rt_lex_float(lx, x) ? rt_set_error(RT_EPARSE, "%s: expected a number near byte %td",
                                            lx->path, lx->p - lx->buf)
                             : RT_OK;
}

static int lex_vec(rt_lex *lx, rt_vec3 *v)
{
  return rt_lex_float(lx, &v->x) || rt_lex_float(lx, &v->y) || rt_lex_float(lx, &v->z)
           ? rt_set_error(RT_EPARSE, "%s: expected 3 numbers near byte %td", lx->path,
                          lx->p - lx->buf)
           : RT_OK;
}

/* cpu/parse_obj.c:42-92 */
static int parse_object(rt_lex *lx, rt_prescan *ps, rt_object *obj, vecbuf *vs, vecbuf *ns)
{
  rt_object_defaults(obj);
  unsigned declared;
  if (rt_lex_uint(lx, &declared))
    return rt_set_error(RT_EPARSE, "%s: object without vertex count", lx->path);
  vs->n = ns->n = 0;
  unsigned seen = 0;
  int rc = RT_OK;
  while (!rc && seen < declared * 2u)
  {
    const char *t;
    size_t n;
    if (!rt_lex_token(lx, &t, &n))
      break; /* EOF ends the object, as fscanf()==EOF does */
    if (RT_TOK_IS(t, n, "Ka")) rc = lex_vec(lx, &obj->ka);
    else if (RT_TOK_IS(t, n, "Kd")) rc = lex_vec(lx, &obj->kd);
    else if (RT_TOK_IS(t, n, "Ks")) rc = lex_vec(lx, &obj->ks);
    else if (RT_TOK_IS(t, n, "Ns")) rc = lex_num(lx, &obj->ns);
    else if (RT_TOK_IS(t, n, "Ni")) rc = lex_num(lx, &obj->ni);
    else if (RT_TOK_IS(t, n, "Nr")) rc = lex_num(lx, &obj->nr);
    else if (RT_TOK_IS(t, n, "d")) rc = lex_num(lx, &obj->d);
    else if (RT_TOK_IS(t, n, "v") || RT_TOK_IS(t, n, "vn"))
    {
      rt_vec3 x;
      float f[3];
      seen++;
      if (rt_prescan_take(ps, lx, t, f))
        x.x = f[0], x.y = f[1], x.z = f[2];
      else
        rc = lex_vec(lx, &x);
      if (!rc)
        rc = vb_push(n == 2 ? ns : vs, x);
    }
    else /* cpu/parse_obj.c:80-81 (object level: "parsing", not "the parsing") */
      rc = rt_set_error(RT_EPARSE, "Error during parsing %.*s", (int)n, t);
  }
  if (rc)
    return rc;
  size_t nv = vs->n;
  /* Deliberately stricter than the reference, which has no defined result
   * here: it pops 3 v + 3 vn per triangle until the v stack is empty
   * (cpu/parse_obj.c:83-88; a NULL head is dereferenced when v is not a
   * multiple of 3 or vn runs out first, cpu/stack.c:36-39) and then sets
   * triangle_count = declared / 3 (cpu/parse_obj.c:89) whatever it popped,
   * so fewer v lines than declared leave triangles it never allocated.  Such
   * files are rejected (tests/test_host.py). */
  if (nv % 3 != 0 || ns->n < nv || nv != declared)
    return rt_set_error(RT_EPARSE, "%s: object declares %u vertices, has %zu v / %zu vn",
                        lx->path, declared, nv, ns->n);
  size_t ntri = nv / 3;
  obj->triangles = malloc((ntri ? ntri : 1) * sizeof *obj->triangles);
  if (!obj->triangles)
    return rt_set_error(RT_ENOMEM, "%zu triangles", ntri);
  /* LIFO pop order of cpu/parse_obj.c:83-88 */
  for (size_t t = 0; t < ntri; t++)
    for (int k = 0; k < 3; k++)
    {
      obj->triangles[t].vertex[k] = vs->a[nv - 1 - 3 * t - (size_t)k];
      obj->triangles[t].normal[k] = ns->a[ns->n - 1 - 3 * t - (size_t)k];
    }
  obj->triangle_count = (unsigned)ntri;
  return RT_OK;
}

static int dir_join(const char *base, const char *rel, size_t rel_len, char *out, size_t cap)
{
  if (rel_len == 0 || rel_len >= cap)
    return RT_EINVAL;
  if (rel[0] == '/')
  {
    memcpy(out, rel, rel_len);
    out[rel_len] = 0;
    return RT_OK;
  }
  const char *slash = strrchr(base, '/');
  size_t dl = slash ? (size_t)(slash - base + 1) : 0;
  if (dl + rel_len + 1 > cap)
    return RT_EINVAL;
  memcpy(out, base, dl);
  memcpy(out + dl, rel, rel_len);
  out[dl + rel_len] = 0;
  return RT_OK;
}

int rt_scene_load_svati(const char *path, rt_scene **out)
{
  if (!path || !out)
    return rt_set_error(RT_EINVAL, "null argument");
  rt_set_error(RT_OK, "");
  rt_lex lx;
  int rc = rt_lex_open(path, &lx);
  if (rc)
    return rc;
  rt_scene *s = calloc(1, sizeof *s);
  if (!s)
  {
    rt_lex_close(&lx);
    return rt_set_error(RT_ENOMEM, "scene");
  }
  size_t obj_cap = 0;
  vecbuf vs = { 0 }, ns = { 0 };
  rt_prescan ps;
  rt_prescan_build(&lx, &ps);
  const char *t;
  size_t n;
  while (!rc && rt_lex_token(&lx, &t, &n))
  {
    rt_light l;
    memset(&l, 0, sizeof l);
    if (RT_TOK_IS(t, n, "camera"))
    {
      /* cpu/parser.c:4-21 */
      rt_camera *c = &s->camera;
      if (rt_lex_int(&lx, &c->width) || rt_lex_int(&lx, &c->height) ||
          lex_vec(&lx, &c->position) || lex_vec(&lx, &c->u) || lex_vec(&lx, &c->v) ||
          rt_lex_float(&lx, &c->fov))
        rc = rt_set_error(RT_EPARSE, "%s: bad camera line", path);
    }
    else if (RT_TOK_IS(t, n, "a_light"))
    {
      /* cpu/parser.c:23-32 */
      l.type = RT_AMBIENT;
      if (rt_lex_float(&lx, &l.r) || rt_lex_float(&lx, &l.g) || rt_lex_float(&lx, &l.b))
        rc = rt_set_error(RT_EPARSE, "%s: bad a_light", path);
      else
        rc = push_light(s, l);
    }
    else if (RT_TOK_IS(t, n, "d_light") || RT_TOK_IS(t, n, "p_light"))
    {
      /* cpu/parser.c:34-60 */
      l.type = t[0] == 'd' ? RT_DIRECTIONAL : RT_POINT;
      if (rt_lex_float(&lx, &l.r) || rt_lex_float(&lx, &l.g) || rt_lex_float(&lx, &l.b) ||
          lex_vec(&lx, &l.v))
        rc = rt_set_error(RT_EPARSE, "%s: bad light", path);
      else
        rc = push_light(s, l);
    }
    else if (RT_TOK_IS(t, n, "object"))
    {
      rt_object o;
      rc = parse_object(&lx, &ps, &o, &vs, &ns);
      if (!rc)
        rc = rt_scene_push_object(s, &o, &obj_cap);
      else
        free(o.triangles);
    }
    else if (RT_TOK_IS(t, n, "#"))
    {
      /* fscanf(" %[^\n]") (cpu/parser.c:108-109): skip blanks *including
       * newlines*, then the rest of that line */
      rt_lex_skip_ws(&lx);
      rt_lex_skip_line(&lx);
    }
    else if (RT_TOK_IS(t, n, "objfile"))
    {
      const char *fp;
      size_t fl;
      char full[4096];
      if (!rt_lex_token(&lx, &fp, &fl) || dir_join(path, fp, fl, full, sizeof full))
        rc = rt_set_error(RT_EPARSE, "%s: objfile needs a path", path);
      else
      {
        /* objects appended in file order after those already read */
        rc = rt_scene_append_obj(s, full);
        obj_cap = s->object_count;
      }
    }
    else
      rc = rt_set_error(RT_EPARSE, "Error during the parsing %.*s", (int)n, t);
  }
  free(vs.a);
  free(ns.a);
  rt_prescan_free(&ps);
  rt_lex_close(&lx);
  if (rc)
  {
    rt_scene_free(s);
    return rc;
  }
  *out = s;
  return RT_OK;
}

size_t rt_scene_triangle_count(const rt_scene *s)
{
  size_t n = 0;
  for (size_t i = 0; s && i < s->object_count; i++)
    n += s->objects[i].triangle_count;
  return n;
}

void rt_scene_free(rt_scene *s)
{
  if (!s)
    return;
  for (size_t i = 0; i < s->object_count; i++)
    free(s->objects[i].triangles);
  free(s->objects);
  free(s->lights);
  free(s);
}

/* ---- writer ---- */

/* unit 0 of an object: its header block; units 1..nv its `v` lines, then nv
 * `vn` lines.  The parser pops from the end: line m holds corner nv-1-m. */
static size_t svati_unit(const void *ctx, size_t oi, size_t j, char *p)
{
  const rt_object *o = &((const rt_scene *)ctx)->objects[oi];
  size_t nv = 3 * (size_t)o->triangle_count;
  if (j == 0)
    return (size_t)snprintf(p, RT_UNIT_MAX,
                            "\nobject %zu\nNs %.9g\nNi %.9g\nNr %.9g\nd %.9g\n"
                            "Ka %.9g %.9g %.9g\nKd %.9g %.9g %.9g\nKs %.9g %.9g %.9g\n",
                            nv, (double)o->ns, (double)o->ni, (double)o->nr, (double)o->d,
                            (double)o->ka.x, (double)o->ka.y, (double)o->ka.z, (double)o->kd.x,
                            (double)o->kd.y, (double)o->kd.z, (double)o->ks.x, (double)o->ks.y,
                            (double)o->ks.z);
  const int normal = j > nv;
  size_t idx = nv - 1 - (normal ? j - 1 - nv : j - 1);
  const rt_vec3 v = normal ? o->triangles[idx / 3].normal[idx % 3]
                           : o->triangles[idx / 3].vertex[idx % 3];
  return (size_t)snprintf(p, RT_UNIT_MAX, "%s %.9g %.9g %.9g\n", normal ? "vn" : "v", (double)v.x,
                          (double)v.y, (double)v.z);
}

int rt_scene_write_svati(const rt_scene *s, const char *path)
{
  FILE *f = fopen(path, "w");
  if (!f)
    return rt_set_error(RT_EIO, "%s: %s", path, strerror(errno));
  const rt_camera *c = &s->camera;
  fprintf(f, "camera %d %d %.9g %.9g %.9g %.9g %.9g %.9g %.9g %.9g %.9g %.9g\n", c->width,
          c->height, (double)c->position.x, (double)c->position.y, (double)c->position.z,
          (double)c->u.x, (double)c->u.y, (double)c->u.z, (double)c->v.x, (double)c->v.y,
          (double)c->v.z, (double)c->fov);
  for (size_t i = 0; i < s->light_count; i++)
  {
    const rt_light *l = &s->lights[i];
    if (l->type == RT_AMBIENT)
      fprintf(f, "a_light %.9g %.9g %.9g\n", (double)l->r, (double)l->g, (double)l->b);
    else if (l->type == RT_DIRECTIONAL || l->type == RT_POINT)
      fprintf(f, "%s %.9g %.9g %.9g %.9g %.9g %.9g\n", l->type == RT_POINT ? "p_light" : "d_light",
              (double)l->r, (double)l->g, (double)l->b, (double)l->v.x, (double)l->v.y,
              (double)l->v.z);
  }
  size_t *units = malloc((s->object_count + 1) * sizeof *units);
  if (!units)
  {
    fclose(f);
    return rt_set_error(RT_ENOMEM, "writer");
  }
  for (size_t i = 0; i < s->object_count; i++)
    units[i] = 1 + 6 * (size_t)s->objects[i].triangle_count;
  int rc = rt_par_write(f, s, s->object_count, units, svati_unit);
  free(units);
  if (fclose(f) != 0 && !rc)
    rc = rt_set_error(RT_EIO, "%s: write failed", path);
  return rc;
}
