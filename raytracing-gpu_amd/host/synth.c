/*
 * synth.c -- deterministic synthetic scene for config C5:
 * a gx x gy field of smooth UV spheres standing on a ground quad, seeded
 * with splitmix64, lit by a_light 0.2 / d_light (1,-1,1) / one p_light,
 * viewed by `camera W H 0 4 -20 1 0 0 0 -1 0 70`.  Every 8th sphere (by the
 * random draw) is reflective (Nr 0.3).  New code: the reference ships no
 * generator.  The result is the same scene rt_scene_write_svati / _obj
 * serialise, so the oracle, the reference parser and the .obj loader all
 * see identical triangles.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static unsigned long long splitmix64(unsigned long long *s)
{
  unsigned long long z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double uniform(unsigned long long *s) { return (double)(splitmix64(s) >> 11) * 0x1.0p-53; }

static rt_vec3 mk(double x, double y, double z)
{
  rt_vec3 v = { (float)x, (float)y, (float)z };
  return v;
}

/* triangles of a stacks x slices UV sphere: 2*slices*(stacks-1).
 * slices / stacks is kept in [1.5, 2.2] so the quads stay near square at the
 * equator (a slice spans 2 pi / slices, a stack pi / stacks); among those
 * shapes the triangle count nearest the target wins, ties towards 1.8.
 * (Round 1 only bounded the ratio from above and picked 258 x 19, i.e.
 * 27:1 sliver triangles -- DESIGN.md §2; rt_scene_synthetic_uv still builds
 * that tessellation on request.) */
static void sphere_shape(unsigned target, unsigned *stacks, unsigned *slices)
{
  unsigned best_st = 3, best_sl = 5;
  unsigned long best_err = ~0ul;
  double best_dev = 1e30;
  for (unsigned st = 3; st < 4096; st++)
  {
    unsigned sl = (unsigned)((double)target / (2.0 * (st - 1)) + 0.5);
    if (sl < 4)
      break;
    if (10 * sl > 22 * st || 2 * sl < 3 * st)
      continue; /* slices / stacks outside [1.5, 2.2] */
    unsigned long n = 2ul * sl * (st - 1);
    unsigned long err = n > target ? n - target : target - n;
    double dev = fabs((double)sl / st - 1.8);
    if (err < best_err || (err == best_err && dev < best_dev))
    {
      best_err = err;
      best_dev = dev;
      best_st = st;
      best_sl = sl;
    }
  }
  *stacks = best_st;
  *slices = best_sl;
}

static void emit_sphere(rt_triangle *out, unsigned stacks, unsigned slices, double cx, double cy,
                        double cz, double r)
{
  size_t n = 0;
  for (unsigned i = 0; i < stacks; i++)
  {
    double t0 = M_PI * i / stacks, t1 = M_PI * (i + 1) / stacks;
    for (unsigned j = 0; j < slices; j++)
    {
      double p0 = 2 * M_PI * j / slices, p1 = 2 * M_PI * (j + 1) / slices;
      double dir[4][3] = {
        { sin(t0) * cos(p0), cos(t0), sin(t0) * sin(p0) },
        { sin(t1) * cos(p0), cos(t1), sin(t1) * sin(p0) },
        { sin(t1) * cos(p1), cos(t1), sin(t1) * sin(p1) },
        { sin(t0) * cos(p1), cos(t0), sin(t0) * sin(p1) },
      };
      int quads[2][3] = { { 0, 1, 2 }, { 0, 2, 3 } };
      for (int q = 0; q < 2; q++)
      {
        if (q == 0 && i == stacks - 1)
          continue; /* bottom cap: 1 triangle per slice */
        if (q == 1 && i == 0)
          continue; /* top cap */
        rt_triangle *t = &out[n++];
        for (int k = 0; k < 3; k++)
        {
          const double *d = dir[quads[q][k]];
          t->vertex[k] = mk(cx + r * d[0], cy + r * d[1], cz + r * d[2]);
          t->normal[k] = mk(d[0], d[1], d[2]);
        }
      }
    }
  }
}

int rt_scene_synthetic(unsigned gx, unsigned gy, unsigned tris_per_sphere, unsigned long long seed,
                       int width, int height, rt_scene **out)
{
  if (tris_per_sphere < 8)
    return rt_set_error(RT_EINVAL, "rt_scene_synthetic: bad argument");
  unsigned stacks, slices;
  sphere_shape(tris_per_sphere, &stacks, &slices);
  return rt_scene_synthetic_uv(gx, gy, stacks, slices, seed, width, height, out);
}

int rt_scene_synthetic_uv(unsigned gx, unsigned gy, unsigned stacks, unsigned slices,
                          unsigned long long seed, int width, int height, rt_scene **out)
{
  if (!out || gx == 0 || gy == 0 || stacks < 3 || slices < 3 || width <= 0 || height <= 0)
    return rt_set_error(RT_EINVAL, "rt_scene_synthetic: bad argument");
  unsigned per = 2 * slices * (stacks - 1);
  rt_scene *s = calloc(1, sizeof *s);
  if (!s)
    return rt_set_error(RT_ENOMEM, "scene");
  size_t nobj = (size_t)gx * gy + 1;
  s->objects = calloc(nobj, sizeof *s->objects);
  s->lights = calloc(3, sizeof *s->lights);
  if (!s->objects || !s->lights)
  {
    rt_scene_free(s);
    return rt_set_error(RT_ENOMEM, "scene");
  }
  s->camera.width = width;
  s->camera.height = height;
  s->camera.position = mk(0, 4, -20);
  s->camera.u = mk(1, 0, 0);
  s->camera.v = mk(0, -1, 0);
  s->camera.fov = 70;
  s->lights[0].type = RT_AMBIENT;
  s->lights[0].r = s->lights[0].g = s->lights[0].b = 0.2f;
  s->lights[1].type = RT_DIRECTIONAL;
  s->lights[1].r = s->lights[1].g = s->lights[1].b = 1.0f;
  s->lights[1].v = mk(1, -1, 1);
  s->lights[2].type = RT_POINT;
  s->lights[2].r = s->lights[2].g = s->lights[2].b = 0.8f;
  s->lights[2].v = mk(-6, 12, -4);
  s->light_count = 3;

  unsigned long long st = seed;
  const double spacing = 3.0, z0 = -10.0;
  /* ground quad under the whole field */
  rt_object *g = &s->objects[0];
  memset(g, 0, sizeof *g);
  g->ni = 1;
  g->d = 1;
  g->ka = g->kd = mk(0.5, 0.5, 0.5);
  g->ks = mk(0.1, 0.1, 0.1);
  g->ns = 10;
  g->triangles = calloc(2, sizeof *g->triangles);
  if (!g->triangles)
  {
    rt_scene_free(s);
    return rt_set_error(RT_ENOMEM, "ground");
  }
  g->triangle_count = 2;
  double xmin = -spacing * gx / 2 - 4, xmax = spacing * gx / 2 + 4;
  double zmin = z0 - 4, zmax = z0 + spacing * gy + 4;
  rt_vec3 gc[4] = { mk(xmin, 0, zmin), mk(xmax, 0, zmin), mk(xmax, 0, zmax), mk(xmin, 0, zmax) };
  int gi[2][3] = { { 0, 2, 1 }, { 0, 3, 2 } };
  for (int t = 0; t < 2; t++)
    for (int k = 0; k < 3; k++)
    {
      g->triangles[t].vertex[k] = gc[gi[t][k]];
      g->triangles[t].normal[k] = mk(0, 1, 0);
    }
  s->object_count = 1;
  for (unsigned iy = 0; iy < gy; iy++)
    for (unsigned ix = 0; ix < gx; ix++)
    {
      rt_object *o = &s->objects[s->object_count];
      memset(o, 0, sizeof *o);
      double r = 0.8 + 0.4 * uniform(&st);
      double cx = spacing * (ix - (gx - 1) / 2.0);
      double cz = z0 + spacing * iy + spacing / 2;
      double cr = uniform(&st), cg = uniform(&st), cb = uniform(&st);
      int reflective = (splitmix64(&st) & 7) == 0;
      o->ka = mk(0.2 * cr, 0.2 * cg, 0.2 * cb);
      o->kd = mk(cr, cg, cb);
      o->ks = mk(0.6, 0.6, 0.6);
      o->ns = 40;
      o->ni = 1;
      o->nr = reflective ? 0.3f : 0.0f;
      o->d = 1;
      o->triangles = malloc((size_t)per * sizeof *o->triangles);
      if (!o->triangles)
      {
        rt_scene_free(s);
        return rt_set_error(RT_ENOMEM, "sphere");
      }
      o->triangle_count = per;
      emit_sphere(o->triangles, stacks, slices, cx, r, cz, r);
      s->object_count++;
    }
  *out = s;
  return RT_OK;
}
