/*
 * rt_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker / CPU baseline).
 *
 * A plain-C restatement of the reference cpu/rt algorithm, operation for
 * operation in the same float/double types so that it reproduces the
 * reference framebuffer bit for bit.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It is pinned against the
 * golden framebuffers in tests/golden/ that the reference's own sources
 * (compiled by oracle/Makefile into oracle/_ref/rt_probe) produced.
 *
 * Deliberately brute force: every query tests every triangle of every
 * object, like /root/reference/cpu/hit.c:72-109, so that timing it is a fair
 * "cpu/rt on the host cores" baseline.  Differences from the reference that
 * do not change any bit: heap framebuffer instead of a stack VLA
 * (cpu/raytracer.c:91), N worker threads pulling pixels from a counter
 * instead of 4 fixed quadrants (cpu/raytracer.c:92-127), arbitrary pixel
 * subsets for sampled timing.
 *
 * Must be compiled with -ffp-contract=off and without fast-math.
 */
#define _GNU_SOURCE
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

typedef struct or_vec3 vec3;
typedef struct or_color color;
typedef struct or_ray ray;

/* ---- vector algebra: cpu/vector3.c:3-47, cpu/vector3-extern.c:5-23 ---- */

static vec3 v_sub(vec3 a, vec3 b) { vec3 r = { a.x - b.x, a.y - b.y, a.z - b.z }; return r; }
static vec3 v_add(vec3 a, vec3 b) { vec3 r = { a.x + b.x, a.y + b.y, a.z + b.z }; return r; }
static vec3 v_cross(vec3 a, vec3 b)
{
  vec3 r = { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x };
  return r;
}
/* vector3_scale multiplies scalar-first: r * a.x (cpu/vector3.c:30-37) */
static vec3 v_scale(vec3 a, float s) { vec3 r = { s * a.x, s * a.y, s * a.z }; return r; }
static float v_dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* length goes through double sqrt (cpu/vector3-extern.c:10-13) */
static float v_length(vec3 a) { return (float)sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static vec3 v_normalize(vec3 a)
{
  float len = v_length(a);
  vec3 r = { a.x / len, a.y / len, a.z / len };
  return r;
}
static int v_is_zero(vec3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }

/* ---- colour algebra: cpu/colors.c:3-49 (float channels 0..255) ---- */

static float clamp_channel(float x)
{
  float y = x * 255;
  if (y > 255)
    y = 255;
  if (y < 0)
    y = 0;
  return y;
}
color oracle_init_color(float r, float g, float b)
{
  color c = { clamp_channel(r), clamp_channel(g), clamp_channel(b) };
  return c;
}
color oracle_color_add(color a, color b)
{
  a.r += b.r;
  if (a.r > 255) a.r = 255;
  a.g += b.g;
  if (a.g > 255) a.g = 255;
  a.b += b.b;
  if (a.b > 255) a.b = 255;
  return a;
}
color oracle_color_mul(color a, float coef)
{
  return oracle_init_color(a.r / 255 * coef, a.g / 255 * coef, a.b / 255 * coef);
}
color oracle_color_mul2(color a, color b)
{
  return oracle_init_color((a.r / 255) * (b.r / 255), (a.g / 255) * (b.g / 255),
                           (a.b / 255) * (b.b / 255));
}

/* ---- intersection: cpu/hit.c:4-109 ---- */

/* Moller-Trumbore exactly as cpu/hit.c:4-44, including the per-test
 * normalisation of the three vertex normals (cpu/hit.c:11-13). */
static int intersect(ray r, const struct or_triangle *tri, vec3 *out, vec3 *normal)
{
  const float eps = 0.0000001;
  vec3 n0 = v_normalize(tri->normal[0]);
  vec3 n1 = v_normalize(tri->normal[1]);
  vec3 n2 = v_normalize(tri->normal[2]);
  vec3 e1 = v_sub(tri->vertex[1], tri->vertex[0]);
  vec3 e2 = v_sub(tri->vertex[2], tri->vertex[0]);
  vec3 h = v_cross(r.direction, e2);
  float a = v_dot(e1, h);
  if (a > -eps && a < eps)
    return 0;
  float f = 1 / a;
  vec3 s = v_sub(r.origin, tri->vertex[0]);
  float u = f * v_dot(s, h);
  if (u < 0.0 || u > 1.0)
    return 0;
  vec3 q = v_cross(s, e1);
  float v = f * v_dot(r.direction, q);
  if (v < 0.0 || u + v > 1.0)
    return 0;
  float t = f * v_dot(e2, q);
  if (!(t > eps))
    return 0;
  vec3 step = v_scale(v_normalize(r.direction), t * v_length(r.direction));
  *out = v_add(r.origin, step);
  *normal = v_add(v_add(v_scale(n0, 1 - u - v), v_scale(n1, u)), v_scale(n2, v));
  return 1;
}

/* Closest hit inside one object (cpu/hit.c:46-70): strict '<' keeps the
 * first triangle on ties; distance 0 means "nothing yet". */
static ray object_closest(const struct or_object *obj, ray r)
{
  float best = 0;
  ray ret = { { 0, 0, 0 }, { 0, 0, 0 } };
  for (size_t i = 0; i < obj->triangle_count; i++)
  {
    vec3 out, normal;
    if (!intersect(r, &obj->triangles[i], &out, &normal))
      continue;
    float d = v_length(v_sub(out, r.origin));
    if (d > 0.01 && (d < best || best == 0))
    {
      best = d;
      ret.origin = out;
      ret.direction = normal;
    }
  }
  return ret;
}

/* cpu/hit.c:72-91.  An object whose closest triangle has an exactly zero
 * interpolated normal is skipped (cpu/hit.c:79). */
ray oracle_collide(const struct or_scene *scene, ray r, int *object_index)
{
  float best = 0;
  ray ret = { { 0, 0, 0 }, { 0, 0, 0 } };
  for (size_t i = 0; i < scene->object_count; i++)
  {
    ray cand = object_closest(&scene->objects[i], r);
    if (v_is_zero(cand.direction))
      continue;
    float d = v_length(v_sub(cand.origin, r.origin));
    if (d > 0.01 && (d < best || best == 0))
    {
      best = d;
      ret = cand;
      *object_index = (int)i;
    }
  }
  return ret;
}

/* cpu/hit.c:93-109 */
float oracle_collide_dist(const struct or_scene *scene, ray r)
{
  float best = 0;
  for (size_t i = 0; i < scene->object_count; i++)
  {
    ray cand = object_closest(&scene->objects[i], r);
    if (v_is_zero(cand.direction))
      continue;
    float d = v_length(v_sub(cand.origin, r.origin));
    if (d > 0.01 && (d < best || best == 0))
      best = d;
  }
  return best;
}

/* ---- shading: cpu/light.c:7-100 ---- */

struct tls_counts { unsigned long long closest, shadow, max_depth; };

/* cpu/light.c:24-31: lit unless collide_dist finds something (fdist != 0) */
static int shadowed(const struct or_scene *scene, ray r, struct tls_counts *cnt)
{
  cnt->shadow++;
  return oracle_collide_dist(scene, r) != 0;
}

/* cpu/light.c:7-22 */
static void specular(color *acc, ray incident, ray hit, const struct or_object *obj)
{
  color k = oracle_init_color(obj->ks.x, obj->ks.y, obj->ks.z);
  vec3 V = v_sub(incident.origin, hit.origin);
  vec3 R = v_sub(incident.direction,
                 v_scale(hit.direction, 2 * v_dot(hit.direction, incident.direction)));
  R = v_normalize(R);
  V = v_normalize(V);
  float ls = (float)pow(fmax(v_dot(R, V), 0.0), obj->ns);
  k = oracle_color_mul(k, ls);
  *acc = oracle_color_add(*acc, k);
}

static color shade(const struct or_scene *scene, const struct or_object *obj, ray hit,
                   struct tls_counts *cnt)
{
  color acc = oracle_init_color(0, 0, 0);
  for (size_t i = 0; i < scene->light_count; i++)
  {
    const struct or_light *l = &scene->lights[i];
    if (l->type == OR_AMBIENT)
    {
      /* cpu/light.c:42-48 */
      color t = oracle_color_mul2(oracle_init_color(l->r, l->g, l->b),
                                  oracle_init_color(obj->ka.x, obj->ka.y, obj->ka.z));
      acc = oracle_color_add(acc, t);
    }
    else if (l->type == OR_DIRECTIONAL)
    {
      /* cpu/light.c:49-69: shadow ray towards -v (not normalised) */
      ray sr = { hit.origin, v_scale(l->v, -1) };
      if (shadowed(scene, sr, cnt))
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
      /* cpu/light.c:70-93: "L" is minus the light *position*; N may flip
       * for the diffuse term only; specular uses the unflipped hit normal. */
      vec3 L = v_scale(l->v, -1);
      vec3 N = hit.direction;
      if (v_dot(L, N) < 0)
        N = v_scale(N, -1);
      vec3 to_light = v_sub(l->v, hit.origin);
      float dist = v_length(v_sub(l->v, hit.origin));
      ray sr = { hit.origin, to_light };
      if (shadowed(scene, sr, cnt))
        continue;
      color t = oracle_color_mul2(oracle_init_color(l->r, l->g, l->b),
                                  oracle_init_color(obj->kd.x, obj->kd.y, obj->kd.z));
      t = oracle_color_mul(t, v_dot(L, N) * 1 / dist);
      ray inc = { v_add(hit.origin, v_scale(to_light, -10)), to_light };
      specular(&t, inc, hit, obj);
      acc = oracle_color_add(acc, t);
    }
    /* SPECULAR / unknown: skipped (cpu/light.c:94-96) */
  }
  return acc;
}

color oracle_apply_light(const struct or_scene *scene, int object_index, ray point)
{
  struct tls_counts cnt = { 0, 0, 0 };
  return shade(scene, &scene->objects[object_index], point, &cnt);
}

/* cpu/ray.c:16-25 */
static ray bounce(ray in, ray hit)
{
  ray r;
  r.origin = hit.origin;
  r.direction = v_sub(in.direction,
                      v_scale(hit.direction, 2 * v_dot(hit.direction, in.direction)));
  return r;
}

/* cpu/raytracer.c:19-34, recursive as in the reference: the reflected
 * contribution is computed first and the local term added to it. */
static color trace(const struct or_scene *scene, ray r, float coef, unsigned depth,
                   struct tls_counts *cnt)
{
  if (coef < 0.01)
    return oracle_init_color(0, 0, 0);
  cnt->closest++;
  if (depth > cnt->max_depth)
    cnt->max_depth = depth;
  int oi = -1;
  ray hit = oracle_collide(scene, r, &oi);
  if (v_is_zero(hit.direction))
    return oracle_init_color(0, 0, 0);
  const struct or_object *obj = &scene->objects[oi];
  color local = shade(scene, obj, hit, cnt);
  color refl = trace(scene, bounce(r, hit), obj->nr * coef, depth + 1, cnt);
  return oracle_color_add(refl, oracle_color_mul(local, coef));
}

/* cpu/raytracer.c:82-86 */
void oracle_camera_frame(const struct or_scene *scene, vec3 *u, vec3 *v, vec3 *C)
{
  *u = v_normalize(scene->camera.u);
  *v = v_normalize(scene->camera.v);
  vec3 w = v_cross(*u, *v);
  float L = scene->camera.width / (2 * tan(scene->camera.fov * M_PI / 360));
  *C = v_add(scene->camera.position, v_scale(w, L));
}

/* One pixel (cpu/raytracer.c:54-71).  PPM pixel (row, col) is the
 * framebuffer slot the print loop (cpu/raytracer.c:128-134) reads at
 * j = (H-row) - H/2, i = (W-col) - W/2; slots the render loop never writes
 * (only for odd W or H) are left as 0 here. */
static color render_pixel(const struct or_scene *scene, vec3 u, vec3 v, vec3 C, int row,
                          int col, struct tls_counts *cnt)
{
  int W = scene->camera.width, H = scene->camera.height;
  int ii = W - col, jj = H - row;
  color black = { 0, 0, 0 };
  if (ii < 1 || ii > 2 * (W / 2) || jj < 1 || jj > 2 * (H / 2))
    return black;
  int i = ii - W / 2, j = jj - H / 2;
  color acc = oracle_init_color(0, 0, 0);
  for (float k = i; k < i + 1; k += 0.5)
    for (float l = j; l < j + 1; l += 0.5)
    {
      vec3 point = v_add(v_add(C, v_scale(u, k)), v_scale(v, l));
      ray r = { point, v_normalize(v_sub(scene->camera.position, point)) };
      color s = trace(scene, r, 1, 0, cnt);
      acc = oracle_color_add(acc, oracle_color_mul(s, 0.25));
    }
  return acc;
}

/* Camera samples (cpu/raytracer.c:50-61, the mapping of render_pixel) of
 * the PPM pixels [row0, row0 + rows) x [col0, col0 + cols) tested against one
 * triangle: out[0] = samples intersect() accepts (cpu/hit.c:15-44), out[1] =
 * samples that pass its a, u and v tests (cpu/hit.c:19-29, t not checked). */
static void camera_tri_accepts(const struct or_scene *scene, vec3 u, vec3 v, vec3 C,
                               const struct or_triangle *tri, int row0, int col0, int rows, int cols,
                               unsigned long long out[2])
{
  int W = scene->camera.width, H = scene->camera.height;
  out[0] = out[1] = 0;
  for (int row = row0; row < row0 + rows; row++)
    for (int col = col0; col < col0 + cols; col++)
    {
      int ii = W - col, jj = H - row;
      if (ii < 1 || ii > 2 * (W / 2) || jj < 1 || jj > 2 * (H / 2))
        continue;
      int i = ii - W / 2, j = jj - H / 2;
      for (float k = i; k < i + 1; k += 0.5)
        for (float l = j; l < j + 1; l += 0.5)
        {
          vec3 point = v_add(v_add(C, v_scale(u, k)), v_scale(v, l));
          ray r = { point, v_normalize(v_sub(scene->camera.position, point)) };
          vec3 hit, nrm;
          out[0] += intersect(r, tri, &hit, &nrm) ? 1 : 0;
          /* the a, u, v stages of intersect() alone */
          const float eps = 0.0000001;
          vec3 e1 = v_sub(tri->vertex[1], tri->vertex[0]);
          vec3 e2 = v_sub(tri->vertex[2], tri->vertex[0]);
          vec3 h = v_cross(r.direction, e2);
          float a = v_dot(e1, h);
          if (a > -eps && a < eps)
            continue;
          float f = 1 / a;
          vec3 s = v_sub(r.origin, tri->vertex[0]);
          float uu = f * v_dot(s, h);
          if (uu < 0.0 || uu > 1.0)
            continue;
          vec3 q = v_cross(s, e1);
          float vv = f * v_dot(r.direction, q);
          if (vv < 0.0 || uu + vv > 1.0)
            continue;
          out[1]++;
        }
    }
}

void oracle_camera_tri_accepts(const struct or_scene *scene, const struct or_triangle *tris,
                               const int *rects, size_t n, unsigned long long *out)
{
  vec3 u, v, C;
  oracle_camera_frame(scene, &u, &v, &C);
  for (size_t i = 0; i < n; i++)
    camera_tri_accepts(scene, u, v, C, &tris[i], rects[4 * i], rects[4 * i + 1], rects[4 * i + 2],
                       rects[4 * i + 3], out + 2 * i);
}

/* The same for gpu/rt's camera rays (gpu/raytracer.cu:97-103, the mapping
 * of gpu_ray_pixel): one ray per pixel (px, py) of the 3x frame (gpu/rt.cpp:
 * 72-83), rects in that frame's pixels: (py0, px0, rows, cols). */
void oracle_camera_tri_accepts_gpu(const struct or_scene *scene, const struct or_triangle *tris,
                                   const int *rects, size_t n, unsigned long long *out)
{
  struct or_scene hi = *scene;
  hi.camera.width = 3 * scene->camera.width;
  hi.camera.height = 3 * scene->camera.height;
  vec3 u, v, C;
  oracle_camera_frame(&hi, &u, &v, &C);
  const int W = hi.camera.width, H = hi.camera.height;
  const float eps = 0.0000001;
  for (size_t i = 0; i < n; i++)
  {
    const struct or_triangle *tri = &tris[i];
    const int *rc = rects + 4 * i;
    unsigned long long acc = 0, uv = 0;
    for (int py = rc[0]; py < rc[0] + rc[2]; py++)
      for (int px = rc[1]; px < rc[1] + rc[3]; px++)
      {
        if (px < 0 || px >= W || py < 0 || py >= H)
          continue;
        vec3 point = v_add(v_add(C, v_scale(u, (float)(px - W / 2))), v_scale(v, (float)(py - H / 2)));
        ray r = { point, v_normalize(v_sub(scene->camera.position, point)) };
        vec3 hit, nrm;
        acc += intersect(r, tri, &hit, &nrm) ? 1 : 0;
        vec3 e1 = v_sub(tri->vertex[1], tri->vertex[0]);
        vec3 e2 = v_sub(tri->vertex[2], tri->vertex[0]);
        vec3 h = v_cross(r.direction, e2);
        float a = v_dot(e1, h);
        if (a > -eps && a < eps)
          continue;
        float f = 1 / a;
        vec3 s = v_sub(r.origin, tri->vertex[0]);
        float uu = f * v_dot(s, h);
        if (uu < 0.0 || uu > 1.0)
          continue;
        vec3 q = v_cross(s, e1);
        float vv = f * v_dot(r.direction, q);
        if (vv < 0.0 || uu + vv > 1.0)
          continue;
        uv++;
      }
    out[2 * i] = acc;
    out[2 * i + 1] = uv;
  }
}

/* ---- gpu/rt compatibility mode ----
 * gpu/raytracer.cu:31-129, gpu/light.cu:12-126, gpu/colors.cu:3-49 as the
 * sources read (PARTITIONING_NONE order of gpu/hit.cu:83-116, which is
 * cpu/hit.c's), without nvcc's default FMA contraction, with pow(float,
 * float) taken as the f64 pow rounded to float.  uint8 colours. */
typedef struct { unsigned char r, g, b; } color8;

/* gpu/colors.cu:3-20 */
static unsigned char chan8(float x)
{
  x = x * 255;
  if (x > 255)
    x = 255;
  if (x < 0)
    x = 0;
  return x == x ? (unsigned char)x : 0;
}
static color8 init8(float r, float g, float b)
{
  color8 c = { chan8(r), chan8(g), chan8(b) };
  return c;
}
/* gpu/colors.cu:23-35 */
static color8 add8(color8 a, color8 b)
{
  int r = a.r + b.r, g = a.g + b.g, bl = a.b + b.b;
  color8 c = { (unsigned char)(r > 255 ? 255 : r), (unsigned char)(g > 255 ? 255 : g),
               (unsigned char)(bl > 255 ? 255 : bl) };
  return c;
}
/* gpu/colors.cu:37-40 */
static color8 mul8(color8 a, float coef)
{
  return init8((float)a.r / 255 * coef, (float)a.g / 255 * coef, (float)a.b / 255 * coef);
}
/* gpu/colors.cu:42-47 */
static color8 mults8(color8 a, color8 b)
{
  return init8(((float)a.r / 255) * ((float)b.r / 255), ((float)a.g / 255) * ((float)b.g / 255),
               ((float)a.b / 255) * ((float)b.b / 255));
}

/* gpu/light.cu:12-28 */
static void specular8(color8 *acc, ray incident, ray hit, const struct or_object *obj)
{
  color8 k = init8(obj->ks.x, obj->ks.y, obj->ks.z);
  vec3 V = v_sub(incident.origin, hit.origin);
  vec3 R = v_sub(incident.direction,
                 v_scale(hit.direction, 2 * v_dot(hit.direction, incident.direction)));
  R = v_normalize(R);
  V = v_normalize(V);
  float d = v_dot(R, V);
  float m = d > 0.0f ? d : 0.0f; /* cufmax(d, 0.0) */
  float ls = (float)pow((double)m, (double)obj->ns);
  k = mul8(k, ls);
  *acc = add8(*acc, k);
}

/* gpu/light.cu:46-126 */
static color8 shade8(const struct or_scene *scene, const struct or_object *obj, ray hit,
                     struct tls_counts *cnt)
{
  color8 acc = init8(0, 0, 0);
  for (size_t i = 0; i < scene->light_count; i++)
  {
    const struct or_light *l = &scene->lights[i];
    if (l->type == OR_AMBIENT)
    {
      color8 t = mults8(init8(l->r, l->g, l->b), init8(obj->ka.x, obj->ka.y, obj->ka.z));
      acc = add8(acc, t);
    }
    else if (l->type == OR_DIRECTIONAL)
    {
      ray sr = { hit.origin, v_scale(l->v, -1) };
      if (shadowed(scene, sr, cnt))
        continue;
      vec3 L = v_scale(l->v, -1);
      color8 t = mults8(init8(l->r, l->g, l->b), init8(obj->kd.x, obj->kd.y, obj->kd.z));
      t = mul8(t, v_dot(L, hit.direction));
      ray inc = { v_add(hit.origin, v_scale(l->v, -10)), l->v };
      specular8(&t, inc, hit, obj);
      acc = add8(acc, t);
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
      if (shadowed(scene, sr, cnt))
        continue;
      color8 t = mults8(init8(l->r, l->g, l->b), init8(obj->kd.x, obj->kd.y, obj->kd.z));
      t = mul8(t, v_dot(L, N) * 1 / dist);
      ray inc = { v_add(hit.origin, v_scale(to_light, -10)), to_light };
      specular8(&t, inc, hit, obj);
      acc = add8(acc, t);
    }
  }
  return acc;
}

/* gpu/raytracer.cu:88-125: one high-resolution pixel (px, py) of the frame
 * whose camera (width, height) is already the upscaled one */
static color8 gpu_ray_pixel(const struct or_scene *scene, vec3 u, vec3 v, vec3 C, int px, int py,
                            struct tls_counts *cnt)
{
  const int W = scene->camera.width, H = scene->camera.height;
  vec3 ui = v_scale(u, (float)(px - W / 2));
  vec3 vj = v_scale(v, (float)(py - H / 2));
  vec3 point = v_add(v_add(C, ui), vj);
  ray r = { point, v_normalize(v_sub(scene->camera.position, point)) };
  float nr_ = 1;
  float r_rn = nr_;
  int max_bounce = 10;
  color8 color = init8(0, 0, 0);
  do
  {
    /* trace(), gpu/raytracer.cu:31-46 */
    color8 tmp = init8(0, 0, 0);
    cnt->closest++;
    int oi = -1;
    ray hit = oracle_collide(scene, r, &oi);
    if (!v_is_zero(hit.direction))
    {
      const struct or_object *obj = &scene->objects[oi];
      tmp = shade8(scene, obj, hit, cnt);
      if (obj->nr > 0)
        r = bounce(r, hit);
      r_rn = obj->nr;
    }
    else
      r_rn = 0;
    tmp = mul8(tmp, nr_);
    color = add8(color, tmp);
    nr_ *= r_rn;
  } while (nr_ > 0.01f && max_bounce-- > 0);
  return color;
}

/* gpu/raytracer.cu:48-85 + gpu/rt.cpp's row order: output pixel (row, col)
 * of the W x H image, RGBA8 */
static void render_pixel_gpu(const struct or_scene *hi, vec3 u, vec3 v, vec3 C, int W, int H,
                             int row, int col, unsigned char *out, struct tls_counts *cnt)
{
  const int px = W - 1 - col, py = H - 1 - row;
  float r = 0, g = 0, b = 0;
  for (int hy = 3 * py; hy < 3 * py + 3; ++hy)
    for (int hx = 3 * px; hx < 3 * px + 3; ++hx)
    {
      color8 c = gpu_ray_pixel(hi, u, v, C, hx, hy, cnt);
      r += (float)c.r;
      g += (float)c.g;
      b += (float)c.b;
    }
  float ali2 = 255.0f * 3.0f * 3.0f;
  color8 e = init8(r / ali2, g / ali2, b / ali2);
  out[0] = e.r;
  out[1] = e.g;
  out[2] = e.b;
  out[3] = 255;
}

struct job {
  const struct or_scene *scene;
  const int *pixels;
  size_t npix;
  float *out;
  vec3 u, v, C;
  atomic_size_t next;
  size_t chunk;  /* pixels per grab: small batches must still spread over every thread */
  pthread_mutex_t lock;
  struct or_counts total;
  unsigned char *out8;  /* gpu/rt mode: RGBA8 per pixel (scene = the 3x camera) */
  int W8, H8;           /* gpu/rt mode: output size */
};

static void *worker(void *arg)
{
  struct job *jb = arg;
  struct tls_counts cnt = { 0, 0, 0 };
  const int W = jb->scene->camera.width;
  for (;;)
  {
    size_t start = atomic_fetch_add(&jb->next, jb->chunk);
    if (start >= jb->npix)
      break;
    size_t stop = start + jb->chunk < jb->npix ? start + jb->chunk : jb->npix;
    for (size_t p = start; p < stop; p++)
    {
      int row, col;
      if (jb->pixels)
      {
        row = jb->pixels[2 * p];
        col = jb->pixels[2 * p + 1];
      }
      else
      {
        const int Wp = jb->out8 ? jb->W8 : W;
        row = (int)(p / (size_t)Wp);
        col = (int)(p % (size_t)Wp);
      }
      if (jb->out8)
      {
        render_pixel_gpu(jb->scene, jb->u, jb->v, jb->C, jb->W8, jb->H8, row, col, jb->out8 + 4 * p,
                         &cnt);
        continue;
      }
      color c = render_pixel(jb->scene, jb->u, jb->v, jb->C, row, col, &cnt);
      jb->out[3 * p + 0] = c.r;
      jb->out[3 * p + 1] = c.g;
      jb->out[3 * p + 2] = c.b;
    }
  }
  pthread_mutex_lock(&jb->lock);
  jb->total.closest += cnt.closest;
  jb->total.shadow += cnt.shadow;
  if (cnt.max_depth > jb->total.max_depth)
    jb->total.max_depth = cnt.max_depth;
  pthread_mutex_unlock(&jb->lock);
  return NULL;
}

static int run_job(struct job *jb, int nthreads, struct or_counts *counts);

int oracle_render(const struct or_scene *scene, const int *pixels, size_t npix, int nthreads,
                  float *out, struct or_counts *counts)
{
  if (!scene || !out)
    return -1;
  struct job jb;
  memset(&jb, 0, sizeof jb);
  jb.scene = scene;
  jb.pixels = pixels;
  jb.npix = npix;
  jb.out = out;
  oracle_camera_frame(scene, &jb.u, &jb.v, &jb.C);
  return run_job(&jb, nthreads, counts);
}

int oracle_render_gpu(const struct or_scene *scene, const int *pixels, size_t npix, int nthreads,
                      unsigned char *out, struct or_counts *counts)
{
  if (!scene || !out)
    return -1;
  /* gpu/rt.cpp:72-83: the camera's width and height times 3, then the frame
   * (L and C) of that camera */
  struct or_scene hi = *scene;
  hi.camera.width = 3 * scene->camera.width;
  hi.camera.height = 3 * scene->camera.height;
  struct job jb;
  memset(&jb, 0, sizeof jb);
  jb.scene = &hi;
  jb.pixels = pixels;
  jb.npix = npix;
  jb.out8 = out;
  jb.W8 = scene->camera.width;
  jb.H8 = scene->camera.height;
  oracle_camera_frame(&hi, &jb.u, &jb.v, &jb.C);
  return run_job(&jb, nthreads, counts);
}

/* Runs a prepared job on nthreads threads (<= 0: all online CPUs). */
static int run_job(struct job *jb, int nthreads, struct or_counts *counts)
{
  if (nthreads <= 0)
    nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (nthreads < 1)
    nthreads = 1;
  atomic_init(&jb->next, 0);
  jb->chunk = jb->npix / ((size_t)nthreads * 4);
  if (jb->chunk < 1)
    jb->chunk = 1;
  if (jb->chunk > 16)
    jb->chunk = 16;
  pthread_mutex_init(&jb->lock, NULL);
  pthread_t *tid = calloc((size_t)nthreads, sizeof *tid);
  if (!tid)
    return -1;
  for (int t = 0; t < nthreads; t++)
    pthread_create(&tid[t], NULL, worker, jb);
  for (int t = 0; t < nthreads; t++)
    pthread_join(tid[t], NULL);
  free(tid);
  pthread_mutex_destroy(&jb->lock);
  if (counts)
    *counts = jb->total;
  return 0;
}

/* ---- loader: cpu/parser.c:4-116, cpu/parse_obj.c:3-92, cpu/stack.c ---- */

/* The reference's vertex "stack" is a LIFO linked list (cpu/stack.c:23-47);
 * create_triangle pops three vertices and three normals per triangle
 * (cpu/parse_obj.c:29-40), so triangle t, vertex k is file line N-1-3t-k.
 * A growable array popped from the end is the same LIFO. */
struct vstack { vec3 *data; size_t size, cap; };

static int vpush(struct vstack *s, vec3 x)
{
  if (s->size == s->cap)
  {
    size_t nc = s->cap ? 2 * s->cap : 64;
    vec3 *nd = realloc(s->data, nc * sizeof *nd);
    if (!nd)
      return -1;
    s->data = nd;
    s->cap = nc;
  }
  s->data[s->size++] = x;
  return 0;
}

static int read_vec(FILE *f, vec3 *x) { return fscanf(f, "%f %f %f", &x->x, &x->y, &x->z) == 3 ? 0 : -2; }

/* cpu/parse_obj.c:42-92 */
static int parse_object(FILE *f, struct or_object *obj)
{
  memset(obj, 0, sizeof *obj);
  obj->ni = 1; /* cpu/parse_obj.c:3-20 defaults */
  obj->d = 1;
  unsigned declared = 0;
  if (fscanf(f, "%u", &declared) != 1)
    return -2;
  struct vstack vs = { 0 }, ns = { 0 };
  unsigned seen = 0;
  char tok[256];
  int rc = 0;
  while (seen < declared * 2 && fscanf(f, "%255s", tok) == 1)
  {
    if (!strcmp(tok, "Ka")) rc = read_vec(f, &obj->ka);
    else if (!strcmp(tok, "Kd")) rc = read_vec(f, &obj->kd);
    else if (!strcmp(tok, "Ks")) rc = read_vec(f, &obj->ks);
    else if (!strcmp(tok, "Ns")) rc = fscanf(f, "%f", &obj->ns) == 1 ? 0 : -2;
    else if (!strcmp(tok, "Ni")) rc = fscanf(f, "%f", &obj->ni) == 1 ? 0 : -2;
    else if (!strcmp(tok, "Nr")) rc = fscanf(f, "%f", &obj->nr) == 1 ? 0 : -2;
    else if (!strcmp(tok, "d")) rc = fscanf(f, "%f", &obj->d) == 1 ? 0 : -2;
    else if (!strcmp(tok, "v") || !strcmp(tok, "vn"))
    {
      vec3 x;
      seen++;
      rc = read_vec(f, &x);
      if (!rc)
        rc = vpush(tok[1] ? &ns : &vs, x);
    }
    else
      rc = -2;
    if (rc)
      break;
  }
  if (!rc && (vs.size % 3 != 0 || ns.size < vs.size))
    rc = -2; /* the reference would dereference an empty stack here */
  if (!rc)
  {
    size_t ntri = vs.size / 3;
    obj->triangles = malloc((ntri ? ntri : 1) * sizeof *obj->triangles);
    if (!obj->triangles)
      rc = -1;
    for (size_t t = 0; !rc && t < ntri; t++)
      for (int k = 0; k < 3; k++)
      {
        obj->triangles[t].vertex[k] = vs.data[--vs.size];
        obj->triangles[t].normal[k] = ns.data[--ns.size];
      }
    obj->triangle_count = declared / 3;
  }
  free(vs.data);
  free(ns.data);
  return rc;
}

static int push_light(struct or_scene *s, struct or_light l)
{
  struct or_light *nl = realloc(s->lights, (s->light_count + 1) * sizeof *nl);
  if (!nl)
    return -1;
  s->lights = nl;
  s->lights[s->light_count++] = l;
  return 0;
}

int oracle_load_svati(const char *path, struct or_scene **out)
{
  FILE *f = fopen(path, "r");
  if (!f)
    return -1;
  struct or_scene *s = calloc(1, sizeof *s);
  if (!s)
  {
    fclose(f);
    return -1;
  }
  char tok[256];
  int rc = 0;
  while (!rc && fscanf(f, "%255s", tok) == 1)
  {
    struct or_light l;
    memset(&l, 0, sizeof l);
    if (!strcmp(tok, "camera"))
    {
      struct or_camera *c = &s->camera;
      rc = fscanf(f, "%d %d %f %f %f %f %f %f %f %f %f %f", &c->width, &c->height,
                  &c->position.x, &c->position.y, &c->position.z, &c->u.x, &c->u.y, &c->u.z,
                  &c->v.x, &c->v.y, &c->v.z, &c->fov) == 12 ? 0 : -2;
    }
    else if (!strcmp(tok, "a_light"))
    {
      l.type = OR_AMBIENT;
      rc = fscanf(f, "%f %f %f", &l.r, &l.g, &l.b) == 3 ? push_light(s, l) : -2;
    }
    else if (!strcmp(tok, "d_light") || !strcmp(tok, "p_light"))
    {
      l.type = tok[0] == 'd' ? OR_DIRECTIONAL : OR_POINT;
      rc = fscanf(f, "%f %f %f %f %f %f", &l.r, &l.g, &l.b, &l.v.x, &l.v.y, &l.v.z) == 6
             ? push_light(s, l) : -2;
    }
    else if (!strcmp(tok, "object"))
    {
      struct or_object *no = realloc(s->objects, (s->object_count + 1) * sizeof *no);
      if (!no)
        rc = -1;
      else
      {
        s->objects = no;
        rc = parse_object(f, &s->objects[s->object_count]);
        if (!rc)
          s->object_count++;
      }
    }
    else if (!strcmp(tok, "#"))
    {
      if (fscanf(f, " %*[^\n]") < 0)
        break;
    }
    else
      rc = -2;
  }
  fclose(f);
  if (rc)
  {
    oracle_free_scene(s);
    return rc;
  }
  *out = s;
  return 0;
}

void oracle_free_scene(struct or_scene *s)
{
  if (!s)
    return;
  for (size_t i = 0; i < s->object_count; i++)
    free(s->objects[i].triangles);
  free(s->objects);
  free(s->lights);
  free(s);
}
