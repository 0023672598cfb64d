/*
 * vecmath.c -- host twins of the reference vector algebra
 * (cpu/vector3.c:3-47, cpu/vector3-extern.c:5-23), used for the camera frame
 * and for pre-normalising vertex normals.  Compiled with -ffp-contract=off so
 * every value is bit-identical to the reference and to the device twins in
 * csrc/rt_device.h.
 */
#include <math.h>

#include "rt_internal.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

rt_vec3 rt_v_sub(rt_vec3 a, rt_vec3 b) { rt_vec3 r = { a.x - b.x, a.y - b.y, a.z - b.z }; return r; }
rt_vec3 rt_v_add(rt_vec3 a, rt_vec3 b) { rt_vec3 r = { a.x + b.x, a.y + b.y, a.z + b.z }; return r; }
rt_vec3 rt_v_cross(rt_vec3 a, rt_vec3 b)
{
  rt_vec3 r = { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x };
  return r;
}
rt_vec3 rt_v_scale(rt_vec3 a, float s) { rt_vec3 r = { s * a.x, s * a.y, s * a.z }; return r; }
float rt_v_length(rt_vec3 a) { return (float)sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
rt_vec3 rt_v_normalize(rt_vec3 a)
{
  float len = rt_v_length(a);
  rt_vec3 r = { a.x / len, a.y / len, a.z / len };
  return r;
}

/* cpu/raytracer.c:82-86, any positive size (the compatibility mode's 3x
 * frame: gpu/rt renders odd sizes, gpu/raytracer.cu:97-103) */
int rt_frame_from_camera_any(const rt_camera *cam, rt_frame *out)
{
  if (!cam || !out)
    return rt_set_error(RT_EINVAL, "null argument");
  if (cam->width <= 0 || cam->height <= 0)
    return rt_set_error(RT_EINVAL, "camera size %dx%d", cam->width, cam->height);
  out->u = rt_v_normalize(cam->u);
  out->v = rt_v_normalize(cam->v);
  rt_vec3 w = rt_v_cross(out->u, out->v);
  float L = cam->width / (2 * tan(cam->fov * M_PI / 360));
  out->C = rt_v_add(cam->position, rt_v_scale(w, L));
  out->position = cam->position;
  out->width = cam->width;
  out->height = cam->height;
  return RT_OK;
}

/* cpu/rt's frame: even sizes only.  cpu/raytracer.c:89-91 writes pixel
 * (i + W/2, j + H/2) for i in (-W/2, W/2], j in (-H/2, H/2] and :128-134 prints
 * j * W + i for i in [1, W], j in [1, H]: the two cover the same slots only
 * when W and H are even -- for odd sizes cpu/rt prints uninitialised stack
 * memory, so there is no output to match and the size is refused. */
int rt_frame_from_camera(const rt_camera *cam, rt_frame *out)
{
  if (cam && ((cam->width & 1) || (cam->height & 1)) && cam->width > 0 && cam->height > 0)
    return rt_set_error(RT_EINVAL, "camera size %dx%d: cpu/rt renders even sizes only", cam->width,
                        cam->height);
  return rt_frame_from_camera_any(cam, out);
}
