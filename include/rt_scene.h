/*
 * rt_scene.h -- scene model and loaders of the MI355X raytracer (C ABI).
 *
 * The structs are layout-identical to the reference's scene model
 * (/root/reference/cpu/headers/scene.h:7-55, vector3.h:4-8, colors.h:4-8,
 * ray.h:5-8) so a caller that already holds a `struct scene` from the
 * reference parser can pass it here unchanged.
 *
 * Error convention for every int-returning entry point in this library:
 * 0 = success, negative = RT_E* code (rt_strerror() names it).  The library
 * never exits the process; the CLI maps errors to errx(1, ...) exactly like
 * the reference (cpu/parser.c:70-71,110-111, cpu/printer.c:6-7).
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RT_OK = 0,
  RT_EINVAL = -1,    /* bad argument / unsupported configuration         */
  RT_EIO = -2,       /* file could not be opened / read / written        */
  RT_EPARSE = -3,    /* malformed .svati / .obj                          */
  RT_ENOMEM = -4,    /* host allocation failed                           */
  RT_EHIP = -5,      /* HIP runtime error (device alloc, launch, copy)   */
  RT_ENODEV = -6,    /* no usable gfx950 device                          */
  RT_EDEPTH = -7,    /* a path needed more than RT_MAX_BOUNCES closest-hit queries
                      * (cpu/rt recursion without end: Nr >= 1 mirrors), or a
                      * traversal stack overflowed                       */
  RT_ERCCL = -8,     /* RCCL collective failed                           */
  RT_EZERONORMAL = -9, /* a closest hit had an exactly zero interpolated normal, or
                       * a shadow ray hit an object that can have one: cpu/hit.c:79,99
                       * skips such an object, which is not reproduced     */
  RT_EHITBUF = -10,  /* the frame made more hits than the hit-record buffer held,
                      * or more camera candidate-list entries than the
                      * asynchronous list build had sized its buffers for: the
                      * image is incomplete; the buffer has been grown to the
                      * frame's need, render the frame again              */
  RT_EINEXACT = -11  /* rendered with a tuning knob that gives up the cpu/rt parity
                      * guarantee (rt_hip_set_exact_camera(0), a camera bound scale
                      * < 1, a culling slack below the default): image written,
                      * parity not guaranteed                             */
};

const char *rt_strerror(int code);
/* Detail message of the last error raised on this thread (parse position,
 * HIP error string, ...); never NULL. */
const char *rt_last_error(void);

typedef struct rt_vec3 { float x, y, z; } rt_vec3;                  /* vector3.h:4-8 */
typedef struct rt_color { float r, g, b; } rt_color;                /* colors.h:4-8  */
typedef struct rt_ray { rt_vec3 origin, direction; } rt_ray;        /* ray.h:5-8     */

typedef struct rt_triangle {                                         /* scene.h:7-10  */
  rt_vec3 vertex[3];
  rt_vec3 normal[3];
} rt_triangle;

typedef struct rt_object {                                           /* scene.h:12-22 */
  rt_triangle *triangles;
  unsigned triangle_count;
  rt_vec3 ka, kd, ks;
  float ns, ni, nr, d;
} rt_object;

typedef enum rt_light_type {                                         /* scene.h:24-29 */
  RT_AMBIENT, RT_DIRECTIONAL, RT_POINT, RT_SPECULAR
} rt_light_type;

typedef struct rt_light {                                            /* scene.h:31-38 */
  rt_light_type type;
  float r, g, b;
  rt_vec3 v;
} rt_light;

typedef struct rt_camera {                                           /* scene.h:40-47 */
  int width, height;
  rt_vec3 position, u, v;
  float fov;
} rt_camera;

typedef struct rt_scene {                                            /* scene.h:49-55 */
  rt_object *objects;
  size_t object_count;
  rt_light *lights;
  size_t light_count;
  rt_camera camera;
} rt_scene;

/* .svati loader; replaces parser() (cpu/headers/parser.h:18,
 * cpu/parser.c:62-116 + cpu/parse_obj.c:42-92).  Same grammar, same
 * LIFO triangle order (triangle t, vertex k = object's file line N-1-3t-k),
 * same material defaults.  Extension (absent from the reference): the
 * directive `objfile <path>` appends the objects of a Wavefront .obj
 * (relative paths resolve against the .svati's directory). */
int rt_scene_load_svati(const char *path, rt_scene **out);

/* Wavefront .obj loader (new; the reference has none).  Each `o`/`g`/
 * `usemtl` group becomes one object; faces are fan-triangulated; face
 * order and corner order are kept (triangle t = t-th triangle of the
 * group, vertex k = k-th corner), i.e. the triangles the LIFO-compensated
 * .svati written by rt_scene_write_svati() yields.  Camera and lights are
 * not part of .obj; they come from the .svati that references it, or
 * default to zero. */
int rt_scene_load_obj(const char *path, rt_scene **out);
int rt_scene_append_obj(rt_scene *scene, const char *path);

/* Writes a .svati that the reference parser reads back to exactly this
 * scene (vertices emitted in reverse so its LIFO stack restores order). */
int rt_scene_write_svati(const rt_scene *scene, const char *path);
/* Writes the objects as a Wavefront .obj (+ no .mtl: materials are
 * written as comments `#rt Ka ...` the .obj loader understands). */
int rt_scene_write_obj(const rt_scene *scene, const char *path);

/* Deterministic synthetic scene: a grid of
 * gx*gy smooth UV spheres of about `tris_per_sphere` triangles each (the
 * 2*slices*(stacks-1) decomposition nearest to it with slices/stacks in
 * [1.5, 2.2], i.e. near-square quads) plus a ground quad, splitmix64(seed)
 * jitter; camera set to width x height.  C5 = 32 x 32 spheres of 9776
 * triangles (53 stacks x 94 slices) = 10,010,626 triangles. */
int rt_scene_synthetic(unsigned gx, unsigned gy, unsigned tris_per_sphere, unsigned long long seed,
                       int width, int height, rt_scene **out);
/* The same field with an explicit stacks x slices tessellation (round 1's
 * C5 was 258 x 19: 27:1 sliver triangles). */
int rt_scene_synthetic_uv(unsigned gx, unsigned gy, unsigned stacks, unsigned slices,
                          unsigned long long seed, int width, int height, rt_scene **out);

size_t rt_scene_triangle_count(const rt_scene *scene);
void rt_scene_free(rt_scene *scene);

/* P3 writer; byte-identical to cpu/printer.c:3-18 driven by the print loop
 * cpu/raytracer.c:128-134 (one line of "%d %d %d " after the header, int
 * truncation).  rgb = width*height*3 floats in PPM order. */
int rt_ppm_write(const char *path, int width, int height, const float *rgb);
/* 8-bit RGBA PNG, rows top down (gpu/rt.cpp:14-54 writes the same image
 * through libpng: colour type RGBA, bit depth 8, no interlace).  zlib
 * deflate, filter 0 on every row. */
int rt_png_write_rgba(const char *path, int width, int height, const unsigned char *rgba);

#ifdef __cplusplus
}
#endif
#endif
