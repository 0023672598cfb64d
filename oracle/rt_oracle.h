/*
 * rt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference cpu/rt hot path, used as the parity
 * checker by tests/ and as the CPU baseline by bench.py.  Nothing in the
 * product (raytracing-gpu_amd/, include/) may link or call this.
 *
 * Parity is pinned by tests/golden/ (framebuffers and query counts produced
 * by the reference's own cpu/ sources compiled here, oracle/_ref/rt_probe).
 *
 * The scene structs below have exactly the layout of
 * /root/reference/cpu/headers/scene.h:7-55 (and of include/rt_scene.h),
 * so a scene built by the product loader can be handed to the oracle.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>

struct or_vec3 { float x, y, z; };
struct or_triangle { struct or_vec3 vertex[3]; struct or_vec3 normal[3]; };
struct or_object {
  struct or_triangle *triangles;
  unsigned triangle_count;
  struct or_vec3 ka, kd, ks;
  float ns, ni, nr, d;
};
enum or_light_type { OR_AMBIENT, OR_DIRECTIONAL, OR_POINT, OR_SPECULAR };
struct or_light { enum or_light_type type; float r, g, b; struct or_vec3 v; };
struct or_camera { int width, height; struct or_vec3 position, u, v; float fov; };
struct or_scene {
  struct or_object *objects;
  size_t object_count;
  struct or_light *lights;
  size_t light_count;
  struct or_camera camera;
};
struct or_color { float r, g, b; };
struct or_ray { struct or_vec3 origin, direction; };

/* Query counters: closest = collide() calls,
 * shadow = collide_dist() calls; max_depth = deepest trace() level reached. */
struct or_counts { unsigned long long closest, shadow, max_depth; };

/* cpu/parser.c:62-116 + cpu/parse_obj.c:42-92 + cpu/stack.c.  Returns 0 on
 * success, -1 on I/O error, -2 on a parse error (the reference errx()es). */
int oracle_load_svati(const char *path, struct or_scene **out);
void oracle_free_scene(struct or_scene *scene);

/* cpu/raytracer.c:82-86 */
void oracle_camera_frame(const struct or_scene *scene, struct or_vec3 *u,
                         struct or_vec3 *v, struct or_vec3 *C);

/* Render the listed PPM pixels (pixels[2k] = row, pixels[2k+1] = col; NULL
 * with npix = W*H renders the whole frame in PPM order).  out receives
 * npix*3 floats in list order.  nthreads <= 0 uses all online CPUs. */
int oracle_render(const struct or_scene *scene, const int *pixels, size_t npix,
                  int nthreads, float *out, struct or_counts *counts);

/* gpu/rt compatibility mode (gpu/raytracer.cu:31-129, gpu/light.cu,
 * gpu/colors.cu, gpu/rt.cpp:56-97): output pixels (row, col) of the
 * camera's W x H image (pixels as above; NULL = whole image, row-major in
 * gpu/rt's PNG order), each the 3x3 downscale of the 3x frame; out receives
 * npix*4 bytes (RGBA8, alpha 255).  counts: queries of the 3x rays. */
int oracle_render_gpu(const struct or_scene *scene, const int *pixels, size_t npix,
                      int nthreads, unsigned char *out, struct or_counts *counts);

/* Camera samples (cpu/raytracer.c:50-61) against one triangle each: for
 * i < n, the PPM pixels [row0, row0 + rows) x [col0, col0 + cols) (rects[4i ..
 * 4i + 3]) against tris[i]: out[2i] = samples cpu/hit.c:15-44 accepts,
 * out[2i + 1] = samples passing its a, u, v tests (t not checked). */
void oracle_camera_tri_accepts(const struct or_scene *scene, const struct or_triangle *tris,
                               const int *rects, size_t n, unsigned long long *out);

/* The same for gpu/rt's camera rays (gpu/raytracer.cu:97-103): one ray per
 * pixel (px, py) of the 3x frame; rects[4i .. 4i + 3] = (py0, px0, rows, cols). */
void oracle_camera_tri_accepts_gpu(const struct or_scene *scene, const struct or_triangle *tris,
                                   const int *rects, size_t n, unsigned long long *out);

/* Single-function entry points, for unit known-answer tests. */
struct or_color oracle_init_color(float r, float g, float b);
struct or_color oracle_color_add(struct or_color a, struct or_color b);
struct or_color oracle_color_mul(struct or_color a, float coef);
struct or_color oracle_color_mul2(struct or_color a, struct or_color b);
struct or_ray oracle_collide(const struct or_scene *scene, struct or_ray ray,
                             int *object_index);
float oracle_collide_dist(const struct or_scene *scene, struct or_ray ray);
struct or_color oracle_apply_light(const struct or_scene *scene, int object_index,
                                   struct or_ray point);

#endif
