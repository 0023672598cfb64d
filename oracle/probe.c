/*
 * probe.c -- TEST INFRASTRUCTURE ONLY (oracle side; never linked into the product).
 *
 * Link-time companion for the *reference* cpu/rt objects compiled by
 * oracle/Makefile into oracle/_ref/rt_probe.  It is our own code; the
 * reference sources are compiled unmodified from /root/reference/cpu.
 *
 *  - replaces cpu/printer.c (open_output / print_color, /root/reference/cpu/printer.c:3-18)
 *    so the float framebuffer is dumped bit-exactly instead of truncated to
 *    P3 integers.  The dump is a text header "RTF32 <W> <H>\n" followed by
 *    W*H*3 little-endian float32 in print (= PPM) order, i.e. exactly the
 *    order cpu/raytracer.c:128-134 visits the framebuffer.
 *  - wraps collide / collide_dist (/root/reference/cpu/hit.c:72,93) with
 *    -Wl,--wrap to count closest-hit and shadow queries.
 *  - when RT_PROBE_PPM=<path> is set it also writes the exact P3 text the
 *    unmodified printer.c would have written, so PPM byte-identity can be
 *    pinned without a second render.
 */
#include <err.h>
#include <errno.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "colors.h"
#include "hit.h"

static FILE *ppm_out;

FILE *open_output(const char *output, int width, int height)
{
  FILE *out = fopen(output, "w+");
  if (!out)
    errx(1, "%s\n", strerror(errno));
  fprintf(out, "RTF32 %d %d\n", width, height);
  const char *ppm = getenv("RT_PROBE_PPM");
  if (ppm && *ppm)
  {
    ppm_out = fopen(ppm, "w+");
    if (!ppm_out)
      errx(1, "%s\n", strerror(errno));
    fprintf(ppm_out, "P3\n%d %d\n255\n", width, height);
  }
  return out;
}

void print_color(struct color color, FILE *output)
{
  float rgb[3] = { color.r, color.g, color.b };
  if (fwrite(rgb, sizeof rgb, 1, output) != 1)
    errx(1, "short write");
  if (ppm_out)
  {
    int r = color.r;
    int g = color.g;
    int b = color.b;
    fprintf(ppm_out, "%d %d %d ", r, g, b);
  }
}

static atomic_ulong n_collide;
static atomic_ulong n_shadow;

struct ray __real_collide(struct scene scene, struct ray ray, struct object *hit);
float __real_collide_dist(struct scene scene, struct ray ray);

struct ray __wrap_collide(struct scene scene, struct ray ray, struct object *hit)
{
  atomic_fetch_add(&n_collide, 1);
  return __real_collide(scene, ray, hit);
}

float __wrap_collide_dist(struct scene scene, struct ray ray)
{
  atomic_fetch_add(&n_shadow, 1);
  return __real_collide_dist(scene, ray);
}

__attribute__((destructor)) static void report(void)
{
  if (ppm_out)
    fclose(ppm_out);
  fprintf(stderr, "closest_hit_queries=%lu shadow_queries=%lu\n",
          (unsigned long)atomic_load(&n_collide),
          (unsigned long)atomic_load(&n_shadow));
}
