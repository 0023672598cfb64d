/*
 * ppm.c -- P3 writer, byte-identical to the reference output path:
 * open_output() writes "P3\n%d %d\n255\n" (cpu/printer.c:3-10), then the print
 * loop (cpu/raytracer.c:128-134) emits every pixel as "%d %d %d " with C's
 * float->int truncation (cpu/printer.c:12-18) and no newline at all.
 * Formatting goes to one buffer in parallel-friendly chunks instead of one
 * fprintf per pixel.
 */
#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"

/* x86-64 cvttss2si: truncation, and INT_MIN for NaN / out of range. */
static int trunc_int(float x)
{
  if (!(x > -2147483904.0f && x < 2147483648.0f))
    return INT_MIN;
  return (int)x;
}

static char *put_int(char *p, int v)
{
  if (v >= 0 && v < 1000)
  {
    if (v >= 100)
      *p++ = (char)('0' + v / 100);
    if (v >= 10)
      *p++ = (char)('0' + (v / 10) % 10);
    *p++ = (char)('0' + v % 10);
    return p;
  }
  return p + sprintf(p, "%d", v);
}

int rt_ppm_write(const char *path, int width, int height, const float *rgb)
{
  if (!path || !rgb || width <= 0 || height <= 0)
    return rt_set_error(RT_EINVAL, "rt_ppm_write: bad argument");
  FILE *f = fopen(path, "w+");
  if (!f)
    return rt_set_error(RT_EIO, "%s", strerror(errno));
  fprintf(f, "P3\n%d %d\n255\n", width, height);
  const size_t chunk_px = 1 << 16;
  char *buf = malloc(chunk_px * 3 * 12);
  if (!buf)
  {
    fclose(f);
    return rt_set_error(RT_ENOMEM, "ppm buffer");
  }
  size_t npx = (size_t)width * (size_t)height;
  int rc = RT_OK;
  for (size_t s = 0; s < npx && !rc; s += chunk_px)
  {
    size_t e = s + chunk_px < npx ? s + chunk_px : npx;
    char *p = buf;
    for (size_t i = s; i < e; i++)
      for (int c = 0; c < 3; c++)
      {
        p = put_int(p, trunc_int(rgb[3 * i + (size_t)c]));
        *p++ = ' ';
      }
    if (fwrite(buf, 1, (size_t)(p - buf), f) != (size_t)(p - buf))
      rc = rt_set_error(RT_EIO, "%s: short write", path);
  }
  free(buf);
  if (fclose(f) != 0 && !rc)
    rc = rt_set_error(RT_EIO, "%s: close failed", path);
  return rc;
}
