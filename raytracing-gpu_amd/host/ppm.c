/*
 * ppm.c -- P3 writer, byte-identical to the reference output path:
 * open_output() writes "P3\n%d %d\n255\n" (cpu/printer.c:3-10), then the print
 * loop (cpu/raytracer.c:128-134) emits every pixel as "%d %d %d " with C's
 * float->int truncation (cpu/printer.c:12-18) and no newline at all.
 * Formatting goes to one buffer in parallel-friendly chunks instead of one
 * fprintf per pixel.
 */
#include <errno.h>
#include <pthread.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"
#include "rt_lex.h"

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

typedef struct {
  const float *rgb;
  size_t s, e;   /* pixel range */
  char *buf;     /* >= (e - s) * 3 * 12 bytes */
  size_t len;
} fmt_task;

static void *fmt_chunk(void *arg)
{
  fmt_task *t = arg;
  char *p = t->buf;
  for (size_t i = t->s; i < t->e; i++)
    for (int c = 0; c < 3; c++)
    {
      p = put_int(p, trunc_int(t->rgb[3 * i + (size_t)c]));
      *p++ = ' ';
    }
  t->len = (size_t)(p - t->buf);
  return NULL;
}

/* Rounds of one 2^16-pixel chunk per host thread, formatted by the host threads in
 * parallel and written in pixel order, so the bytes are those of the serial
 * loop. */
int rt_ppm_write(const char *path, int width, int height, const float *rgb)
{
  if (!path || !rgb || width <= 0 || height <= 0)
    return rt_set_error(RT_EINVAL, "rt_ppm_write: bad argument");
  FILE *f = fopen(path, "w+");
  if (!f)
    return rt_set_error(RT_EIO, "%s", strerror(errno));
  fprintf(f, "P3\n%d %d\n255\n", width, height);
  const size_t chunk_px = 1 << 16;
  size_t npx = (size_t)width * (size_t)height;
  size_t nchunk = (npx + chunk_px - 1) / chunk_px;
  int nt = rt_host_threads();
  size_t per_round = nchunk < (size_t)nt ? nchunk : (size_t)nt; /* nt <= 64 */
  char *buf = malloc(per_round * chunk_px * 3 * 12);
  if (!buf)
  {
    fclose(f);
    return rt_set_error(RT_ENOMEM, "ppm buffer");
  }
  int rc = RT_OK;
  fmt_task task[64];
  pthread_t tid[64];
  for (size_t c0 = 0; c0 < nchunk && !rc; c0 += per_round)
  {
    size_t m = nchunk - c0 < per_round ? nchunk - c0 : per_round;
    for (size_t k = 0; k < m; k++)
    {
      size_t s = (c0 + k) * chunk_px;
      task[k] = (fmt_task){ rgb, s, s + chunk_px < npx ? s + chunk_px : npx,
                            buf + k * chunk_px * 3 * 12, 0 };
    }
    /* one thread per chunk of the round (m <= nt) */
    if (m < 2)
      for (size_t k = 0; k < m; k++)
        fmt_chunk(&task[k]);
    else
    {
      int started[64] = { 0 };
      for (size_t k = 0; k < m; k++)
        started[k] = pthread_create(&tid[k], NULL, fmt_chunk, &task[k]) == 0;
      for (size_t k = 0; k < m; k++)
        if (started[k])
          pthread_join(tid[k], NULL);
        else
          fmt_chunk(&task[k]);
    }
    for (size_t k = 0; k < m && !rc; k++)
      if (fwrite(task[k].buf, 1, task[k].len, f) != task[k].len)
        rc = rt_set_error(RT_EIO, "%s: short write", path);
  }
  free(buf);
  if (fclose(f) != 0 && !rc)
    rc = rt_set_error(RT_EIO, "%s: close failed", path);
  return rc;
}
