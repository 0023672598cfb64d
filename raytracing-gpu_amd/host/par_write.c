/*
 * par_write.c -- parallel text formatting for the scene writers
 * (rt_scene_write_svati / _obj), same scheme as rt_ppm_write: the file is a
 * sequence of "units" (an object's header block, then one unit per line),
 * cut into chunks of 2^16 units; the host threads format one chunk each
 * with snprintf -- the same conversions the serial fprintf loop made -- and
 * the chunks are written in order, so the bytes are identical to a serial
 * writer's.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "rt_internal.h"
#include "rt_lex.h"
#include "rt_par_write.h"

typedef struct {
  const void *ctx;
  const size_t *first; /* first[o] = global index of object o's first unit; first[nobj] = total */
  size_t nobj;
  rt_unit_fmt fmt;
  size_t u0, u1;       /* chunk [u0, u1) */
  char *buf;
  size_t cap, len;
  int oom;
} chunk_task;

static size_t object_of(const size_t *first, size_t nobj, size_t u)
{
  size_t lo = 0, hi = nobj; /* largest o with first[o] <= u */
  while (hi - lo > 1)
  {
    size_t mid = lo + (hi - lo) / 2;
    if (first[mid] <= u)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

static void *fmt_units(void *arg)
{
  chunk_task *t = arg;
  size_t o = object_of(t->first, t->nobj, t->u0);
  t->len = 0;
  for (size_t u = t->u0; u < t->u1; u++)
  {
    while (u >= t->first[o + 1])
      o++;
    if (t->cap - t->len < RT_UNIT_MAX)
    {
      size_t nc = t->cap ? 2 * t->cap : (size_t)1 << 20;
      char *nb = realloc(t->buf, nc);
      if (!nb)
      {
        t->oom = 1;
        return NULL;
      }
      t->buf = nb;
      t->cap = nc;
    }
    t->len += t->fmt(t->ctx, o, u - t->first[o], t->buf + t->len);
  }
  return NULL;
}

int rt_par_write(FILE *f, const void *ctx, size_t nobj, const size_t *units, rt_unit_fmt fmt)
{
  size_t *first = malloc((nobj + 1) * sizeof *first);
  if (!first)
    return rt_set_error(RT_ENOMEM, "writer index");
  first[0] = 0;
  for (size_t o = 0; o < nobj; o++)
    first[o + 1] = first[o] + units[o];
  const size_t total = first[nobj], chunk = (size_t)1 << 16;
  const size_t nchunk = (total + chunk - 1) / chunk;
  int nt = rt_host_threads();
  chunk_task task[64];
  pthread_t tid[64];
  memset(task, 0, sizeof task);
  int rc = RT_OK;
  for (size_t c0 = 0; c0 < nchunk && !rc; c0 += (size_t)nt)
  {
    size_t m = nchunk - c0 < (size_t)nt ? nchunk - c0 : (size_t)nt;
    for (size_t k = 0; k < m; k++)
    {
      chunk_task *t = &task[k];
      t->ctx = ctx;
      t->first = first;
      t->nobj = nobj;
      t->fmt = fmt;
      t->u0 = (c0 + k) * chunk;
      t->u1 = t->u0 + chunk < total ? t->u0 + chunk : total;
    }
    int started[64] = { 0 };
    for (size_t k = 1; k < m; k++)
      started[k] = pthread_create(&tid[k], NULL, fmt_units, &task[k]) == 0;
    fmt_units(&task[0]);
    for (size_t k = 1; k < m; k++)
      if (started[k])
        pthread_join(tid[k], NULL);
      else
        fmt_units(&task[k]);
    for (size_t k = 0; k < m && !rc; k++)
      if (task[k].oom)
        rc = rt_set_error(RT_ENOMEM, "writer buffer");
      else if (fwrite(task[k].buf, 1, task[k].len, f) != task[k].len)
        rc = rt_set_error(RT_EIO, "short write");
  }
  for (int k = 0; k < nt && k < 64; k++)
    free(task[k].buf);
  free(first);
  return rc;
}
