/*
 * lex_prescan.c -- parallel pre-parse of vertex lines for the .svati / .obj
 * loaders.
 *
 * The reference parses every number with fscanf("%f") from one FILE
 * (cpu/parse_obj.c:25, called per `v` / `vn` token from cpu/parse_obj.c:68-76),
 * one token at a time.  A 10M-triangle scene is 60 M such lines (~1.8 GB of
 * text), so the float conversions dominate loading.  Here the file (already
 * in memory, rt_lex) is cut into one chunk per host thread at line starts;
 * every thread records, for each line whose first token is `v` or `vn`, the
 * token's offset, the three floats and the cursor after them -- converted
 * with exactly the calls the serial scanner makes (skip blanks, strtof, three
 * times), so the values and the end cursor are the same bytes-for-bytes.
 *
 * The serial grammar pass then consumes the table: when it meets a `v`/`vn`
 * token at offset o it takes the entry recorded for o (if any) and jumps to
 * its end.  Entries that the grammar never reaches as tokens (a `v` line
 * swallowed by a `#` comment, say) are skipped; tokens the prescan did not
 * record (a `v` in mid-line) fall back to the serial conversion.  So the
 * result is identical to the serial parse for every input, not just for
 * well-formed ones.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "rt_internal.h"
#include "rt_lex.h"

int rt_host_threads(void)
{
  const char *e = getenv("RT_HOST_THREADS");
  if (!e || !*e)
    e = getenv("OMP_NUM_THREADS");
  long n = e && *e ? strtol(e, NULL, 10) : 0;
  if (n <= 0)
    n = sysconf(_SC_NPROCESSORS_ONLN);
  if (n < 1)
    n = 1;
  if (n > 64)
    n = 64;
  return (int)n;
}

typedef struct {
  const rt_lex *lx;
  const char *s, *e;  /* chunk: [s, e), s at a line start */
  rt_vline *v;
  size_t n, cap;
  int oom;
} scan_task;

static void *scan_chunk(void *arg)
{
  scan_task *t = arg;
  rt_lex cur = *t->lx;
  const char *p = t->s;
  /* a table entry per line at most: sized once from the chunk's newlines,
   * so the scan never reallocates (first-touch page faults then happen on
   * this thread, in parallel with the others) */
  size_t lines = 1;
  for (const char *q = p; q < t->e; q++)
  {
    q = memchr(q, '\n', (size_t)(t->e - q));
    if (!q)
      break;
    lines++;
  }
  t->cap = lines;
  t->v = malloc(t->cap * sizeof *t->v);
  if (!t->v)
  {
    t->oom = 1;
    return NULL;
  }
  while (p < t->e)
  {
    const char *q = p;
    while (q < t->e && (*q == ' ' || *q == '\t' || *q == '\r' || *q == '\v' || *q == '\f'))
      q++;
    if (q + 1 < t->lx->end && q[0] == 'v' &&
        (rt_lex_space(q[1]) || (q[1] == 'n' && q + 2 < t->lx->end && rt_lex_space(q[2]))))
    {
      int len = q[1] == 'n' ? 2 : 1;
      rt_vline l;
      cur.p = q + len;
      if (!rt_lex_float(&cur, &l.x) && !rt_lex_float(&cur, &l.y) && !rt_lex_float(&cur, &l.z) &&
          cur.p - q < (ptrdiff_t)UINT32_MAX)
      {
        l.off = (size_t)(q - t->lx->buf);
        l.len = (uint32_t)(cur.p - q);
        t->v[t->n++] = l;
      }
    }
    p = memchr(q, '\n', (size_t)(t->e - q));
    if (!p)
      break;
    p++;
  }
  return NULL;
}

int rt_prescan_build(const rt_lex *lx, rt_prescan *ps)
{
  memset(ps, 0, sizeof *ps);
  size_t size = (size_t)(lx->end - lx->buf);
  int nt = rt_host_threads();
  if (size < ((size_t)4 << 20) || nt < 2)
    return RT_OK; /* small file: the serial scanner alone */
  if ((size_t)nt > size / (1u << 20))
    nt = (int)(size / (1u << 20));
  scan_task task[64];
  pthread_t tid[64];
  const char *s = lx->buf;
  for (int i = 0; i < nt; i++)
  {
    const char *e = i + 1 == nt ? lx->end : lx->buf + size / (size_t)nt * (size_t)(i + 1);
    if (e < s)
      e = s;
    if (i + 1 < nt)
    {
      const char *nl = memchr(e, '\n', (size_t)(lx->end - e));
      e = nl ? nl + 1 : lx->end;
    }
    memset(&task[i], 0, sizeof task[i]);
    task[i].lx = lx;
    task[i].s = s;
    task[i].e = e;
    s = e;
  }
  int started[64] = { 0 };
  for (int i = 0; i < nt; i++)
    started[i] = pthread_create(&tid[i], NULL, scan_chunk, &task[i]) == 0;
  for (int i = 0; i < nt; i++)
    if (started[i])
      pthread_join(tid[i], NULL);
    else
      scan_chunk(&task[i]);
  int oom = 0;
  for (int i = 0; i < nt; i++)
    oom |= task[i].oom;
  if (oom)
  {
    /* out of memory for the tables: fall back to the serial scanner */
    for (int i = 0; i < nt; i++)
      free(task[i].v);
    return RT_OK;
  }
  /* the threads' tables, in file order, are the segments (no merge copy) */
  for (int i = 0; i < nt; i++)
  {
    ps->seg_v[i] = task[i].v;
    ps->seg_n[i] = task[i].n;
  }
  ps->nseg = nt;
  return RT_OK;
}

void rt_prescan_free(rt_prescan *ps)
{
  for (int i = 0; i < ps->nseg; i++)
    free(ps->seg_v[i]);
  memset(ps, 0, sizeof *ps);
}
