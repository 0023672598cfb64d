/* rt_lex.h -- in-memory scanner with fscanf("%s"/"%f"/"%d"/"%u") semantics. */
#ifndef RT_LEX_H
#define RT_LEX_H

#include <stdlib.h>
#include <string.h>

typedef struct rt_lex {
  char *buf;          /* whole file, NUL-terminated */
  const char *p, *end;
  const char *path;
} rt_lex;

int rt_lex_open(const char *path, rt_lex *lx);
void rt_lex_close(rt_lex *lx);

/* C-locale isspace(), the set scanf skips */
static inline int rt_lex_space(char c)
{
  return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f';
}

static inline void rt_lex_skip_ws(rt_lex *lx)
{
  while (lx->p < lx->end && rt_lex_space(*lx->p))
    lx->p++;
}

static inline void rt_lex_skip_line(rt_lex *lx)
{
  while (lx->p < lx->end && *lx->p != '\n')
    lx->p++;
}

/* "%s": returns 0 at end of input */
static inline int rt_lex_token(rt_lex *lx, const char **tok, size_t *len)
{
  rt_lex_skip_ws(lx);
  if (lx->p >= lx->end)
    return 0;
  const char *s = lx->p;
  while (lx->p < lx->end && !rt_lex_space(*lx->p))
    lx->p++;
  *tok = s;
  *len = (size_t)(lx->p - s);
  return 1;
}

#define RT_TOK_IS(t, n, lit) ((n) == sizeof(lit) - 1 && memcmp((t), (lit), (n)) == 0)

/* "%f": strtof rounds exactly like scanf's conversion; 0 = ok */
static inline int rt_lex_float(rt_lex *lx, float *out)
{
  rt_lex_skip_ws(lx);
  char *e;
  float v = strtof(lx->p, &e);
  if (e == lx->p)
    return 1;
  lx->p = e;
  *out = v;
  return 0;
}

static inline int rt_lex_int(rt_lex *lx, int *out)
{
  rt_lex_skip_ws(lx);
  char *e;
  long v = strtol(lx->p, &e, 10);
  if (e == lx->p)
    return 1;
  lx->p = e;
  *out = (int)v;
  return 0;
}

static inline int rt_lex_uint(rt_lex *lx, unsigned *out)
{
  rt_lex_skip_ws(lx);
  char *e;
  unsigned long v = strtoul(lx->p, &e, 10);
  if (e == lx->p)
    return 1;
  lx->p = e;
  *out = (unsigned)v;
  return 0;
}

#endif
