/* rt_lex.h -- in-memory scanner with fscanf("%s"/"%f"/"%d"/"%u") semantics. */
#ifndef RT_LEX_H
#define RT_LEX_H

#include <stdint.h>
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

/* Parallel pre-parse of `v` / `vn` lines (lex_prescan.c). */
typedef struct rt_vline {
  size_t off;    /* offset of the `v`/`vn` token                  */
  uint32_t len;  /* bytes from the token to the end of the 3rd float */
  float x, y, z;
} rt_vline;

typedef struct rt_prescan {
  rt_vline *v;   /* increasing off; NULL = no table (small file)   */
  size_t n, cur;
} rt_prescan;

int rt_prescan_build(const rt_lex *lx, rt_prescan *ps);
void rt_prescan_free(rt_prescan *ps);
int rt_host_threads(void);

/* The `v`/`vn` token at `tok` was pre-parsed: store its three floats, move
 * the cursor past them and return 1; else 0 (convert serially). */
static inline int rt_prescan_take(rt_prescan *ps, rt_lex *lx, const char *tok, float out[3])
{
  if (!ps->v)
    return 0;
  size_t off = (size_t)(tok - lx->buf);
  while (ps->cur < ps->n && ps->v[ps->cur].off < off)
    ps->cur++;
  if (ps->cur >= ps->n || ps->v[ps->cur].off != off)
    return 0;
  const rt_vline *l = &ps->v[ps->cur++];
  out[0] = l->x;
  out[1] = l->y;
  out[2] = l->z;
  lx->p = lx->buf + off + l->len;
  return 1;
}

#endif
