/* rt_lex.h -- in-memory scanner with fscanf("%s"/"%f"/"%d"/"%u") semantics. */
#ifndef RT_LEX_H
#define RT_LEX_H

#include <math.h>
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

/* Exact fast path of strtof() for plain decimals [+-]digits[.digits][e[+-]digits]
 * (Clinger): with at most 19 significant digits the value is m 10^k exactly,
 * m an integer; for m <= 2^53 and |k| <= 22 the double m * 10^k (or m / 10^-k)
 * is the correctly rounded double of that value, and rounding it to float
 * gives strtof's correctly rounded float unless the double is itself a float
 * rounding midpoint (the one double-rounding hazard).  Returns 0 when it
 * cannot decide (hex, inf/nan, too many digits, large exponents, midpoints,
 * results outside the normal float range): the caller then uses strtof.
 * *next = the end of the number exactly as strtof would consume it. */
static inline int rt_fast_strtof(const char *s, float *out, const char **next)
{
  static const double p10[23] = { 1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22 };
  const char *p = s;
  int neg = 0;
  if (*p == '+' || *p == '-')
    neg = *p++ == '-';
  if (p[0] == '0' && (p[1] == 'x' || p[1] == 'X'))
    return 0; /* hexadecimal float: strtof's business */
  uint64_t m = 0;
  int nd = 0, k = 0, any = 0;
  for (; *p >= '0' && *p <= '9'; p++, any = 1)
  {
    if (m == 0 && *p == '0')
      continue; /* leading zeros carry no digits */
    if (++nd > 19)
      return 0;
    m = m * 10 + (uint64_t)(*p - '0');
  }
  if (*p == '.')
  {
    p++;
    for (; *p >= '0' && *p <= '9'; p++, any = 1)
    {
      k--;
      if (m == 0 && *p == '0')
        continue;
      if (++nd > 19)
        return 0;
      m = m * 10 + (uint64_t)(*p - '0');
    }
  }
  if (!any)
    return 0; /* no digits: "inf", "nan", "." ... */
  if (*p == 'e' || *p == 'E')
  {
    const char *q = p + 1;
    int eneg = 0;
    if (*q == '+' || *q == '-')
      eneg = *q++ == '-';
    if (*q >= '0' && *q <= '9')
    {
      int ex = 0;
      for (; *q >= '0' && *q <= '9'; q++)
        if (ex < 10000)
          ex = ex * 10 + (*q - '0');
      k += eneg ? -ex : ex;
      p = q;
    } /* else the 'e' is not part of the number, as in strtof */
  }
  double d;
  if (m == 0)
    d = 0.0;
  else
  {
    if (m > (1ull << 53) || k > 22 || k < -22)
      return 0;
    d = k >= 0 ? (double)m * p10[k] : (double)m / p10[-k];
    if (d < 1.1754943508222875e-38 || d > 3.4028234663852886e38)
      return 0; /* subnormal or overflowing float: strtof decides */
    const float f = (float)d;
    if ((double)f != d)
    {
      const float g = nextafterf(f, d > (double)f ? __builtin_inff() : -__builtin_inff());
      if (d == ((double)f + (double)g) * 0.5)
        return 0; /* a float midpoint: the tie needs the exact decimal */
    }
  }
  const float v = (float)d;
  *out = neg ? -v : v;
  *next = p;
  return 1;
}

/* "%f": the conversion of scanf (correctly rounded strtof); 0 = ok */
static inline int rt_lex_float(rt_lex *lx, float *out)
{
  rt_lex_skip_ws(lx);
  const char *n;
  if (rt_fast_strtof(lx->p, out, &n))
  {
    lx->p = n;
    return 0;
  }
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
  /* one table per prescan thread, each in increasing off, the tables in
   * file order; seg == nseg or no tables = serial scanner only */
  rt_vline *seg_v[64];
  size_t seg_n[64];
  int nseg, seg;
  size_t cur;    /* cursor in table seg */
} rt_prescan;

int rt_prescan_build(const rt_lex *lx, rt_prescan *ps);
void rt_prescan_free(rt_prescan *ps);
int rt_host_threads(void);

/* The `v`/`vn` token at `tok` was pre-parsed: store its three floats, move
 * the cursor past them and return 1; else 0 (convert serially). */
static inline int rt_prescan_take(rt_prescan *ps, rt_lex *lx, const char *tok, float out[3])
{
  size_t off = (size_t)(tok - lx->buf);
  for (;;)
  {
    if (ps->seg >= ps->nseg)
      return 0;
    const rt_vline *v = ps->seg_v[ps->seg];
    const size_t n = ps->seg_n[ps->seg];
    while (ps->cur < n && v[ps->cur].off < off)
      ps->cur++;
    if (ps->cur < n)
      break;
    ps->seg++;  /* this table is spent: the next one starts further on */
    ps->cur = 0;
  }
  const rt_vline *l = &ps->seg_v[ps->seg][ps->cur];
  if (l->off != off)
    return 0;
  ps->cur++;
  out[0] = l->x;
  out[1] = l->y;
  out[2] = l->z;
  lx->p = tok + l->len;
  return 1;
}

#endif
