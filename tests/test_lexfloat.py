"""The loaders' float conversion (host/rt_lex.h rt_lex_float: an exact fast
path with strtof fallback) against glibc strtof -- the conversion of the
reference's fscanf("%f") (cpu/parse_obj.c:25) -- on random and adversarial
inputs: identical float bits and identical consumed length."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(REPO, "raytracing-gpu_amd", "host")

HARNESS = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "rt_lex.h"

static unsigned long long st = 0x9E3779B97F4A7C15ull;
static unsigned long long rnd(void) {  /* splitmix64 */
  unsigned long long z = (st += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static long bad = 0, fast = 0, total = 0;

static void check(const char *s) {
  char buf[256];
  snprintf(buf, sizeof buf, "%s", s);
  rt_lex lx = { buf, buf, buf + strlen(buf), "t" };
  float a = 0.0f;
  int ra = rt_lex_float(&lx, &a);
  char *e;
  float b = strtof(buf, &e);
  int rb = e == buf;
  const char *n;
  float c;
  fast += rt_fast_strtof(buf + strspn(buf, " \t\n"), &c, &n);
  total++;
  if (ra != rb || (!ra && (memcmp(&a, &b, 4) != 0 || lx.p != e))) {
    if (bad < 20) fprintf(stderr, "MISMATCH '%s': %d %a (+%td) vs %d %a (+%td)\n", s, ra, a,
                          lx.p - buf, rb, b, e - buf);
    bad++;
  }
}

int main(int argc, char **argv) {
  long n = atol(argv[1]);
  const char *fixed[] = {"0", "-0", "+0", "0.0", ".5", "5.", "-.5e3", "1e", "1e+", "1e-", "1.5x",
                         "0x1p3", "-0X1.8p1", "inf", "-inf", "nan", "NaN(123)", ".", "-", "+",
                         "e5", "1e-38", "1.1754943e-38", "1.17549435e-38", "1e-39", "1e-45",
                         "3.4028235e38", "3.40282357e38", "3.5e38", "1e39", "123456789012345678",
                         "1234567890123456789", "12345678901234567890", "0.00000000000000000001",
                         "1e22", "1e23", "1e-22", "1e-23", "9007199254740993", "9007199254740992e-5",
                         "16777217", "16777219", "0.1", "0.2", "0.3", "33554433", "1.00000006",
                         "1.000000059604644775390625", "1.0000000596046447753906250001",
                         "  7.25", "4.99999999e-1", "00000000000000000000000001.5",
                         "1.5e0000000000000000000", "2.5E+10", "2.5e-10", "-9.98747798e-17", 0};
  for (int i = 0; fixed[i]; i++) check(fixed[i]);
  char s[128];
  for (long i = 0; i < n; i++) {
    unsigned long long r = rnd();
    int form = (int)(r % 6);
    if (form == 0) {  /* %.9g of a random float: the loaders' own output format */
      unsigned u = (unsigned)(rnd() >> 32);
      float f;
      memcpy(&f, &u, 4);
      if (!isfinite(f)) continue;
      snprintf(s, sizeof s, "%.9g", f);
    } else if (form == 1) {  /* decimal midpoint of two adjacent floats (the tie cases) */
      unsigned u = (unsigned)(rnd() >> 34) + 0x00800000u;
      float f, g;
      memcpy(&f, &u, 4);
      g = nextafterf(f, INFINITY);
      snprintf(s, sizeof s, "%.40g", ((double)f + (double)g) * 0.5);
    } else if (form == 2) {  /* random digits, random point and exponent */
      int nd = 1 + (int)(rnd() % 22), dot = (int)(rnd() % (nd + 1)), k = 0;
      if (rnd() & 1) s[k++] = '-';
      for (int j = 0; j < nd; j++) {
        if (j == dot) s[k++] = '.';
        s[k++] = (char)('0' + rnd() % 10);
      }
      if (rnd() % 3 == 0) k += sprintf(s + k, "e%d", (int)(rnd() % 90) - 45);
      s[k] = 0;
    } else if (form == 3) {  /* short values like hand-written scenes */
      snprintf(s, sizeof s, "%.*f", (int)(rnd() % 7), ((double)(long long)(rnd() % 2000001) - 1e6) / 997.0);
    } else if (form == 4) {  /* %.17g of a random double near float precision */
      double d = ((double)(rnd() >> 11) / 9007199254740992.0 - 0.5) * pow(10.0, (int)(rnd() % 20) - 10);
      snprintf(s, sizeof s, "%.17g", d);
    } else {  /* just above / below a float midpoint */
      unsigned u = (unsigned)(rnd() >> 34) + 0x00800000u;
      float f, g;
      memcpy(&f, &u, 4);
      g = nextafterf(f, INFINITY);
      double mid = ((double)f + (double)g) * 0.5;
      snprintf(s, sizeof s, "%.20g", nextafter(mid, (rnd() & 1) ? INFINITY : -INFINITY));
    }
    check(s);
  }
  printf("%ld %ld %ld\n", total, fast, bad);
  return 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("lexfloat")
    src = d / "h.c"
    src.write_text(HARNESS)
    exe = d / "h"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-ffp-contract=off", "-I" + HOST, str(src), "-o",
                    str(exe), "-lm"], check=True)
    return str(exe)


def test_fast_float_matches_strtof(harness):
    p = subprocess.run([harness, "400000"], capture_output=True, text=True, check=True)
    total, fast, bad = map(int, p.stdout.split())
    assert bad == 0, p.stderr
    assert total > 300000
    assert fast > total // 3  # the fast path decides most of them
