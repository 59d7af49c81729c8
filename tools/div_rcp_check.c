/* Host check of k_div_rcp (ur3e_amd/csrc/ur3e_engine.h): with r = 1.0 / d and q0 = n * r,
   fma(-fma(d, q0, -n), r, q0) == n / d bit for bit (signed zeros included), d > 0.
   Operands: random across 120 binades of n and 60 of d (signed zeros every 17th pair), then
   structured pairs (integers, d near 1 and near powers of two, quotients near representable values),
   then the numerator extremes the guard sends to a true division (subnormal, tiny, huge, infinite).
   gcc -O2 -ffp-contract=off tools/div_rcp_check.c -lm -o /tmp/drc && /tmp/drc [pairs]
   (tests/test_div_rcp.py builds and runs it with a smaller count; the round-3 run used 4e8 + 2e8). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) {
  s ^= s << 13;
  s ^= s >> 7;
  s ^= s << 17;
  return s;
}
static double rnd(int emin, int emax) {
  uint64_t m = xr() & ((1ull << 52) - 1);
  int e = emin + (int)(xr() % (uint64_t)(emax - emin + 1));
  uint64_t b = ((uint64_t)(e + 1023) << 52) | m;
  if (xr() & 1) b |= 1ull << 63;
  double d;
  memcpy(&d, &b, 8);
  return d;
}
static long bad = 0;
/* k_div_rcp as ur3e_engine.h defines it (the guard included) */
static double div_rcp(double n, double d, double r) {
  double q0 = n * r, e = fma(d, q0, -n), q = fma(-e, r, q0), an = fabs(n);
  if (an > 0.0 && (an < 0x1p-960 || an > 0x1p+960)) q = n / d;
  return q;
}
static void check(double a, double d) {
  double r = 1.0 / d, q1 = div_rcp(a, d, r), ref = a / d;
  if (memcmp(&q1, &ref, 8)) {
    if (bad < 10) printf("a=%a d=%a ref=%a got=%a\n", a, d, ref, q1);
    bad++;
  }
}
int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 400000000L;
  for (long i = 0; i < n; i++) {
    double d = fabs(rnd(-30, 30)), a = rnd(-60, 60);
    if (i % 17 == 0) a = (i & 1) ? 0.0 : -0.0;
    check(a, d);
  }
  for (long i = 0; i < n / 2; i++) {
    double a, d;
    switch (i % 4) {
      case 0:
        a = (double)(int64_t)(xr() % 2000001 - 1000000);
        d = (double)(xr() % 100000 + 1);
        break;
      case 1:
        d = 1.0 + ldexp((double)(xr() % 1024), -52);
        a = ldexp((double)(xr() >> 11), -53) * ((xr() & 1) ? 1 : -1);
        break;
      case 2:
        d = ldexp(1.0, (int)(xr() % 40) - 20) * (1.0 - ldexp((double)(xr() % 64 + 1), -53));
        a = ldexp((double)(xr() >> 11), -(int)(xr() % 60));
        break;
      default:
        d = 1.0 + ldexp((double)(xr() >> 12), -52);
        a = ldexp((double)((xr() >> 11) | 1), -52) * d;
        break;
    }
    check(a, d);
  }
  /* the numerator extremes: subnormal, tiny (binades -1074..-850), huge (900..1023) and infinite, with
     divisors over the callers' range (2^-50: norms >= mjMINVAL = 1e-15; up to 2^40: Cholesky pivots) */
  for (long i = 0; i < n / 2; i++) {
    double a, d = ldexp(1.0 + ldexp((double)(xr() >> 12), -52), -50 + (int)(xr() % 91));
    uint64_t b;
    switch (i % 4) {
      case 0:
        b = xr() & ((1ull << 52) - 1);
        if (xr() & 1) b |= 1ull << 63;
        memcpy(&a, &b, 8);
        break;
      case 1: a = rnd(-1022, -850); break;
      case 2: a = rnd(900, 1023); if (fabs(a) / d > 1.7e308) a = ldexp(a, -60); break;
      default: a = (xr() & 1) ? INFINITY : -INFINITY; break;
    }
    check(a, d);
  }
  printf("pairs=%ld bad=%ld\n", n + n, bad);
  return bad != 0;
}
