/* ORACLE TEST INFRASTRUCTURE -- pins parameter_server_amd/csrc/glibc_log.h
 * (the NOISE kernel's double log) to the libm the reference links (glibc).
 *   log_check SAMPLE   SAMPLE pseudo-random doubles of each kind: uniform bit
 *                      patterns in (0, 1], values within 1/16 of 1 (the
 *                      polynomial path), polar-method r2 = a*a + b*b, and
 *                      every exponent's first/last mantissas (subnormals
 *                      included), plus values above 1
 * Prints the mismatch count; exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../parameter_server_amd/csrc/glibc_log.h"

static long bad = 0, n = 0;

static void check(double x) {
  double a = psf::glibc_log(x), g = log(x);
  uint64_t ua, ug;
  memcpy(&ua, &a, 8);
  memcpy(&ug, &g, 8);
  ++n;
  if (ua != ug) {
    if (bad < 5) printf("mismatch x=%a ours=%a libm=%a\n", x, a, g);
    ++bad;
  }
}

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}

int main(int argc, char** argv) {
  const long s = argc > 1 ? atol(argv[1]) : 1000000;
  const uint64_t one = 0x3ff0000000000000ull;
  for (long i = 0; i < s; ++i) {
    uint64_t u = next() % one + 1;  // (0, 1]
    double x;
    memcpy(&x, &u, 8);
    check(x);
    check(1.0 + ((double)(next() >> 11) * 0x1p-53 - 0.5) * 0.13);  // near 1, both paths
    const double a = (double)(next() >> 11) * 0x1p-52 - 1.0, b = (double)(next() >> 11) * 0x1p-52 - 1.0;
    const double r2 = a * a + b * b;
    if (r2 > 0.0 && r2 <= 1.0) check(r2);
    u = next() % (0x7ff0000000000000ull - one) + one;  // (1, inf)
    memcpy(&x, &u, 8);
    check(x);
  }
  for (uint64_t e = 0; e < 2047; ++e)
    for (uint64_t m = 0; m < 64; ++m) {
      double x;
      uint64_t u = (e << 52) | (m + (e == 0));
      memcpy(&x, &u, 8);
      check(x);
      u = (e << 52) | (0xFFFFFFFFFFFFFull - m);
      memcpy(&x, &u, 8);
      check(x);
    }
  printf("checked %ld doubles, %ld mismatches\n", n, bad);
  return bad != 0;
}
