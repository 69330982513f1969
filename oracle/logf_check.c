/* ORACLE TEST INFRASTRUCTURE -- pins parameter_server_amd/csrc/glibc_logf.h
 * (the NOISE kernel's logf) to the libm the reference links (glibc).
 *   logf_check            every float in (0, 1]   (~1.07e9 values, ~25 s)
 *   logf_check SAMPLE     SAMPLE pseudo-random floats in (0, 1] plus every
 *                         exponent's first/last mantissas
 * Prints the mismatch count; exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../parameter_server_amd/csrc/glibc_logf.h"

static int check(uint32_t u, long* bad) {
  float x;
  memcpy(&x, &u, 4);
  float a = psf::glibc_logf(x), g = logf(x);
  uint32_t ua, ug;
  memcpy(&ua, &a, 4);
  memcpy(&ug, &g, 4);
  if (ua != ug) ++*bad;
  return 0;
}

int main(int argc, char** argv) {
  long bad = 0, n = 0;
  if (argc < 2) {
    for (uint32_t u = 1; u <= 0x3f800000u; ++u, ++n) check(u, &bad);
  } else {
    long s = atol(argv[1]);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    for (long i = 0; i < s; ++i, ++n) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      check((uint32_t)(st % 0x3f800000u) + 1u, &bad);
    }
    for (uint32_t e = 0; e < 127; ++e)
      for (uint32_t m = 0; m < 64; ++m, n += 2) {
        check((e << 23) | (m + (e == 0)), &bad);
        check((e << 23) | (0x7FFFFFu - m), &bad);
      }
  }
  printf("checked %ld floats, %ld mismatches\n", n, bad);
  return bad != 0;
}
