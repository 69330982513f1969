// logf exactly as the reference's libm computes it.
// License: the algorithm and the table values are glibc's (sysdeps/ieee754/{f,dbl}-64/e_log*.c,
// GNU LGPL v2.1 or later; originally Arm's optimized-routines, MIT), restated here; this
// file is distributed under those terms.
//
// NOISE (add_noise.h:29-39) calls std::log(float) inside libstdc++'s polar
// method; on the reference's platform that is glibc's logf (glibc >= 2.28,
// sysdeps/ieee754/flt-32/e_logf.c, from ARM optimized-routines): x = 2^k z with
// z in [0x3f330000, 2*0x3f330000), a 16-entry {1/c, log c} table indexed by the
// top 4 mantissa bits of z, log(x) = k ln2 + log c + log1p(z/c - 1) with a
// degree-3 polynomial, all in double, rounded to float once.  It is not
// correctly rounded (max error 0.82 ulp), so a correctly rounded device log
// disagrees with it on ~10 % of NOISE samples; this restatement agrees with
// the image's glibc 2.35 logf on every float in (0, 1] -- the only range the
// polar method feeds it (checked exhaustively; oracle/logf_check.c re-checks a
// sample in the CPU test suite).  Valid for 0 < x <= 1 and finite x > 0.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define PSF_HD __host__ __device__
#else
#define PSF_HD
#endif

namespace psf {

struct LogfEntry { double invc, logc; };

PSF_HD inline float glibc_logf(float x) {
  const LogfEntry T[16] = {
      {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
      {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
      {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
      {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
      {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
      {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
      {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
      {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
  };
  const double kLn2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  uint32_t ix;
  memcpy(&ix, &x, 4);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {  // subnormal (x > 0 here)
    float xs = x * 0x1p23f;
    memcpy(&ix, &xs, 4);
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  float zf;
  memcpy(&zf, &iz, 4);
  const double z = (double)zf;
  const double r = z * T[i].invc - 1.0;  // no FMA: compiled with -ffp-contract=off
  const double y0 = T[i].logc + (double)k * kLn2;
  const double r2 = r * r;
  double y = A1 * r + A2;
  y = A0 * r2 + y;
  y = y * r2 + (y0 + r);
  return (float)y;
}

}  // namespace psf
