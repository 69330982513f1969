// log(double) exactly as the reference's libm computes it.
// License: the algorithm and the table values are glibc's (sysdeps/ieee754/{f,dbl}-64/e_log*.c,
// GNU LGPL v2.1 or later; originally Arm's optimized-routines, MIT), restated here; this
// file is distributed under those terms.
//
// NOISE (add_noise.h:29-39) on DOUBLE values calls std::log(double) inside
// libstdc++'s polar method; on the reference's platform that is glibc's log
// (glibc >= 2.28, sysdeps/ieee754/dbl-64/e_log.c, from ARM
// optimized-routines), in the x86_64 build selected on CPUs with FMA
// (__log_fma: every CPU the reference's host and this image run on).  The
// algorithm: x = 2^k z with z in [0x1.6p-1, 0x1.6p0), a 128-entry {1/c, log c}
// table indexed by the top 7 mantissa bits of z, r = z/c - 1 as one fma,
// log(x) = k ln2 + log c + r + r^2 poly(r) with a hi/lo split of the
// first sum; x within 1/16 of 1 takes a degree-11 polynomial in r = x - 1
// with a 27-bit split of r.  It is not correctly rounded (max error 0.52
// ulp), so a correctly rounded or differently contracted device log
// disagrees with it on some NOISE samples.
//
// Every operation below is the one the image's libm executes, including
// which multiply-adds its compiler fused (read from the disassembly of the
// resolved __log_finite; the data is glibc_log_data.h, read out of the same
// libm).  Unfused operations rely on -ffp-contract=off.  Checked against the
// image's libm on every exponent and on random inputs (oracle/log_check.c in
// the CPU suite, tests/test_oracle.py).  Valid for finite x > 0.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "glibc_log_data.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define PSF_HD __host__ __device__
#else
#define PSF_HD
#endif

namespace psf {

PSF_HD inline double glibc_log(double x) {
  using namespace glibc_log_data;
  uint64_t ix;
  memcpy(&ix, &x, 8);
  // |x - 1| < ~1/16: log1p by polynomial (0x3fee000000000000 = 1 - 2^-4)
  if (ix - 0x3fee000000000000ull <= 0x308ffffffffffull) {
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
    const double r2 = r * r;
    const double r3 = r * r2;
    const double p0 = fma(r2, kB[3], fma(r, kB[2], kB[1]));
    const double p1 = fma(r2, kB[6], fma(r, kB[5], kB[4]));
    const double p2 = fma(r3, kB[10], fma(r2, kB[9], fma(r, kB[8], kB[7])));
    const double p = fma(fma(p2, r3, p1), r3, p0);
    // rhi = r + w - w with w = r * 2^27: the top 26 bits of r
    const double rhi = fma(-0x1p27, r, fma(r, 0x1p27, r));
    const double rlo = r - rhi;
    const double rr = rhi * rhi;
    const double hi = fma(rr, kB[0], r);  // r + rhi*rhi*B0 (B0 = -0.5: the product is exact)
    double lo = fma(rr, kB[0], r - hi);
    lo = fma(kB[0] * rlo, r + rhi, lo);
    const double y = fma(p, r3, lo);
    return hi + y;
  }
  const uint32_t top = (uint32_t)(ix >> 48);
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {  // subnormal (x > 0 finite here): normalise
    const double xs = x * 0x1p52;
    memcpy(&ix, &xs, 8);
    ix -= 52ull << 52;
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  double z;
  memcpy(&z, &iz, 8);
  const double r = fma(z, kTab[i].invc, -1.0);
  const double kd = (double)k;
  const double w = fma(kd, kLn2hi, kTab[i].logc);
  const double hi = r + w;
  const double lo = fma(kd, kLn2lo, (w - hi) + r);
  const double r2 = r * r;
  const double q = fma(fma(r, kA[4], kA[3]), r2, fma(r, kA[2], kA[1]));
  return fma(r * r2, q, fma(r2, kA[0], lo)) + hi;
}

}  // namespace psf
