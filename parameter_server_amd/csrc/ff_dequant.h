// FIXING_FLOAT's dequantise (fixing_float.h:89-101), shared by the decode
// kernels (ff_codec.hip) and the uncompress kernels that decode FIXING_FLOAT
// codes as they leave a COMPRESSING stream (snappy.hip).  The two must give the
// same bits, so there is one definition.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psf {

// value = code / ratio * bin + min, in the reference's double sequence
template <typename V>
__device__ __forceinline__ V dequant(uint64_t code, double ratio, double bin, double min_v) {
  double r = (double)code;
  return (V)(r / ratio * bin + min_v);
}

// The same value with the quotient r / ratio formed from inv = RN(1/ratio):
// q0 = RN(r * inv), e = r - q0 * ratio (exact, one fma), q = RN(q0 + e * inv).
// Markstein's correction; checked exhaustively to equal the IEEE quotient for
// every code of num_bytes 1..3 (tests/test_oracle.py::test_decode_quotient),
// so the decoded values stay bit-identical at a third of the f64 work of the
// division sequence, which bounded the nb=2/3 decode.
template <typename V>
__device__ __forceinline__ V dequant_q(uint64_t code, double ratio, double inv, double bin, double min_v) {
  const double r = (double)code;
  const double q0 = r * inv;
  const double q = __builtin_fma(__builtin_fma(-q0, ratio, r), inv, q0);
  return (V)(q * bin + min_v);
}

}  // namespace psf
