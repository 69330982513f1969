// Debug: device glibc_logf / __fdiv_rn / __fsqrt_rn vs host libm, bit for bit.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/debug_ops tools/debug_ops.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../parameter_server_amd/csrc/glibc_logf.h"

__global__ void k(const float* x, float* lg, float* q, float* s, float* s2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r2 = x[i];
  float l = psf::glibc_logf(r2);
  lg[i] = l;
  float qq = __fdiv_rn(__fmul_rn(-2.0f, l), r2);
  q[i] = qq;
  s[i] = __fsqrt_rn(qq);
  // candidate fix: double root + exact midpoint test
  float c = (float)__dsqrt_rn((double)qq);
  float lo = __uint_as_float(__float_as_uint(c) - 1u), hi = __uint_as_float(__float_as_uint(c) + 1u);
  double mlo = ((double)lo + (double)c) * 0.5, mhi = ((double)c + (double)hi) * 0.5;
  if ((double)qq < mlo * mlo) c = lo; else if ((double)qq > mhi * mhi) c = hi;
  s2[i] = c;
}

int main() {
  const int n = 1 << 20;
  float *x = (float*)malloc(n * 4), *lg = (float*)malloc(n * 4), *q = (float*)malloc(n * 4),
        *s = (float*)malloc(n * 4), *s2 = (float*)malloc(n * 4);
  unsigned st = 12345;
  for (int i = 0; i < n; ++i) {
    st = st * 1664525u + 1013904223u;
    x[i] = (float)((st >> 8) + 1) / 16777216.0f;
  }
  float *dx, *dl, *dq, *ds, *ds2;
  hipMalloc(&dx, n * 4); hipMalloc(&dl, n * 4); hipMalloc(&dq, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&ds2, n * 4);
  hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dl, dq, ds, ds2, n);
  hipMemcpy(lg, dl, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(q, dq, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s, ds, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s2, ds2, n * 4, hipMemcpyDeviceToHost);
  int bl = 0, bq = 0, bs = 0, bs2 = 0, bh = 0;
  for (int i = 0; i < n; ++i) {
    float hl = logf(x[i]);
    float hl2 = psf::glibc_logf(x[i]);
    if (memcmp(&hl, &hl2, 4)) ++bh;
    if (memcmp(&hl, &lg[i], 4)) { if (bl < 3) printf("log x=%a dev=%a host=%a\n", x[i], lg[i], hl); ++bl; }
    float hq = (-2.0f * lg[i]) / x[i];
    if (memcmp(&hq, &q[i], 4)) ++bq;
    float hs = sqrtf(q[i]);
    if (memcmp(&hs, &s[i], 4)) ++bs;
    if (memcmp(&hs, &s2[i], 4)) ++bs2;
  }
  printf("n=%d  host-restated-logf-vs-libm %d  dev-logf %d  div %d  sqrt_rn %d  sqrtf %d\n", n, bh, bl, bq, bs, bs2);
  return 0;
}
