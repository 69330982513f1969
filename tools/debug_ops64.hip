// Debug: device double log / sqrt vs host libm (bit for bit).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
__global__ void k(const double* x, double* lg, double* s, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  lg[i] = log(x[i]);
  s[i] = __dsqrt_rn(x[i] * 3.7);
}
int main() {
  const int n = 1 << 20;
  double *x = (double*)malloc(n * 8), *lg = (double*)malloc(n * 8), *s = (double*)malloc(n * 8);
  unsigned long long st = 12345;
  for (int i = 0; i < n; ++i) { st = st * 6364136223846793005ull + 1442695040888963407ull; x[i] = (double)((st >> 11) + 1) / 9007199254740992.0; }
  double *dx, *dl, *ds;
  hipMalloc(&dx, n * 8); hipMalloc(&dl, n * 8); hipMalloc(&ds, n * 8);
  hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dl, ds, n);
  hipMemcpy(lg, dl, n * 8, hipMemcpyDeviceToHost); hipMemcpy(s, ds, n * 8, hipMemcpyDeviceToHost);
  int bl = 0, bs = 0;
  for (int i = 0; i < n; ++i) {
    double hl = log(x[i]), hs = sqrt(x[i] * 3.7);
    if (memcmp(&hl, &lg[i], 8)) ++bl;
    if (memcmp(&hs, &s[i], 8)) ++bs;
  }
  printf("n=%d  log mismatches %d  sqrt mismatches %d\n", n, bl, bs);
  return 0;
}
