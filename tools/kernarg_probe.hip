#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N> struct Big { unsigned v[N]; };
template <int N>
__global__ void k(Big<N> b, unsigned* out) {
  out[blockIdx.x] = b.v[(blockIdx.x * 977) % N] + b.v[N - 1];
}
template <int N> int run() {
  Big<N> b;
  for (int i = 0; i < N; ++i) b.v[i] = i * 3 + 1;
  unsigned* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k<N>, dim3(64), dim3(64), 0, 0, b, d);
  hipError_t e = hipGetLastError();
  unsigned h[64]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  hipError_t e2 = hipDeviceSynchronize();
  int bad = 0;
  for (int i = 0; i < 64; ++i) bad += h[i] != b.v[(i * 977) % N] + b.v[N - 1];
  printf("N=%d bytes=%zu launch=%s sync=%s bad=%d\n", N, sizeof(Big<N>), hipGetErrorString(e), hipGetErrorString(e2), bad);
  hipFree(d);
  return 0;
}
int main() { run<1000>(); run<2000>(); run<4000>(); run<8000>(); return 0; }
