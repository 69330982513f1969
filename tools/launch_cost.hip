// Launch cost of empty kernels by workgroup shape, LDS and VGPR footprint
// (diagnostic): hipcc --offload-arch=gfx950 -O3 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_runtime.h>

#include <cstdio>

template <int T, int LDS_BYTES, bool BIGV>
__global__ __launch_bounds__(T) void k_empty(int* out, int n) {
  __shared__ char lds[LDS_BYTES > 0 ? LDS_BYTES : 4];
  if (BIGV) {  // keep ~200 VGPRs live
    float v[192];
#pragma unroll
    for (int i = 0; i < 192; ++i) v[i] = (float)(threadIdx.x * i);
#pragma unroll
    for (int i = 0; i < 192; ++i) asm volatile("" : "+v"(v[i]));
    float s = 0;
#pragma unroll
    for (int i = 0; i < 192; ++i) s += v[i];
    if (s == -1.f) out[0] = 1;
  }
  lds[threadIdx.x % (LDS_BYTES > 0 ? LDS_BYTES : 4)] = (char)n;
  __syncthreads();
  if (n < 0 && threadIdx.x == 0) out[blockIdx.x] = lds[0];
}

template <typename K>
float timeit(K k, int grid, int threads, int* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 0, 0, d, 1);
  hipEventRecord(a, 0);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 0, 0, d, 1);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000 / 20;
}

int main() {
  int* d;
  hipMalloc(&d, 1 << 20);
  printf("512 thr, 256 wg, no lds        : %.2f us\n", timeit(k_empty<512, 0, false>, 256, 512, d));
  printf("512 thr, 256 wg, 116 KiB lds   : %.2f us\n", timeit(k_empty<512, 116 * 1024, false>, 256, 512, d));
  printf("512 thr, 256 wg, 60 KiB lds    : %.2f us\n", timeit(k_empty<512, 60 * 1024, false>, 256, 512, d));
  printf("512 thr, 256 wg, 200 vgpr      : %.2f us\n", timeit(k_empty<512, 0, true>, 256, 512, d));
  printf("512 thr, 256 wg, 116K + 200vgpr: %.2f us\n", timeit(k_empty<512, 116 * 1024, true>, 256, 512, d));
  printf("256 thr, 2048 wg, no lds       : %.2f us\n", timeit(k_empty<256, 0, false>, 2048, 256, d));
  printf("256 thr, 2048 wg, 76 KiB lds   : %.2f us\n", timeit(k_empty<256, 76 * 1024, false>, 2048, 256, d));
  printf("64 thr, 8192 wg, 18 KiB lds    : %.2f us\n", timeit(k_empty<64, 18 * 1024, false>, 8192, 64, d));
  return 0;
}
