// Probe: a 16-byte vector load from an address that is only 4-byte aligned
// (global_load_dwordx4 at base + 4): value check and bandwidth against the
// aligned load and four dword loads, over 256 MiB.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void k(const float* __restrict__ x, size_t ngroups, float* __restrict__ out) {
  float acc = 0.f;
  for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (size_t)gridDim.x * blockDim.x) {
    const float* p = x + 4 * g;
    f32x4 v;
    if (MODE == 2) {
      v.x = __builtin_nontemporal_load(p); v.y = __builtin_nontemporal_load(p + 1);
      v.z = __builtin_nontemporal_load(p + 2); v.w = __builtin_nontemporal_load(p + 3);
    } else {
      v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    }
    acc += v.x + 2.f * v.y + 3.f * v.z + 4.f * v.w;
  }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  const size_t n = (256u << 20) / 4, ng = n / 4 - 1;
  float *x, *o;
  hipMalloc(&x, n * 4 + 64);
  hipMalloc(&o, 2048 * 256 * 4);
  float* h = (float*)malloc(n * 4 + 64);
  for (size_t i = 0; i < n + 16; ++i) h[i] = (float)(i % 1000) * 0.001f;
  hipMemcpy(x, h, n * 4 + 64, hipMemcpyHostToDevice);
  // correctness of the unaligned vector load: group 0 at x + 1
  float* o1; hipMalloc(&o1, 4);
  hipLaunchKernelGGL((k<1>), dim3(1), dim3(1), 0, 0, x + 1, (size_t)1, o1);
  float r = 0; hipMemcpy(&r, o1, 4, hipMemcpyDeviceToHost);
  printf("unaligned dwordx4: %s (got %f want %f) err=%s\n", r == h[1] + 2 * h[2] + 3 * h[3] + 4 * h[4] ? "ok" : "BAD", r,
         h[1] + 2 * h[2] + 3 * h[3] + 4 * h[4], hipGetErrorString(hipGetLastError()));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[3] = {"aligned x4", "offset+4 x4", "offset+4 4xdword"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      const float* src = m == 0 ? x : x + 1;
      hipEventRecord(a);
      for (int it = 0; it < 10; ++it) {
        if (m == 2) hipLaunchKernelGGL((k<2>), dim3(2048), dim3(256), 0, 0, src, ng, o);
        else hipLaunchKernelGGL((k<1>), dim3(2048), dim3(256), 0, 0, src, ng, o);
      }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("%-18s %.1f GB/s\n", names[m], 10.0 * ng * 16 / (ms * 1e6));
    }
  return 0;
}
