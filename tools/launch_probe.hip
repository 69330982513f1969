// Host cost of one hipLaunchKernelGGL against the kernel-argument size
// (trivial kernel, 1 workgroup): launches are timed back to back on one
// stream, then drained.
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
template <int N> struct Args { unsigned v[N]; };
template <int N> __global__ void k(Args<N> a, unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = a.v[N - 1];
}
template <int N> void run(hipStream_t st, unsigned* d) {
  Args<N> a;
  for (int i = 0; i < N; ++i) a.v[i] = i;
  for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, st, a, d);
  (void)hipStreamSynchronize(st);
  const int iters = 2000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, st, a, d);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(st);
  auto t2 = std::chrono::steady_clock::now();
  printf("args %6zu B: host %.2f us/launch, drained %.2f us/launch\n", sizeof(Args<N>),
         std::chrono::duration<double, std::micro>(t1 - t0).count() / iters,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / iters);
}
int main() {
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  unsigned* d;
  (void)hipMalloc(&d, 4096);
  run<4>(st, d);
  run<64>(st, d);
  run<256>(st, d);
  run<1024>(st, d);
  run<4000>(st, d);
  return 0;
}
