// What an event record between two back-to-back kernels costs the device:
// a chain of streaming kernels (each reads 64 MiB) with 0-3 hipEventRecord
// calls between consecutive launches, for events created with
// hipEventDisableTiming, with hipEventDisableTiming | hipEventDisableSystemFence,
// and with timing on.  Reported: device time per kernel over the chain.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/event_gap_probe tools/event_gap_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_sum(const f4v* __restrict__ x, size_t n4, float* out) {
  float s = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const f4v v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

int main() {
  const size_t n = 1ull << 24;  // 64 MiB of floats
  f4v* x;
  float* o;
  CK(hipMalloc(&x, n * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMalloc(&o, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  struct F { const char* name; unsigned flags; };
  const F fl[] = {{"DisableTiming", hipEventDisableTiming},
                  {"DisableTiming|DisableSystemFence", hipEventDisableTiming | hipEventDisableSystemFence},
                  {"timing", hipEventDefault}};
  const int chain = 40;
  for (int rep = 0; rep < 2; ++rep)
    for (const F& f : fl) {
      hipEvent_t ev[3 * chain];
      for (auto& h : ev) CK(hipEventCreateWithFlags(&h, f.flags));
      for (int k = 0; k <= 3; ++k) {
        float best = 1e30f;
        for (int trial = 0; trial < 5; ++trial) {
          CK(hipEventRecord(t0, st));
          for (int i = 0; i < chain; ++i) {
            k_sum<<<2048, 256, 0, st>>>(x, n / 4, o);
            for (int r = 0; r < k; ++r) CK(hipEventRecord(ev[3 * i + r], st));
          }
          CK(hipEventRecord(t1, st));
          CK(hipEventSynchronize(t1));
          float ms;
          CK(hipEventElapsedTime(&ms, t0, t1));
          if (ms < best) best = ms;
        }
        printf("%-34s records between kernels %d: %7.2f us per kernel\n", f.name, k, best * 1e3f / chain);
      }
      for (auto& h : ev) CK(hipEventDestroy(h));
    }
  return 0;
}
