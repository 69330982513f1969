// Probe: FIXING_FLOAT-like streaming (read 4 f32, write one dword of 4 codes)
// with the codes written (0) contiguously, or into a snappy stored-stream
// layout (fragment k's 65536 code bytes at hdr + k * 65539 + 3: every wave's
// 256-byte run misaligned by the same 0..3 bytes) by (1) unaligned dword
// stores or (2) aligned dwords funnel-shifted from the next lane plus byte
// stores at the run's two ends.  Checks the bytes and prints GB/s of
// algorithmic traffic (5 bytes per value).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__device__ __forceinline__ uint32_t code4(float4 v) {
  return ((uint32_t)(int)(v.x * 7.f) & 255) | (((uint32_t)(int)(v.y * 7.f) & 255) << 8) |
         (((uint32_t)(int)(v.z * 7.f) & 255) << 16) | (((uint32_t)(int)(v.w * 7.f) & 255) << 24);
}
__host__ __device__ __forceinline__ size_t staged_off(size_t b, uint32_t hdr) { return hdr + (b >> 16) * 65539 + 3 + (b & 65535); }

template <int MODE>
__global__ __launch_bounds__(256) void k(const float4* __restrict__ x, size_t ngroups, uint8_t* __restrict__ out,
                                         uint32_t hdr) {
  const size_t per = 4096;  // groups per workgroup tile loop (16 KiB of f32 per tile)
  for (size_t t = (size_t)blockIdx.x * per; t < ngroups; t += (size_t)gridDim.x * per) {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = x[t + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const size_t g = t + u * 256 + threadIdx.x;
      const uint32_t w = code4(v[u]);
      if (MODE == 0) {
        reinterpret_cast<uint32_t*>(out)[g] = w;
      } else if (MODE == 1) {
        uint8_t* p = out + staged_off(4 * g, hdr);
        typedef uint32_t __attribute__((aligned(1))) u32u;
        *reinterpret_cast<u32u*>(p) = w;
      } else if (MODE == 3) {  // one dword store at the unaligned address (hardware unaligned mode)
        uint8_t* p = out + staged_off(4 * g, hdr);
        asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(w) : "memory");
      } else {
        const uint32_t lane = threadIdx.x & 63;
        const size_t b0 = 4 * (g - lane);  // the run's first code byte
        const size_t s0 = staged_off(b0, hdr);
        const uint32_t m = (uint32_t)(s0 & 3);
        const uint32_t nx = __shfl_down(w, 1, 64);
        if (m == 0) {
          reinterpret_cast<uint32_t*>(out + s0)[lane] = w;
        } else {
          uint32_t* a = reinterpret_cast<uint32_t*>(out + s0 - m) + 1;  // aligned dwords after the first partial
          if (lane < 63) a[lane] = __builtin_amdgcn_alignbyte(nx, w, 4 - m);
          if (lane == 0)
            for (uint32_t i = 0; i < 4 - m; ++i) out[s0 + i] = (uint8_t)(w >> (8 * i));
          if (lane == 63)
            for (uint32_t i = 4 - m; i < 4; ++i) out[s0 + 252 + i] = (uint8_t)(w >> (8 * i));
        }
      }
    }
  }
}

int main() {
  const size_t n = 1ull << 28, ng = n / 4, hdr = 5;
  const size_t nfrag = n / 65536, sbytes = hdr + nfrag * 65539 + 64;
  float4* x;
  uint8_t* o;
  hipMalloc(&x, n * 4);
  hipMalloc(&o, sbytes);
  float* h = (float*)malloc(n * 4);
  for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.01f;
  hipMemcpy(x, h, n * 4, hipMemcpyHostToDevice);
  uint8_t* got = (uint8_t*)malloc(sbytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[4] = {"contiguous", "staged aligned(1) store", "staged funnel", "staged asm dword"};
  for (int rep = 0; rep < 3; ++rep)
    for (int m = 0; m < 4; ++m) {
      hipMemset(o, 0, sbytes);
      hipEventRecord(a);
      for (int it = 0; it < 10; ++it) {
        if (m == 0) hipLaunchKernelGGL((k<0>), dim3(16384), dim3(256), 0, 0, x, ng, o, (uint32_t)hdr);
        if (m == 1) hipLaunchKernelGGL((k<1>), dim3(16384), dim3(256), 0, 0, x, ng, o, (uint32_t)hdr);
        if (m == 2) hipLaunchKernelGGL((k<2>), dim3(16384), dim3(256), 0, 0, x, ng, o, (uint32_t)hdr);
        if (m == 3) hipLaunchKernelGGL((k<3>), dim3(16384), dim3(256), 0, 0, x, ng, o, (uint32_t)hdr);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      int bad = 0;
      if (rep == 0) {
        hipMemcpy(got, o, sbytes, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < n && bad < 3; i += 997) {
          const float* f = h + i;
          const uint8_t want = (uint8_t)((int)(f[0] * 7.f) & 255);
          const size_t at = m == 0 ? i : staged_off(i, hdr);
          if (got[at] != want) ++bad;
        }
        for (size_t i = 3; i < n && bad < 3; i += 65536) {  // a run's last bytes
          const uint8_t want = (uint8_t)((int)(h[i] * 7.f) & 255);
          if (got[m == 0 ? i : staged_off(i, hdr)] != want) ++bad;
        }
      }
      printf("%-24s %8.1f GB/s  %.1f us/launch %s\n", names[m], 10.0 * n * 5 / (ms * 1e6), ms * 100.0,
             rep == 0 ? (bad ? "BAD" : "ok") : "");
    }
  return 0;
}
