// Streaming-bandwidth probe for MI355X: which launch shape reaches HBM peak
// for read-reduce (min/max) and read->write (copy / 4:1 pack) streams.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <int U>
__global__ __launch_bounds__(256) void rd_stride(const float4* __restrict__ x, size_t n4, uint32_t* out) {
  uint32_t lo = ~0u, hi = 0;
  size_t t = blockIdx.x * 256ull + threadIdx.x, T = gridDim.x * 256ull;
  for (size_t g = t; g < n4; g += U * T) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (g + u * T < n4) ? x[g + u * T] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  if ((lo ^ hi) == 0x12345678u) out[0] = lo;  // keep live
}

// each block owns a contiguous chunk
template <int U>
__global__ __launch_bounds__(256) void rd_chunk(const float4* __restrict__ x, size_t n4, size_t per_block, uint32_t* out) {
  uint32_t lo = ~0u, hi = 0;
  size_t b0 = blockIdx.x * per_block, b1 = min(n4, b0 + per_block);
  for (size_t g = b0 + threadIdx.x; g < b1; g += U * 256) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (g + u * 256 < b1) ? x[g + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  if ((lo ^ hi) == 0x12345678u) out[0] = lo;
}

template <int U>
__global__ __launch_bounds__(256) void copy_stride(const float4* __restrict__ x, float4* __restrict__ y, size_t n4) {
  size_t t = blockIdx.x * 256ull + threadIdx.x, T = gridDim.x * 256ull;
  for (size_t g = t; g < n4; g += U * T) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (g + u * T < n4) v[u] = x[g + u * T];
#pragma unroll
    for (int u = 0; u < U; ++u) if (g + u * T < n4) y[g + u * T] = v[u];
  }
}

// 4 floats -> 4 bytes (encode-shaped traffic), and the inverse (decode-shaped)
template <int U>
__global__ __launch_bounds__(256) void pack_stride(const float4* __restrict__ x, uint32_t* __restrict__ y, size_t n4) {
  size_t t = blockIdx.x * 256ull + threadIdx.x, T = gridDim.x * 256ull;
  for (size_t g = t; g < n4; g += U * T) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (g + u * T < n4) v[u] = x[g + u * T];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (g + u * T < n4)
        y[g + u * T] = (uint32_t)(int)v[u].x ^ ((uint32_t)(int)v[u].y << 8) ^ ((uint32_t)(int)v[u].z << 16) ^ ((uint32_t)(int)v[u].w << 24);
  }
}
template <int U>
__global__ __launch_bounds__(256) void unpack_stride(const uint32_t* __restrict__ x, float4* __restrict__ y, size_t n4) {
  size_t t = blockIdx.x * 256ull + threadIdx.x, T = gridDim.x * 256ull;
  for (size_t g = t; g < n4; g += U * T) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (g + u * T < n4) v[u] = x[g + u * T];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (g + u * T < n4) y[g + u * T] = make_float4(v[u] & 255, (v[u] >> 8) & 255, (v[u] >> 16) & 255, v[u] >> 24);
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const size_t n = 1ull << 28;  // floats (1 GiB)
  const size_t n4 = n / 4;
  float4* x; float4* y; uint32_t* o; uint32_t* c;
  CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&o, 64)); CK(hipMalloc(&c, n));
  CK(hipMemset(x, 0x3f, n * 4)); CK(hipMemset(c, 1, n));
  int reps = 20;
  auto rep = [&](const char* name, double bytes, float ms) {
    printf("%-36s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  for (int grid : {1024, 2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, 64, "rd_stride<4> grid=%d", grid);
    rep(nm, n * 4.0, timeit([&] { rd_stride<4><<<grid, 256>>>(x, n4, o); }, reps));
    snprintf(nm, 64, "rd_stride<8> grid=%d", grid);
    rep(nm, n * 4.0, timeit([&] { rd_stride<8><<<grid, 256>>>(x, n4, o); }, reps));
  }
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64];
    size_t per = (n4 + grid - 1) / grid;
    snprintf(nm, 64, "rd_chunk<4> grid=%d", grid);
    rep(nm, n * 4.0, timeit([&] { rd_chunk<4><<<grid, 256>>>(x, n4, per, o); }, reps));
    snprintf(nm, 64, "rd_chunk<8> grid=%d", grid);
    rep(nm, n * 4.0, timeit([&] { rd_chunk<8><<<grid, 256>>>(x, n4, per, o); }, reps));
  }
  {
    unsigned grid = (unsigned)(n4 / 256 / 4);
    char nm[64];
    snprintf(nm, 64, "rd_stride<4> one-shot grid=%u", grid);
    rep(nm, n * 4.0, timeit([&] { rd_stride<4><<<grid, 256>>>(x, n4, o); }, reps));
  }
  for (int grid : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "copy_stride<4> grid=%d", grid);
    rep(nm, n * 8.0, timeit([&] { copy_stride<4><<<grid, 256>>>(x, y, n4); }, reps));
    snprintf(nm, 64, "pack_stride<4> grid=%d", grid);
    rep(nm, n * 5.0, timeit([&] { pack_stride<4><<<grid, 256>>>(x, c, n4); }, reps));
    snprintf(nm, 64, "unpack_stride<4> grid=%d", grid);
    rep(nm, n * 5.0, timeit([&] { unpack_stride<4><<<grid, 256>>>(c, y, n4); }, reps));
  }
  for (int grid : {2048, 8192}) {
    char nm[64];
    snprintf(nm, 64, "pack_stride<8> grid=%d", grid);
    rep(nm, n * 5.0, timeit([&] { pack_stride<8><<<grid, 256>>>(x, c, n4); }, reps));
    snprintf(nm, 64, "unpack_stride<8> grid=%d", grid);
    rep(nm, n * 5.0, timeit([&] { unpack_stride<8><<<grid, 256>>>(c, y, n4); }, reps));
  }
  return 0;
}
