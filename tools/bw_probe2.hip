// Probe 2: encode/decode-shaped streams on MI355X.
//  - pack (4 B in -> 1 B out) with u32 stores vs LDS-staged 16-B stores
//  - block-contiguous chunks, forward vs reverse order
//  - minmax(fwd) followed by pack(reverse) on the same input: Infinity-Cache reuse
//  - unpack (1 B in -> 4 B out) shapes
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bw_probe2 tools/bw_probe2.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t q8(float v) { return (uint32_t)(int)(v * 3.0f + 100.0f) & 255; }

// tile = 1024 float4 per block-iteration (256 thr x 4)
template <bool REV>
__global__ __launch_bounds__(256) void rd_chunk(const float4* __restrict__ x, size_t ntiles, size_t tiles_per_block, uint32_t* out) {
  uint32_t lo = ~0u, hi = 0;
  size_t t0 = blockIdx.x * tiles_per_block, t1 = min(ntiles, t0 + tiles_per_block);
  for (size_t k = 0; k < t1 - t0 && t0 < t1; ++k) {
    size_t t = REV ? (t1 - 1 - k) : (t0 + k);
    const float4* p = x + t * 1024;
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  if ((lo ^ hi) == 0x12345678u) out[0] = lo;
}

// pack with u32 stores (lane-coalesced, 256 B per wave store)
template <bool REV>
__global__ __launch_bounds__(256) void pack_u32(const float4* __restrict__ x, uint32_t* __restrict__ y, size_t ntiles, size_t tpb) {
  size_t t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  for (size_t k = 0; t0 < t1 && k < t1 - t0; ++k) {
    size_t t = REV ? (t1 - 1 - k) : (t0 + k);
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = x[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      y[t * 1024 + u * 256 + threadIdx.x] = q8(v[u].x) | (q8(v[u].y) << 8) | (q8(v[u].z) << 16) | (q8(v[u].w) << 24);
  }
}

// pack staged through LDS -> one 16-B store per lane per tile
template <bool REV>
__global__ __launch_bounds__(256) void pack_lds(const float4* __restrict__ x, uint4* __restrict__ y, size_t ntiles, size_t tpb) {
  __shared__ uint32_t s[1024];
  size_t t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  for (size_t k = 0; t0 < t1 && k < t1 - t0; ++k) {
    size_t t = REV ? (t1 - 1 - k) : (t0 + k);
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = x[t * 1024 + u * 256 + threadIdx.x];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u)
      s[u * 256 + threadIdx.x] = q8(v[u].x) | (q8(v[u].y) << 8) | (q8(v[u].z) << 16) | (q8(v[u].w) << 24);
    __syncthreads();
    y[t * 256 + threadIdx.x] = reinterpret_cast<const uint4*>(s)[threadIdx.x];
  }
}

// unpack: u32 load -> float4 store (coalesced)
__global__ __launch_bounds__(256) void unpack_u32(const uint32_t* __restrict__ c, float4* __restrict__ y, size_t ntiles, size_t tpb) {
  size_t t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  for (size_t t = t0; t < t1; ++t) {
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = c[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      y[t * 1024 + u * 256 + threadIdx.x] = make_float4(w[u] & 255, (w[u] >> 8) & 255, (w[u] >> 16) & 255, w[u] >> 24);
  }
}
// unpack with one 16-B load per lane, LDS transpose, coalesced float4 stores
__global__ __launch_bounds__(256) void unpack_lds(const uint4* __restrict__ c, float4* __restrict__ y, size_t ntiles, size_t tpb) {
  __shared__ uint32_t s[1024];
  size_t t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  for (size_t t = t0; t < t1; ++t) {
    uint4 w = c[t * 256 + threadIdx.x];
    __syncthreads();
    reinterpret_cast<uint4*>(s)[threadIdx.x] = w;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t q = s[u * 256 + threadIdx.x];
      y[t * 1024 + u * 256 + threadIdx.x] = make_float4(q & 255, (q >> 8) & 255, (q >> 16) & 255, q >> 24);
    }
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

// time only the second kernel of a pair (events around it)
template <typename F, typename G>
float time_second(F first, G second, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float tot = 0;
  for (int i = 0; i < reps + 2; ++i) {
    first();
    CK(hipEventRecord(a));
    second();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (i >= 2) tot += ms;
  }
  return tot / reps;
}

int main() {
  const size_t maxn = 1ull << 28;
  float4 *x, *x2, *y; uint32_t *o, *c;
  CK(hipMalloc(&x, maxn * 4)); CK(hipMalloc(&x2, maxn * 4)); CK(hipMalloc(&y, maxn * 4));
  CK(hipMalloc(&o, 64)); CK(hipMalloc(&c, maxn));
  CK(hipMemset(x, 0x3f, maxn * 4)); CK(hipMemset(x2, 0x3e, maxn * 4)); CK(hipMemset(c, 1, maxn));
  const int reps = 10;
  for (size_t n : {1ull << 27, 1ull << 28}) {
    size_t ntiles = n / 4096;  // 1024 float4 per tile
    printf("--- n = 2^%d floats (%zu MiB)\n", n == (1ull << 27) ? 27 : 28, n * 4 >> 20);
    for (int grid : {1024, 2048, 4096}) {
      size_t tpb = (ntiles + grid - 1) / grid;
      double rb = n * 4.0, pb = n * 5.0;
      auto pr = [&](const char* nm, double bytes, float ms) {
        printf("  %-44s grid=%5d %8.1f us %7.1f GB/s\n", nm, grid, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
      };
      pr("rd_chunk fwd (cold: other buffer before)", rb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x2, ntiles, tpb, o); }, [&] { rd_chunk<false><<<grid, 256>>>(x, ntiles, tpb, o); }, reps));
      pr("pack_u32 fwd (cold)", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x2, ntiles, tpb, o); }, [&] { pack_u32<false><<<grid, 256>>>(x, c, ntiles, tpb); }, reps));
      pr("pack_lds fwd (cold)", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x2, ntiles, tpb, o); }, [&] { pack_lds<false><<<grid, 256>>>(x, (uint4*)c, ntiles, tpb); }, reps));
      pr("pack_u32 REV after rd fwd same x", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x, ntiles, tpb, o); }, [&] { pack_u32<true><<<grid, 256>>>(x, c, ntiles, tpb); }, reps));
      pr("pack_lds REV after rd fwd same x", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x, ntiles, tpb, o); }, [&] { pack_lds<true><<<grid, 256>>>(x, (uint4*)c, ntiles, tpb); }, reps));
      pr("pack_lds FWD after rd fwd same x", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x, ntiles, tpb, o); }, [&] { pack_lds<false><<<grid, 256>>>(x, (uint4*)c, ntiles, tpb); }, reps));
      pr("unpack_u32 (cold)", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x2, ntiles, tpb, o); }, [&] { unpack_u32<<<grid, 256>>>(c, y, ntiles, tpb); }, reps));
      pr("unpack_lds (cold)", pb,
         time_second([&] { rd_chunk<false><<<grid, 256>>>(x2, ntiles, tpb, o); }, [&] { unpack_lds<<<grid, 256>>>((uint4*)c, y, ntiles, tpb); }, reps));
      pr("unpack_u32 after pack_u32 (codes warm)", pb,
         time_second([&] { pack_u32<false><<<grid, 256>>>(x, c, ntiles, tpb); }, [&] { unpack_u32<<<grid, 256>>>(c, y, ntiles, tpb); }, reps));
    }
  }
  return 0;
}
