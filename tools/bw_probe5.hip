// Probe 5: does keeping part of the value array on chip (registers + LDS)
// across a grid barrier beat the two-pass minmax -> encode stream?  One
// launch: stream the non-resident tiles (min/max), load R register tiles and
// L LDS tiles per workgroup (min/max), grid barrier (monotonic counter,
// bounded spin), fold the partials, quantise the resident tiles without
// re-reading them, then stream the rest again.  Trivial quantiser: memory
// behaviour only.  Compared with the two-kernel form over the same rotating
// inputs (2^27 f32, 3 buffers).  Diagnostic only.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bw_probe5 tools/bw_probe5.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ void acc(f4v v, uint32_t& lo, uint32_t& hi) {
  uint32_t a = key(v.x), b = key(v.y), c = key(v.z), d = key(v.w);
  lo = min(lo, min(min(a, b), min(c, d)));
  hi = max(hi, max(max(a, b), max(c, d)));
}
__device__ __forceinline__ uint32_t q4(f4v v, float mn, float sc) {
  uint32_t w = 0;
  w = __builtin_amdgcn_cvt_pk_u8_f32((v.x - mn) * sc, 0, w);
  w = __builtin_amdgcn_cvt_pk_u8_f32((v.y - mn) * sc, 1, w);
  w = __builtin_amdgcn_cvt_pk_u8_f32((v.z - mn) * sc, 2, w);
  w = __builtin_amdgcn_cvt_pk_u8_f32((v.w - mn) * sc, 3, w);
  return w;
}
__device__ __forceinline__ f4v ld(const f4v* p) { return __builtin_nontemporal_load(p); }

template <typename K>
__device__ __forceinline__ void block_mm(K& lo, K& hi) {
  __shared__ K s_lo[4], s_hi[4];
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (K)__shfl_xor(lo, o, 64));
    hi = max(hi, (K)__shfl_xor(hi, o, 64));
  }
  if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
  __syncthreads();
  lo = min(min(s_lo[0], s_lo[1]), min(s_lo[2], s_lo[3]));
  hi = max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3]));
  __syncthreads();
}

// ---- two-kernel baseline ----
__global__ __launch_bounds__(256) void k_minmax(const f4v* __restrict__ x, size_t ntiles, uint32_t* part) {
  uint32_t lo = ~0u, hi = 0;
  size_t per = (ntiles + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(x + t * 1024 + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc(v[u], lo, hi);
  }
  block_mm(lo, hi);
  if (threadIdx.x == 0) { part[blockIdx.x] = lo; part[gridDim.x + blockIdx.x] = hi; }
}
__global__ __launch_bounds__(256) void k_encode(const f4v* __restrict__ x, uint32_t* __restrict__ y, size_t ntiles,
                                                const uint32_t* part, int nparts) {
  uint32_t lo = ~0u, hi = 0;
  for (int i = threadIdx.x; i < nparts; i += 256) { lo = min(lo, part[i]); hi = max(hi, part[nparts + i]); }
  block_mm(lo, hi);
  const float mn = unkey(lo), sc = 254.0f / (unkey(hi) - mn);
  size_t per = (ntiles + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(x + t * 1024 + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(q4(v[u], mn, sc), y + t * 1024 + u * 256 + threadIdx.x);
  }
}

// ---- fused, resident ----
template <int R, int L, bool REV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void k_fused(const f4v* __restrict__ x, uint32_t* __restrict__ y, size_t ntiles, unsigned* bar, unsigned target,
             uint32_t* part, unsigned* timeout) {
  const unsigned G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  const size_t nres = (size_t)G * (R + L);
  const size_t ns = ntiles - nres, per = (ns + G - 1) / G;
  const size_t s0 = nres + min(ns, (size_t)b * per), s1 = nres + min(ns, (size_t)(b + 1) * per);
  uint32_t lo = ~0u, hi = 0;
  for (size_t t = s0; t < s1; ++t) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(x + t * 1024 + u * 256 + tid);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc(v[u], lo, hi);
  }
  const size_t r0 = (size_t)b * (R + L);
  f4v reg[R > 0 ? R : 1][4];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u) reg[r][u] = ld(x + (r0 + r) * 1024 + u * 256 + tid);
  __shared__ f4v lds[L > 0 ? L : 1][4][256];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(x + (r0 + R + l) * 1024 + u * 256 + tid);
#pragma unroll
    for (int u = 0; u < 4; ++u) { lds[l][u][tid] = v[u]; acc(v[u], lo, hi); }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc(reg[r][u], lo, hi);
  block_mm(lo, hi);
  if (tid == 0) {
    __hip_atomic_store(part + b, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + G + b, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 100000;  // 1 ms at 100 MHz
    while ((int)(__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() > t_end) {
        __hip_atomic_fetch_add(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  lo = ~0u; hi = 0;
  for (unsigned i = tid; i < G; i += 256) {
    lo = min(lo, __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    hi = max(hi, __hip_atomic_load(part + G + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  block_mm(lo, hi);
  const float mn = unkey(lo), sc = 254.0f / (unkey(hi) - mn);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_nontemporal_store(q4(reg[r][u], mn, sc), y + (r0 + r) * 1024 + u * 256 + tid);
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_nontemporal_store(q4(lds[l][u][tid], mn, sc), y + (r0 + R + l) * 1024 + u * 256 + tid);
  for (size_t k = 0; k < s1 - s0; ++k) {
    const size_t t = REV ? s1 - 1 - k : s0 + k;
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(x + t * 1024 + u * 256 + tid);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(q4(v[u], mn, sc), y + t * 1024 + u * 256 + tid);
  }
}

int main() {
  const size_t n = 1ull << 27, ntiles = n / 4096;
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  f4v* x[3];
  for (int i = 0; i < 3; ++i) {
    CK(hipMalloc(&x[i], n * 4));
    CK(hipMemset(x[i], 0x3f + i, n * 4));
  }
  uint32_t *y, *part;
  unsigned *bar, *tmo;
  CK(hipMalloc(&y, n));
  CK(hipMalloc(&part, 1 << 16));
  CK(hipMalloc(&bar, 256));
  CK(hipMemset(bar, 0, 256));
  tmo = bar + 16;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 30;
  unsigned target = 0;
  auto run_two = [&](int i) {
    hipLaunchKernelGGL(k_minmax, dim3(1024), dim3(256), 0, 0, x[i % 3], ntiles, part);
    hipLaunchKernelGGL(k_encode, dim3(8192), dim3(256), 0, 0, x[i % 3], y, ntiles, part, 1024);
  };
  auto time = [&](const char* name, auto&& f) {
    for (int i = 0; i < 6; ++i) f(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) f(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned t = 0;
    CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
    printf("%-28s %8.2f us  (9n bytes: %.2f TB/s)  timeouts %u\n", name, ms * 1e3 / iters,
           9.0 * n / (ms * 1e-3 / iters) * 1e-12, t);
  };
  time("two kernels", run_two);
#define FUSED(R, L, REV)                                                                                   \
  {                                                                                                         \
    int occ = 0;                                                                                            \
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused<R, L, REV>, 256, 0));                     \
    const int per_cu = occ < 2 ? occ : 2;                                                                   \
    const unsigned G = per_cu * ncu;                                                                        \
    char nm[64];                                                                                            \
    snprintf(nm, sizeof nm, "fused R=%d L=%d rev=%d occ=%d", R, L, (int)REV, occ);                           \
    if (per_cu >= 1)                                                                                        \
      time(nm, [&](int i) {                                                                                 \
        target += G;                                                                                        \
        hipLaunchKernelGGL((k_fused<R, L, REV>), dim3(G), dim3(256), 0, 0, x[i % 3], y, ntiles, bar, target, \
                           part, tmo);                                                                      \
      });                                                                                                   \
  }
  FUSED(0, 0, false)
  FUSED(8, 0, false)
  FUSED(8, 4, false)
  FUSED(8, 4, true)
  FUSED(12, 4, false)
  FUSED(12, 4, true)
  FUSED(12, 2, true)
  time("two kernels", run_two);
  return 0;
}
