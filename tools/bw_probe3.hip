// Probe 3: an emulated FIXING_FLOAT round-trip step (minmax -> encode ->
// decode) over rotating inputs, to pick cache policies for the real kernels.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bw_probe3 tools/bw_probe3.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t q8(float v) { return (uint32_t)(int)(v * 3.0f + 100.0f) & 255; }

template <bool NT_LOAD>
__global__ __launch_bounds__(256) void k_minmax(const f4v* __restrict__ x, size_t ntiles, uint32_t* out) {
  uint32_t lo = ~0u, hi = 0;
  size_t per = (ntiles + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = NT_LOAD ? __builtin_nontemporal_load(x + t * 1024 + u * 256 + threadIdx.x) : x[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  if ((lo ^ hi) == 0x12345678u) out[0] = lo;
}

template <bool REV, bool NT_LOAD>
__global__ __launch_bounds__(256) void k_encode(const f4v* __restrict__ x, uint32_t* __restrict__ y, size_t ntiles) {
  size_t per = (ntiles + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t k = 0; t0 < t1 && k < t1 - t0; ++k) {
    size_t t = REV ? (t1 - 1 - k) : (t0 + k);
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = NT_LOAD ? __builtin_nontemporal_load(x + t * 1024 + u * 256 + threadIdx.x) : x[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      y[t * 1024 + u * 256 + threadIdx.x] = q8(v[u].x) | (q8(v[u].y) << 8) | (q8(v[u].z) << 16) | (q8(v[u].w) << 24);
  }
}

template <bool NT_STORE, bool NT_LOAD = false>
__global__ __launch_bounds__(256) void k_decode(const uint32_t* __restrict__ c, f4v* __restrict__ y, size_t ntiles) {
  size_t per = (ntiles + gridDim.x - 1) / gridDim.x, t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = NT_LOAD ? __builtin_nontemporal_load(c + t * 1024 + u * 256 + threadIdx.x) : c[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f4v v = {(float)(w[u] & 255), (float)((w[u] >> 8) & 255), (float)((w[u] >> 16) & 255), (float)(w[u] >> 24)};
      if (NT_STORE) __builtin_nontemporal_store(v, y + t * 1024 + u * 256 + threadIdx.x);
      else y[t * 1024 + u * 256 + threadIdx.x] = v;
    }
  }
}

int main() {
  const size_t n = 1ull << 27;
  const size_t ntiles = n / 4096;
  const int NB = 3;
  f4v* xs[NB]; f4v* y; uint32_t *c, *o;
  for (int i = 0; i < NB; ++i) { CK(hipMalloc(&xs[i], n * 4)); CK(hipMemset(xs[i], 0x3f + i, n * 4)); }
  CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&c, n)); CK(hipMalloc(&o, 64));
  hipEvent_t ev[4];
  for (int i = 0; i < 4; ++i) CK(hipEventCreate(&ev[i]));
  struct V { const char* name; bool mm_nt, enc_rev, enc_nt, dec_ntld, dec_ntst; };
  V vs[] = {
      {"plain", false, false, false, false, false},
      {"encREV+encNT+decNTst (prev best)", false, true, true, false, true},
      {"encNT+decNTst (fwd)", false, false, true, false, true},
      {"encREV+encNT (dec plain)", false, true, true, false, false},
      {"mmNT+encREV+encNT+decNTst", true, true, true, false, true},
      {"encREV+encNT+decNTld+decNTst", false, true, true, true, true},
      {"mmNT+encREV+encNT+decNTld+decNTst", true, true, true, true, true},
  };
  for (const V& v : vs) {
    float tm = 0, te = 0, td = 0;
    const int steps = 40, warm = 8;
    for (int s = 0; s < steps; ++s) {
      const f4v* x = xs[s % NB];
      CK(hipEventRecord(ev[0]));
      if (v.mm_nt) k_minmax<true><<<1024, 256>>>(x, ntiles, o); else k_minmax<false><<<1024, 256>>>(x, ntiles, o);
      CK(hipEventRecord(ev[1]));
      if (v.enc_rev && v.enc_nt) k_encode<true, true><<<4096, 256>>>(x, c, ntiles);
      else if (v.enc_rev) k_encode<true, false><<<4096, 256>>>(x, c, ntiles);
      else if (v.enc_nt) k_encode<false, true><<<4096, 256>>>(x, c, ntiles);
      else k_encode<false, false><<<4096, 256>>>(x, c, ntiles);
      CK(hipEventRecord(ev[2]));
      if (v.dec_ntst && v.dec_ntld) k_decode<true, true><<<4096, 256>>>(c, y, ntiles);
      else if (v.dec_ntst) k_decode<true, false><<<4096, 256>>>(c, y, ntiles);
      else if (v.dec_ntld) k_decode<false, true><<<4096, 256>>>(c, y, ntiles);
      else k_decode<false, false><<<4096, 256>>>(c, y, ntiles);
      CK(hipEventRecord(ev[3]));
      CK(hipEventSynchronize(ev[3]));
      float a, b, d;
      CK(hipEventElapsedTime(&a, ev[0], ev[1]));
      CK(hipEventElapsedTime(&b, ev[1], ev[2]));
      CK(hipEventElapsedTime(&d, ev[2], ev[3]));
      if (s >= warm) { tm += a; te += b; td += d; }
    }
    const int k = steps - warm;
    double tot = (tm + te + td) / k;
    printf("%-40s minmax %6.1f us  encode %6.1f us  decode %6.1f us  step %6.1f us  -> %6.1f GB/s of 14n bytes\n",
           v.name, tm / k * 1e3, te / k * 1e3, td / k * 1e3, tot * 1e3, 14.0 * n / (tot * 1e-3) / 1e9);
  }
  return 0;
}
