// C3-shape probe: where a 10M-value single-array encode's time goes.
// Each iteration runs a min/max read pass over array i (of 3 rotating 40 MB
// f32 arrays) and then one variant kernel over the same array; run under
// `rocprofv3 --kernel-trace --stats` and read each variant's average.
//   v_copy     one tile per workgroup: 16 values per lane in, one byte each
//              out (v * s), nothing else: the floor of the read + write shape
//   v_lcg      + the LCG-bit table words per group (as encode_full_tile)
//   v_fold     + the partials fold (1024 pairs) and the f64 quantiser constants
//   v_full     + the guard-band floor and the band test (the real tile math)
//   v_dec      the decode's shape: 10 MB of codes in, 40 MB of floats out
//   tpw<k>     v_full with k tiles per workgroup (grid ntiles / k)
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/c3enc_probe tools/c3enc_probe.hip
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

template <bool NT>
__device__ __forceinline__ f4v ld(const f4v* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

__global__ __launch_bounds__(256) void k_minmax(const f4v* __restrict__ x, size_t ntiles, uint32_t* part) {
  uint32_t lo = ~0u, hi = 0;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld<true>(x + t * 1024 + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  for (int o = 32; o; o >>= 1) { lo = min(lo, (uint32_t)__shfl_xor((int)lo, o)); hi = max(hi, (uint32_t)__shfl_xor((int)hi, o)); }
  __shared__ uint32_t sl[4], sh[4];
  if ((threadIdx.x & 63) == 0) { sl[threadIdx.x >> 6] = lo; sh[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = min(min(sl[0], sl[1]), min(sl[2], sl[3]));
    part[gridDim.x + blockIdx.x] = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
  }
}

__global__ __launch_bounds__(256) void k_minmax_t(const f4v* __restrict__ x, size_t ntiles, uint32_t* part) {
  uint32_t lo = ~0u, hi = 0;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld<false>(x + t * 1024 + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t a = key(v[u].x), b = key(v[u].y), c = key(v[u].z), d = key(v[u].w);
      lo = min(lo, min(min(a, b), min(c, d)));
      hi = max(hi, max(max(a, b), max(c, d)));
    }
  }
  if ((lo ^ hi) == 0x12345678u) part[blockIdx.x] = lo;
}

struct P {
  const uint32_t* part;
  int nparts;
  const uint32_t* bits;
  uint32_t pos;
  double ratio;
};

// MODE 0 copy, 1 + lcg, 2 + fold, 3 full
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k_enc(const f4v* __restrict__ x, uint32_t* __restrict__ y, size_t ntiles, P p) {
  const size_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  const size_t t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  if (t0 >= t1) return;
  f4v first[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) first[u] = ld<NT>(x + t0 * 1024 + u * 256 + threadIdx.x);
  float mn = -4.f, mx = 4.f, sc = 31.75f;
  bool fast = true;
  if (MODE >= 2) {
    uint32_t lo = ~0u, hi = 0;
    for (int i = threadIdx.x; i < p.nparts; i += 256) { lo = min(lo, p.part[i]); hi = max(hi, p.part[p.nparts + i]); }
    for (int o = 32; o; o >>= 1) { lo = min(lo, (uint32_t)__shfl_xor((int)lo, o)); hi = max(hi, (uint32_t)__shfl_xor((int)hi, o)); }
    __shared__ uint32_t sl[4], sh[4];
    if ((threadIdx.x & 63) == 0) { sl[threadIdx.x >> 6] = lo; sh[threadIdx.x >> 6] = hi; }
    __syncthreads();
    lo = min(min(sl[0], sl[1]), min(sl[2], sl[3]));
    hi = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
    mn = unkey(lo);
    mx = (float)((double)unkey(hi) + 1e-6);
    const double bin = (double)mx - (double)mn;
    const double s = p.ratio / bin;
    sc = (float)s;
    fast = bin < __builtin_huge_val();
  }
  for (size_t t = t0; t < t1; ++t) {
    f4v v[4];
    if (t == t0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = first[u];
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld<NT>(x + t * 1024 + u * 256 + threadIdx.x);
    }
    const size_t gb = t * 1024 + threadIdx.x;
    uint32_t b4[4] = {0, 0, 0, 0};
    if (MODE >= 1) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = (p.pos + 1u + 4u * (uint32_t)(gb + u * 256)) & 0x1FFFFu;
        const uint2 w = *reinterpret_cast<const uint2*>(p.bits + (k >> 5));
        b4[u] = __builtin_amdgcn_alignbit(w.y, w.x, k & 31u) & 0xFu;
      }
    }
    uint32_t w[4];
    uint32_t lo = 0x7F800000u, hi = 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t acc = 0;
      float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MODE >= 3) {
          const float t = (__builtin_amdgcn_fmed3f(e[j], mn, mx) - mn) * sc;
          const float f = floorf(t);
          const uint32_t fr = __float_as_uint(t - f);
          lo = min(lo, fr);
          hi = max(hi, fr);
          acc = __builtin_amdgcn_cvt_pk_u8_f32(f, j, acc);
        } else {
          acc = __builtin_amdgcn_cvt_pk_u8_f32((e[j] - mn) * sc, j, acc);
        }
      }
      w[u] = acc;
    }
    if (MODE >= 3) {
      const bool ok = fast && lo > 0x38800000u && hi < 0x3F7FFC00u;
      if (!ok) w[0] ^= 1u;  // stand-in for the exact redo (never taken with these inputs' shape)
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) y[gb + u * 256] = w[u] + ((b4[u] * 0x204081u) & 0x01010101u);
  }
}

__global__ __launch_bounds__(256) void k_dec(const uint32_t* __restrict__ c, f4v* __restrict__ y, size_t ntiles) {
  __shared__ float tab[256];
  tab[threadIdx.x] = (float)((double)threadIdx.x * (8.0 / 254.0) - 4.0);
  __syncthreads();
  const size_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  const size_t t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = c[t * 1024 + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f4v o = {tab[w[u] & 255], tab[(w[u] >> 8) & 255], tab[(w[u] >> 16) & 255], tab[w[u] >> 24]};
      __builtin_nontemporal_store(o, y + t * 1024 + u * 256 + threadIdx.x);
    }
  }
}

int main(int argc, char** argv) {
  const size_t n = 10000000 / 4096 * 4096;  // full tiles only
  const size_t ntiles = n / 4096;
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int NA = 3, NPART = 1024;
  f4v* xs[NA];
  uint32_t *codes, *part, *bits;
  f4v* dec;
  float* h = (float*)malloc(n * 4);
  for (size_t i = 0; i < n; ++i) h[i] = (float)((int)((i * 2654435761u) >> 8) % 8000) / 1000.0f - 4.0f;
  for (int i = 0; i < NA; ++i) { CK(hipMalloc(&xs[i], n * 4)); CK(hipMemcpy(xs[i], h, n * 4, hipMemcpyHostToDevice)); }
  CK(hipMalloc(&codes, n)); CK(hipMalloc(&dec, n * 4)); CK(hipMalloc(&part, 2 * NPART * 4));
  CK(hipMalloc(&bits, (1 << 17) / 8 + 64)); CK(hipMemset(bits, 0x5a, (1 << 17) / 8 + 64));
  P p{part, NPART, bits, 12345, 254.0};
  const int g1 = (int)ntiles;
  printf("n %zu ntiles %zu\n", n, ntiles);
  auto mm = [&](int i) { hipLaunchKernelGGL(k_minmax, dim3(NPART), dim3(256), 0, 0, xs[i], ntiles, part); };
  auto run = [&](const char* name, auto kern, int grid, auto a0, auto a1, bool enc) {
    for (int it = 0; it < iters; ++it) {
      const int i = it % NA;
      mm(i);
      if (enc) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a0 ? a0 : xs[i], a1, ntiles, p);
    }
    CK(hipDeviceSynchronize());
    printf("%s done\n", name);
  };
  run("copy", k_enc<0, true>, g1, (f4v*)nullptr, codes, true);
  // the copy over the array the min/max pass did NOT just read (Infinity Cache cold for it)
  for (int it = 0; it < iters; ++it) {
    const int i = it % NA;
    mm(i);
    hipLaunchKernelGGL((k_enc<0, false>), dim3(g1), dim3(256), 0, 0, xs[(i + 1) % NA], codes, ntiles, p);
  }
  CK(hipDeviceSynchronize());
  // min/max with temporal loads, then the copy (cached loads) over the same array
  for (int it = 0; it < iters; ++it) {
    const int i = it % NA;
    hipLaunchKernelGGL(k_minmax_t, dim3(NPART), dim3(256), 0, 0, xs[i], ntiles, part);
    hipLaunchKernelGGL((k_enc<1, false>), dim3(g1), dim3(256), 0, 0, xs[i], codes, ntiles, p);
  }
  CK(hipDeviceSynchronize());
  run("lcg", k_enc<1, true>, g1, (f4v*)nullptr, codes, true);
  run("fold", k_enc<2, true>, g1, (f4v*)nullptr, codes, true);
  run("full", k_enc<3, true>, g1, (f4v*)nullptr, codes, true);
  run("full_t", k_enc<3, false>, g1, (f4v*)nullptr, codes, true);
  run("copy_t", k_enc<0, false>, g1, (f4v*)nullptr, codes, true);
  run("tpw2", k_enc<2, true>, (g1 + 1) / 2, (f4v*)nullptr, codes, true);
  for (int it = 0; it < iters; ++it) {
    mm(it % NA);
    hipLaunchKernelGGL(k_dec, dim3(g1), dim3(256), 0, 0, codes, dec, ntiles);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
