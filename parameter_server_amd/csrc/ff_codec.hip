// FIXING_FLOAT codec kernels for gfx950 (CDNA4).
//
// Restates FixingFloatFilter::convert<V> (reference src/filter/fixing_float.h:50-101)
// as three HBM-streaming kernels:
//
//   ff_minmax_partials  pass 1 of encode when min/max are not preset
//                       (fixing_float.h:57-64): per-workgroup min/max of the
//                       value array as order-preserving integer keys.
//   ff_encode           pass 2 (fixing_float.h:73-88): every workgroup first folds
//                       the <= kMaxGrid partials (8-16 KiB, L2-resident), derives
//                       min/max/bin exactly as the reference, then quantises
//                       4 values per lane with the stochastic-rounding LCG bit
//                       (fixing_float.h:18-21) reproduced by affine jump-ahead.
//   ff_decode           fixing_float.h:89-101; nb==1 uses a 256-entry LDS table
//                       built with the same double formula (bit-identical).
//
// Bit-exactness rules: IEEE double division (hipcc's
// default f64 fdiv lowering is correctly rounded), NO FMA contraction (this file
// is compiled with -ffp-contract=off), clamp on the double-promoted value, the
// x86 double->uint64 cast semantics for the degenerate nb>=4 ratios.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psf_internal.h"

namespace psf {

// ------------------------------------------------------------ helpers ------
__device__ __forceinline__ uint32_t f32_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_f32(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t f64_key(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_f64(uint64_t k) {
  uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

template <typename V> struct KeyOf;
template <> struct KeyOf<float> {
  typedef uint32_t K;
  static constexpr uint32_t kLoId = 0xFFFFFFFFu;  // min identity (above every key)
  static constexpr uint32_t kHiId = 0u;           // max identity
  __device__ static K key(float v) { return f32_key(v); }
};
template <> struct KeyOf<double> {
  typedef uint64_t K;
  static constexpr uint64_t kLoId = 0xFFFFFFFFFFFFFFFFull;
  static constexpr uint64_t kHiId = 0ull;
  __device__ static K key(double v) { return f64_key(v); }
};

template <typename K> __device__ __forceinline__ K wave_min(K v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    K w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
template <typename K> __device__ __forceinline__ K wave_max(K v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    K w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// Block-wide (256 threads = 4 waves) min/max of keys; result valid in all threads.
template <typename K>
__device__ __forceinline__ void block_minmax(K& lo, K& hi) {
  __shared__ K s_lo[kBlock / 64], s_hi[kBlock / 64];
  lo = wave_min(lo);
  hi = wave_max(hi);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
  __syncthreads();
  lo = s_lo[0]; hi = s_hi[0];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) {
    lo = s_lo[w] < lo ? s_lo[w] : lo;
    hi = s_hi[w] > hi ? s_hi[w] : hi;
  }
  __syncthreads();
}

// 4-element vector load of V.
template <typename V> struct Vec4;
template <> struct Vec4<float> {
  __device__ static void load(const float* p, float v[4]) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static void store(float* p, const float v[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<double> {
  __device__ static void load(const double* p, double v[4]) {
    double2 a = reinterpret_cast<const double2*>(p)[0];
    double2 b = reinterpret_cast<const double2*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ static void store(double* p, const double v[4]) {
    reinterpret_cast<double2*>(p)[0] = make_double2(v[0], v[1]);
    reinterpret_cast<double2*>(p)[1] = make_double2(v[2], v[3]);
  }
};

// ------------------------------------------------------ pass 1: min/max ----
// partials layout: K lo[grid], K hi[grid].
template <typename V, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_minmax_partials(const V* __restrict__ x, size_t n,
                                                              void* __restrict__ partials) {
  typedef typename KeyOf<V>::K K;
  K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t nthreads = (size_t)gridDim.x * kBlock;
  if (kVec) {
    const size_t ngroups = n >> 2;
    size_t g = tid;
    // 4 groups (16 values) in flight per lane per iteration
    for (; g + 3 * nthreads < ngroups; g += 4 * nthreads) {
      V v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) Vec4<V>::load(x + 4 * (g + u * nthreads), v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          V e = v[u][j];
          if (e == e) {
            K k = KeyOf<V>::key(e);
            lo = k < lo ? k : lo;
            hi = k > hi ? k : hi;
          }
        }
    }
    for (; g < ngroups; g += nthreads) {
      V v[4];
      Vec4<V>::load(x + 4 * g, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        V e = v[j];
        if (e == e) {
          K k = KeyOf<V>::key(e);
          lo = k < lo ? k : lo;
          hi = k > hi ? k : hi;
        }
      }
    }
    for (size_t i = (ngroups << 2) + tid; i < n; i += nthreads) {
      V e = x[i];
      if (e == e) {
        K k = KeyOf<V>::key(e);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
      }
    }
  } else {
    for (size_t i = tid; i < n; i += nthreads) {
      V e = x[i];
      if (e == e) {
        K k = KeyOf<V>::key(e);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
      }
    }
  }
  block_minmax(lo, hi);
  if (threadIdx.x == 0) {
    K* p = reinterpret_cast<K*>(partials);
    p[blockIdx.x] = lo;
    p[gridDim.x + blockIdx.x] = hi;
  }
}

// Fold the partials (every workgroup of the encode kernel does this; the
// partials are <= 2*kMaxGrid keys and stay in L2).  Returns min/max in the
// reference's FilterConfig representation (float), fixing_float.h:57-64.
template <typename V>
__device__ __forceinline__ void fold_partials(const void* partials, int nparts, float& mn_f,
                                              float& mx_f) {
  typedef typename KeyOf<V>::K K;
  const K* p = reinterpret_cast<const K*>(partials);
  K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
  for (int i = threadIdx.x; i < nparts; i += kBlock) {
    K a = p[i], b = p[nparts + i];
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  block_minmax(lo, hi);
  if (sizeof(V) == 4) {
    // all-NaN / empty: lo stays at the identity, which decodes to a NaN
    float lo_v = key_f32((uint32_t)lo), hi_v = key_f32((uint32_t)hi);
    mn_f = lo_v;
    mx_f = (float)((double)hi_v + 1e-6);
  } else {
    double lo_v = key_f64((uint64_t)lo), hi_v = key_f64((uint64_t)hi);
    mn_f = (float)lo_v;
    mx_f = (float)(hi_v + 1e-6);
  }
}

// x86-64 g++ lowering of static_cast<uint64>(double) for the values that can
// arise here (|d| < 2^63 or NaN): negatives wrap through int64, NaN's low 56
// bits are zero.
__device__ __forceinline__ uint64_t x86_d2u64(double d) {
  if (d != d) return 0;
  return (uint64_t)(int64_t)d;
}

// ------------------------------------------------------ pass 2: encode -----
struct EncodeParams {
  const void* partials;   // null when both min and max are preset
  int nparts;
  int has_min, has_max;
  float preset_min, preset_max;
  uint32_t seed;
  uint32_t jump_a, jump_c;  // LCG affine map for 4*nthreads steps
  double ratio;
  float* range_out;       // device float[2] side-info, may be null
  int* status_out;        // device int, may be null
};

// s -> a*s + c, composed k times, k < 2^63.
__device__ __forceinline__ uint32_t lcg_jump(uint32_t s, uint64_t k) {
  uint32_t a = kLcgA, c = kLcgC;
  while (k) {
    if (k & 1) s = a * s + c;
    c = a * c + c;
    a = a * a;
    k >>= 1;
  }
  return s;
}

template <int NB>
__device__ __forceinline__ void store_codes(uint8_t* __restrict__ out, size_t g, const uint64_t r[4]) {
  if (NB == 1) {
    uint32_t w = (uint32_t)(r[0] & 0xFF) | ((uint32_t)(r[1] & 0xFF) << 8) |
                 ((uint32_t)(r[2] & 0xFF) << 16) | ((uint32_t)(r[3] & 0xFF) << 24);
    __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(out) + g);
  } else if (NB == 2) {
    uint32_t w0 = (uint32_t)(r[0] & 0xFFFF) | ((uint32_t)(r[1] & 0xFFFF) << 16);
    uint32_t w1 = (uint32_t)(r[2] & 0xFFFF) | ((uint32_t)(r[3] & 0xFFFF) << 16);
    reinterpret_cast<uint2*>(out)[g] = make_uint2(w0, w1);
  } else if (NB == 3) {
    uint32_t a = (uint32_t)r[0] & 0xFFFFFF, b = (uint32_t)r[1] & 0xFFFFFF;
    uint32_t c = (uint32_t)r[2] & 0xFFFFFF, d = (uint32_t)r[3] & 0xFFFFFF;
    uint32_t* o = reinterpret_cast<uint32_t*>(out) + 3 * g;
    o[0] = a | (b << 24);
    o[1] = (b >> 8) | (c << 16);
    o[2] = (c >> 16) | (d << 8);
  } else {
    uint8_t* o = out + (size_t)NB * 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint64_t v = r[e];
#pragma unroll
      for (int j = 0; j < NB; ++j) { o[e * NB + j] = (uint8_t)(v & 0xFF); v >>= 8; }
    }
  }
}

template <typename V, int NB>
__device__ __forceinline__ uint64_t quantize(V xv, double min_v, double max_v, double bin,
                                            double ratio, uint32_t& s) {
  double x = (double)xv;
  double proj = x > max_v ? max_v : (x < min_v ? min_v : x);
  double tmp = (proj - min_v) / bin * ratio;
  s = kLcgA * s + kLcgC;
  uint64_t bit = ((s >> 16) & 1u) == 0u ? 1u : 0u;
  uint64_t q;
  if (NB <= 3) {
    // ratio > 0 and proj >= min_v: tmp is in [0, ratio] or NaN
    q = (tmp == tmp) ? (uint64_t)(uint32_t)floor(tmp) : 0;
  } else {
    q = x86_d2u64(floor(tmp));
  }
  return q + bit;
}

template <typename V, int NB, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_encode(const V* __restrict__ x, size_t n,
                                                     uint8_t* __restrict__ out, EncodeParams p) {
  __shared__ float s_range[2];
  float mn_f = p.preset_min, mx_f = p.preset_max;
  if (p.partials != nullptr) {
    float cmn, cmx;
    fold_partials<V>(p.partials, p.nparts, cmn, cmx);
    if (!p.has_min) mn_f = cmn;
    if (!p.has_max) mx_f = cmx;
  }
  (void)s_range;
  const double min_v = (double)mn_f, max_v = (double)mx_f;
  const double bin = max_v - min_v;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (p.range_out) { p.range_out[0] = mn_f; p.range_out[1] = mx_f; }
    if (p.status_out) *p.status_out = (bin > 0) ? kOk : kErrBin;
  }
  if (!(bin > 0)) return;  // CHECK_GT(bin, 0), fixing_float.h:71
  const double ratio = p.ratio;

  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t nthreads = (size_t)gridDim.x * kBlock;
  if (kVec) {
    const size_t ngroups = n >> 2;
    // state before element 4g is s_{4g}; element i consumes s_{i+1}
    uint32_t s = lcg_jump(p.seed, 4 * tid);
    for (size_t g = tid; g < ngroups; g += nthreads) {
      V v[4];
      Vec4<V>::load(x + 4 * g, v);
      uint64_t r[4];
      uint32_t t = s;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = quantize<V, NB>(v[j], min_v, max_v, bin, ratio, t);
      store_codes<NB>(out, g, r);
      s = p.jump_a * s + p.jump_c;
    }
    // ragged tail (< 4 elements): one thread
    const size_t tail = ngroups << 2;
    if (tid == 0 && tail < n) {
      uint32_t t = lcg_jump(p.seed, tail);
      for (size_t i = tail; i < n; ++i) {
        uint64_t r = quantize<V, NB>(x[i], min_v, max_v, bin, ratio, t);
        for (int j = 0; j < NB; ++j) { out[i * NB + j] = (uint8_t)(r & 0xFF); r >>= 8; }
      }
    }
  } else {
    // unaligned input: scalar path, one element per lane per step
    uint32_t s = lcg_jump(p.seed, tid);
    const uint32_t ja = p.jump_a, jc = p.jump_c;  // here: affine map for nthreads steps
    for (size_t i = tid; i < n; i += nthreads) {
      uint32_t t = s;
      uint64_t r = quantize<V, NB>(x[i], min_v, max_v, bin, ratio, t);
      for (int j = 0; j < NB; ++j) { out[i * NB + j] = (uint8_t)(r & 0xFF); r >>= 8; }
      s = ja * s + jc;
    }
  }
}

// ------------------------------------------------------------- decode ------
struct DecodeParams {
  const float* range;     // device float[2] or null -> use (mn, mx)
  float mn, mx;
  double ratio;
};

template <typename V>
__device__ __forceinline__ V dequant(uint64_t code, double ratio, double bin, double min_v) {
  double r = (double)code;
  return (V)(r / ratio * bin + min_v);
}

template <typename V, int NB, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_decode(const uint8_t* __restrict__ code, size_t n,
                                                     V* __restrict__ out, DecodeParams p) {
  float mn_f = p.mn, mx_f = p.mx;
  if (p.range) { mn_f = p.range[0]; mx_f = p.range[1]; }
  const double min_v = (double)mn_f, max_v = (double)mx_f;
  const double bin = max_v - min_v;
  const double ratio = p.ratio;
  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t nthreads = (size_t)gridDim.x * kBlock;

  if (NB == 1 && kVec) {
    // 256-entry table, same formula => bit-identical to the per-element path
    __shared__ V lut[256];
    lut[threadIdx.x] = dequant<V>((uint64_t)threadIdx.x, ratio, bin, min_v);
    __syncthreads();
    const size_t ngroups = n >> 2;
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(code);
    size_t g = tid;
    for (; g + 3 * nthreads < ngroups; g += 4 * nthreads) {
      uint32_t w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = __builtin_nontemporal_load(c32 + g + u * nthreads);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        V v[4] = {lut[w[u] & 0xFF], lut[(w[u] >> 8) & 0xFF], lut[(w[u] >> 16) & 0xFF], lut[w[u] >> 24]};
        Vec4<V>::store(out + 4 * (g + u * nthreads), v);
      }
    }
    for (; g < ngroups; g += nthreads) {
      uint32_t w = c32[g];
      V v[4] = {lut[w & 0xFF], lut[(w >> 8) & 0xFF], lut[(w >> 16) & 0xFF], lut[w >> 24]};
      Vec4<V>::store(out + 4 * g, v);
    }
    for (size_t i = (ngroups << 2) + tid; i < n; i += nthreads) out[i] = lut[code[i]];
    return;
  }

  if (kVec && (NB == 2 || NB == 3)) {
    const size_t ngroups = n >> 2;
    for (size_t g = tid; g < ngroups; g += nthreads) {
      uint64_t r[4];
      if (NB == 2) {
        uint2 w = reinterpret_cast<const uint2*>(code)[g];
        r[0] = w.x & 0xFFFF; r[1] = w.x >> 16; r[2] = w.y & 0xFFFF; r[3] = w.y >> 16;
      } else {
        const uint32_t* c = reinterpret_cast<const uint32_t*>(code) + 3 * g;
        uint32_t a = c[0], b = c[1], d = c[2];
        r[0] = a & 0xFFFFFF;
        r[1] = (a >> 24) | ((b & 0xFFFF) << 8);
        r[2] = (b >> 16) | ((d & 0xFF) << 16);
        r[3] = d >> 8;
      }
      V v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = dequant<V>(r[j], ratio, bin, min_v);
      Vec4<V>::store(out + 4 * g, v);
    }
    for (size_t i = (ngroups << 2) + tid; i < n; i += nthreads) {
      uint64_t r = 0;
      for (int j = 0; j < NB; ++j) r |= (uint64_t)code[i * NB + j] << (8 * j);
      out[i] = dequant<V>(r, ratio, bin, min_v);
    }
    return;
  }

  // generic byte path (nb >= 4, or unaligned buffers)
  for (size_t i = tid; i < n; i += nthreads) {
    uint64_t r = 0;
    for (int j = 0; j < NB; ++j) r |= (uint64_t)code[i * NB + j] << (8 * j);
    out[i] = dequant<V>(r, ratio, bin, min_v);
  }
}

// ------------------------------------------------------------ launchers ----
static inline void lcg_affine_pow(uint64_t k, uint32_t& A, uint32_t& Cc) {
  uint32_t a = kLcgA, c = kLcgC;
  A = 1u; Cc = 0u;
  while (k) {
    if (k & 1) { A = a * A; Cc = a * Cc + c; }
    c = a * c + c;
    a = a * a;
    k >>= 1;
  }
}

double ff_ratio(int nb) {
  // fixing_float.h:55 -- 32-bit int shift, count masked to 5 bits on x86
  int32_t one_shifted = (int32_t)(1u << ((unsigned)(nb * 8) & 31u));
  return (double)one_shifted - 2.0;
}

int ff_grid(size_t work_items) {
  size_t g = (work_items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > (size_t)kMaxGrid) g = kMaxGrid;
  return (int)g;
}

template <typename V, int NB, bool kVec>
static void launch_encode(const V* x, size_t n, uint8_t* out, EncodeParams p, hipStream_t st) {
  const size_t items = kVec ? (n >> 2) : n;
  const int grid = ff_grid(items);
  const uint64_t stride = (uint64_t)grid * kBlock * (kVec ? 4 : 1);
  lcg_affine_pow(stride, p.jump_a, p.jump_c);
  hipLaunchKernelGGL((ff_encode<V, NB, kVec>), dim3(grid), dim3(kBlock), 0, st, x, n, out, p);
}

template <typename V, bool kVec>
static int dispatch_encode_nb(const V* x, size_t n, int nb, uint8_t* out, const EncodeParams& p,
                              hipStream_t st) {
  switch (nb) {
    case 1: launch_encode<V, 1, kVec>(x, n, out, p, st); break;
    case 2: launch_encode<V, 2, kVec>(x, n, out, p, st); break;
    case 3: launch_encode<V, 3, kVec>(x, n, out, p, st); break;
    case 4: launch_encode<V, 4, kVec>(x, n, out, p, st); break;
    case 5: launch_encode<V, 5, kVec>(x, n, out, p, st); break;
    case 6: launch_encode<V, 6, kVec>(x, n, out, p, st); break;
    case 7: launch_encode<V, 7, kVec>(x, n, out, p, st); break;
    default: return kErrNbytes;
  }
  return kOk;
}

template <typename V>
static int encode_typed(const V* x, size_t n, int nb, const FixedPoint& preset, uint32_t seed,
                        uint8_t* out, void* partials, float* range_out, int* status_out,
                        hipStream_t st, Profiler* prof) {
  EncodeParams p{};
  p.has_min = preset.has_min;
  p.has_max = preset.has_max;
  p.preset_min = preset.min_value;
  p.preset_max = preset.max_value;
  p.seed = seed;
  p.ratio = ff_ratio(nb);
  p.range_out = range_out;
  p.status_out = status_out;
  // 16-byte alignment of the input and 4-byte alignment of the output
  const bool vec = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & (nb == 2 ? 7 : 3)) == 0);
  if (!(preset.has_min && preset.has_max)) {
    const size_t items = vec ? (n >> 2) : n;
    const int grid = ff_grid(items);
    ProfScope ps(prof, kKMinmax, st, (double)n * sizeof(V));
    if (vec)
      hipLaunchKernelGGL((ff_minmax_partials<V, true>), dim3(grid), dim3(kBlock), 0, st, x, n, partials);
    else
      hipLaunchKernelGGL((ff_minmax_partials<V, false>), dim3(grid), dim3(kBlock), 0, st, x, n, partials);
    p.partials = partials;
    p.nparts = grid;
    if (launch_status() != kOk) return kErrHip;
  }
  ProfScope ps(prof, kKEncode, st, (double)n * (sizeof(V) + nb));
  int s = vec ? dispatch_encode_nb<V, true>(x, n, nb, out, p, st)
              : dispatch_encode_nb<V, false>(x, n, nb, out, p, st);
  return s == kOk ? launch_status() : s;
}

int ff_encode_launch(const void* x, size_t n, int value_type, int nb, const FixedPoint& preset,
                     uint32_t seed, void* out, void* partials, float* range_out, int* status_out,
                     hipStream_t st, Profiler* prof) {
  if (nb <= 0 || nb >= 8) return kErrNbytes;
  if (n == 0) return kOk;
  if (value_type == kFloat)
    return encode_typed<float>(static_cast<const float*>(x), n, nb, preset, seed,
                               static_cast<uint8_t*>(out), partials, range_out, status_out, st, prof);
  if (value_type == kDouble)
    return encode_typed<double>(static_cast<const double*>(x), n, nb, preset, seed,
                                static_cast<uint8_t*>(out), partials, range_out, status_out, st, prof);
  return kErrArg;
}

template <typename V, int NB, bool kVec>
static void launch_decode(const uint8_t* code, size_t n, V* out, const DecodeParams& p,
                          hipStream_t st) {
  const size_t items = kVec ? (n >> 2) : n;
  const int grid = ff_grid(items);
  hipLaunchKernelGGL((ff_decode<V, NB, kVec>), dim3(grid), dim3(kBlock), 0, st, code, n, out, p);
}

template <typename V, bool kVec>
static int dispatch_decode_nb(const uint8_t* code, size_t n, int nb, V* out, const DecodeParams& p,
                              hipStream_t st) {
  switch (nb) {
    case 1: launch_decode<V, 1, kVec>(code, n, out, p, st); break;
    case 2: launch_decode<V, 2, kVec>(code, n, out, p, st); break;
    case 3: launch_decode<V, 3, kVec>(code, n, out, p, st); break;
    case 4: launch_decode<V, 4, false>(code, n, out, p, st); break;
    case 5: launch_decode<V, 5, false>(code, n, out, p, st); break;
    case 6: launch_decode<V, 6, false>(code, n, out, p, st); break;
    case 7: launch_decode<V, 7, false>(code, n, out, p, st); break;
    default: return kErrNbytes;
  }
  return kOk;
}

int ff_decode_launch(const void* code, size_t n, int value_type, int nb, const float* range,
                     float mn, float mx, void* out, hipStream_t st, Profiler* prof) {
  if (nb <= 0 || nb >= 8) return kErrNbytes;
  if (n == 0) return kOk;
  if (value_type != kFloat && value_type != kDouble) return kErrArg;
  DecodeParams p{range, mn, mx, ff_ratio(nb)};
  const uintptr_t ca = reinterpret_cast<uintptr_t>(code), oa = reinterpret_cast<uintptr_t>(out);
  const bool vec = ((oa & 15) == 0) && ((ca & (nb == 2 ? 7 : 3)) == 0);
  const uint8_t* c = static_cast<const uint8_t*>(code);
  const size_t vsz = value_type == kFloat ? 4 : 8;
  ProfScope ps(prof, kKDecode, st, (double)n * (nb + vsz));
  int s;
  if (value_type == kFloat) {
    float* o = static_cast<float*>(out);
    s = vec ? dispatch_decode_nb<float, true>(c, n, nb, o, p, st)
            : dispatch_decode_nb<float, false>(c, n, nb, o, p, st);
  } else {
    double* o = static_cast<double*>(out);
    s = vec ? dispatch_decode_nb<double, true>(c, n, nb, o, p, st)
            : dispatch_decode_nb<double, false>(c, n, nb, o, p, st);
  }
  return s == kOk ? launch_status() : s;
}

}  // namespace psf
