// FIXING_FLOAT codec kernels for gfx950 (CDNA4).
//
// Restates FixingFloatFilter::convert<V> (reference src/filter/fixing_float.h:50-101)
// as three HBM-streaming kernels:
//
//   ff_minmax_partials  pass 1 of encode when min/max are not preset
//                       (fixing_float.h:57-64): per-workgroup min/max of the
//                       value array as order-preserving integer keys.
//   ff_encode           pass 2 (fixing_float.h:73-88): every workgroup folds the
//                       <= kMinmaxGrid partials (L2-resident), derives min/max/bin
//                       exactly as the reference, then quantises 4 values per lane
//                       per group with the stochastic-rounding LCG bit
//                       (fixing_float.h:18-21) reproduced by affine jump-ahead.
//   ff_decode           fixing_float.h:89-101; nb==1 uses a 256-entry LDS table
//                       built with the same double formula (bit-identical).
//
// Data layout: the value array is cut into tiles of kTileGroups groups of 4
// values (16 KiB of f32); a workgroup owns a contiguous run of tiles and walks
// it front to back (block-contiguous streams measured 6.1 TB/s read vs 5.2 TB/s
// for a grid-stride walk on MI355X, tools/bw_probe*.hip).  Inside a tile lane l
// handles groups l, l+256, l+512, l+768, so every load/store instruction of a
// wave is one contiguous 1 KiB (f32 in) / 256 B (nb=1 codes out) span.
//
// Bit-exactness rules: IEEE double division (hipcc's
// default f64 fdiv lowering is correctly rounded), NO FMA contraction (this file
// is compiled with -ffp-contract=off), clamp on the double-promoted value, the
// x86 double->uint64 cast semantics for the degenerate nb>=4 ratios.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

#include "psf_internal.h"
#include "ff_dequant.h"

namespace psf {

constexpr int kTileGroups = 4 * kBlock;  // groups of 4 values per tile
#ifndef PSF_MINMAX_GRID
#define PSF_MINMAX_GRID 1024
#endif
constexpr int kMinmaxGrid = PSF_MINMAX_GRID;  // partials the encode kernel folds
// workgroups for the store-heavy passes: 16384 (2 tiles each at 2^27 values,
// 4 at 2^28) measured 3 % faster than 8192 for the C2 step at both sizes
// (encode 227 -> 220 us, decode 202 -> 194 us at 2^28; 12288, which splits
// the tiles unevenly, no faster than 8192; 32768 +0.6 % at 2^28 but -2.5 % at
// 2^27, one tile per workgroup; tools/ab_c2.sh, r02); 8192 was 1.5-5 % faster
// than 4096 for encode (r01).  The min/max grid at 2048 lost 3 % (its
// partials fold in every encode workgroup), at 256-512 up to 23 %.
#ifndef PSF_STREAM_GRID
#define PSF_STREAM_GRID 16384
#endif
constexpr int kStreamGrid = PSF_STREAM_GRID;
constexpr int kDecodeGridBig = 2 * PSF_STREAM_GRID;
constexpr uint32_t kMask17 = 0x1FFFFu;   // the LCG bits the encoder uses depend on the state mod 2^17

// ------------------------------------------------------------ helpers ------
#ifdef PSF_WG_TRACE
// diagnostic builds only (tools/c3real_probe.hip, tools/c1_trace.py):
// per-workgroup s_memrealtime stamps, 8 words a workgroup: [0] entry, [1]
// quantiser ready, [2] last store done, [3] XCC id << 32 | HW id; the batched
// encode also [4] its min/max items done, [5] the hand-off waited out, [6] its
// own run claimed, [7] its own run published.  Nothing is stamped while the
// buffer (psf_debug_wg_trace) is unset or past kTraceMax workgroups.
__device__ uint64_t* g_wg_trace;  // 8 * kTraceMax words
constexpr uint32_t kTraceMax = 16384;
#define PSF_STAMP(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
#define PSF_STAMP_AT(k)                                                                \
  do {                                                                                 \
    if (threadIdx.x == 0 && g_wg_trace && blockIdx.x < kTraceMax)                      \
      g_wg_trace[8 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)
#define PSF_TRACE_END(a, b)                                                                           \
  do {                                                                                               \
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");                                             \
    __syncthreads();                                                                                 \
    if (threadIdx.x == 0 && g_wg_trace && blockIdx.x < kTraceMax) {                                  \
      uint64_t* tr = g_wg_trace + 8 * blockIdx.x;                                                    \
      tr[0] = a;                                                                                     \
      if (b) tr[1] = b;                                                                              \
      tr[2] = __builtin_amdgcn_s_memrealtime();                                                      \
      tr[3] = (uint64_t)__builtin_amdgcn_s_getreg(6164) << 32 | (uint32_t)__builtin_amdgcn_s_getreg(63492); \
    }                                                                                                \
  } while (0)
extern "C" int psf_debug_wg_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wg_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#else
#define PSF_STAMP(v)
#define PSF_STAMP_AT(k)
#define PSF_TRACE_END(a, b)
#endif
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

// 32-bit keys: the GFX9 DPP reduction -- xor 1 and xor 2 within a quad, the
// half-row and row mirrors, then row 15 broadcast into rows 1 / 3 and lane 31
// into rows 2-3 -- leaves the wave's result in lane 63, read out as a scalar.
// Six DPP-operand min/max instructions against the butterfly's six
// ds_bpermute round trips and their index arithmetic (~40 VALU per wave in
// each encode workgroup's prologue fold, on its critical path).  Masked-off
// rows get the op's identity as `old` (op(v, id) = v), which also lets the
// compiler fold each DPP move into its min / max (one VALU a step).
template <int kCtrl, int kRowMask, uint32_t kId>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)kId, (int)v, kCtrl, kRowMask, 0xF, false);
}
template <bool kMax>
__device__ __forceinline__ uint32_t wave_reduce_dpp(uint32_t v) {
  constexpr uint32_t I = kMax ? 0u : 0xFFFFFFFFu;
  auto op = [](uint32_t a, uint32_t b) { return kMax ? (a > b ? a : b) : (a < b ? a : b); };
  v = op(v, dpp_u32<0xB1, 0xF, I>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_u32<0x4E, 0xF, I>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_u32<0x141, 0xF, I>(v));  // row_half_mirror
  v = op(v, dpp_u32<0x140, 0xF, I>(v));  // row_mirror
  v = op(v, dpp_u32<0x142, 0xA, I>(v));  // row_bcast:15 -> rows 1, 3
  v = op(v, dpp_u32<0x143, 0xC, I>(v));  // row_bcast:31 -> rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
template <> __device__ __forceinline__ uint32_t wave_min<uint32_t>(uint32_t v) { return wave_reduce_dpp<false>(v); }
template <> __device__ __forceinline__ uint32_t wave_max<uint32_t>(uint32_t v) { return wave_reduce_dpp<true>(v); }

// A workgroup barrier for an LDS hand-off only: it waits for this wave's LDS
// operations (lgkmcnt), not for its global loads.  __syncthreads' release
// fence waits for every outstanding load (vmcnt(0)), which held the encode's
// partials fold until its first tile had arrived.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block-wide (256 threads = 4 waves) min/max of keys; result valid in all
// threads (32-bit keys: as scalars).  kOnce: the call site runs once per
// workgroup, so its LDS slots are never rewritten and the trailing barrier
// that guards them goes.
template <typename K, bool kOnce = false>
__device__ __forceinline__ void block_minmax(K& lo, K& hi) {
  __shared__ K s_lo[kBlock / 64], s_hi[kBlock / 64];
  lo = wave_min(lo);
  hi = wave_max(hi);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
  lds_barrier();
  lo = s_lo[0]; hi = s_hi[0];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) {
    lo = s_lo[w] < lo ? s_lo[w] : lo;
    hi = s_hi[w] > hi ? s_hi[w] : hi;
  }
  if constexpr (sizeof(K) == 4) {  // uniform: the key decode that follows runs on the SALU
    lo = (K)__builtin_amdgcn_readfirstlane((int)lo);
    hi = (K)__builtin_amdgcn_readfirstlane((int)hi);
  }
  if (!kOnce) lds_barrier();
}

// 4-element vector access of V.  Cache policy (tools/bw_probe3.hip, emulated
// round trip, MI355X): the value array is streamed with non-temporal loads in
// both encode passes and the decoded array is written with non-temporal
// stores, which keeps the 256 MiB Infinity Cache for the codes the decode pass
// re-reads and stops the decoded output's write-back from landing on the next
// message's min/max pass (369 -> 298 us per 2^27-value step).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
template <typename V> struct Vec4;
template <> struct Vec4<float> {
  // a temporal load (the batched min/max pass: its encode re-reads the values)
  __device__ static void load_keep(const float* p, float v[4]) {
    f32x4 t = *reinterpret_cast<const f32x4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static void loadu_keep(const float* p, float v[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = p[j];
  }
  __device__ static void load(const float* p, float v[4]) {
#ifdef PSF_PLAIN_LOADS
    f32x4 t = *reinterpret_cast<const f32x4*>(p);
#else
    f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
#endif
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  // only element-aligned (a slice of a value array, message.h:141-143)
  __device__ static void loadu(const float* p, float v[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(p + j);
  }
  __device__ static void store(float* p, const float v[4]) {
    f32x4 t = {v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
  }
};
template <> struct Vec4<double> {
  __device__ static void load_keep(const double* p, double v[4]) { load(p, v); }
  __device__ static void loadu_keep(const double* p, double v[4]) { loadu(p, v); }
  __device__ static void load(const double* p, double v[4]) {
    f64x2 a = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p));
    f64x2 b = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p) + 1);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ static void loadu(const double* p, double v[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(p + j);
  }
  __device__ static void store(double* p, const double v[4]) {
    f64x2 a = {v[0], v[1]}, b = {v[2], v[3]};
    __builtin_nontemporal_store(a, reinterpret_cast<f64x2*>(p));
    __builtin_nontemporal_store(b, reinterpret_cast<f64x2*>(p) + 1);
  }
};

// Full-tile loads of a value array that starts off a 16-byte boundary (a
// slice of a value array, message.h:141-143, starts at any element).  f32: the
// array begins r = 1..3 elements past the aligned address xa; lane l loads the
// aligned block under its group and takes the rest of the group from lane
// l+1's block (DPP wave_shl:1), the wave's last lane loading its second block
// itself -- one 16-byte load per group instead of four 4-byte ones.  Every
// block read holds at least one element of the array, so no read leaves the
// array's pages.  f64 keeps the element loads.  All 64 lanes must be active.
__device__ __forceinline__ float next_lane(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}
template <typename V> struct Shifted {
  __device__ static void load(const V* x, const V*, int, size_t g, V v[4]) { Vec4<V>::loadu(x + 4 * g, v); }
};
#ifdef PSF_SHIFTED_LOADS
template <> struct Shifted<float> {
  __device__ static void load(const float*, const float* xa, int r, size_t g, float v[4]) {
    const f32x4* a4 = reinterpret_cast<const f32x4*>(xa) + g;
    const f32x4 a = __builtin_nontemporal_load(a4);
#ifdef PSF_SHIFT_DPP
    f32x4 b = {next_lane(a.x), next_lane(a.y), next_lane(a.z), next_lane(a.w)};
    if ((threadIdx.x & 63) == 63) b = __builtin_nontemporal_load(a4 + 1);
#else
    const f32x4 b = __builtin_nontemporal_load(a4 + 1);
#endif
    if (r == 1) { v[0] = a.y; v[1] = a.z; v[2] = a.w; v[3] = b.x; }
    else if (r == 2) { v[0] = a.z; v[1] = a.w; v[2] = b.x; v[3] = b.y; }
    else { v[0] = a.w; v[1] = b.x; v[2] = b.y; v[3] = b.z; }
  }
};
#endif

// tiles [t0, t1) owned by this workgroup
__device__ __forceinline__ void tile_range(size_t ntiles, size_t& t0, size_t& t1, uint32_t b = blockIdx.x) {
  const size_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  t0 = (size_t)b * per;
  t1 = t0 + per < ntiles ? t0 + per : ntiles;
  if (t0 > ntiles) t0 = ntiles;
}

// ------------------------------------------------------ pass 1: min/max ----
template <typename V, typename K>
__device__ __forceinline__ void acc_minmax(V e, K& lo, K& hi) {
  if (e == e) {  // NaNs are skipped (documented divergence)
    K k = KeyOf<V>::key(e);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
}

// partials layout: K lo[grid], K hi[grid].
// strided: workgroup b reads tiles b, b + grid, ... (the grid sweeps the
// array front to back together, so the tiles read last are its end);
// otherwise a contiguous run of tiles each.
template <typename V, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_minmax_partials(const V* __restrict__ x, size_t n,
                                                              void* __restrict__ partials, uint32_t strided) {
  typedef typename KeyOf<V>::K K;
  K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
  if (kVec) {
    const size_t ngroups = n >> 2;
    const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
    size_t t0, t1, dt = 1;
    tile_range(ntiles, t0, t1);
    if (strided) {
      t0 = blockIdx.x;
      t1 = ntiles;
      dt = gridDim.x;
    }
    for (size_t t = t0; t < t1; t += dt) {
      const size_t gb = t * kTileGroups + threadIdx.x;
      if ((t + 1) * kTileGroups <= ngroups) {
        V v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) Vec4<V>::load(x + 4 * (gb + u * kBlock), v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v[u][j], lo, hi);
      } else {
        // the array's partial last tile: every load issued before any use
        // (one group at a time, its loads waited one memory latency each)
        V v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (gb + u * kBlock < ngroups) Vec4<V>::load(x + 4 * (gb + u * kBlock), v[u]);
          else
#pragma unroll
            for (int j = 0; j < 4; ++j) v[u][j] = (V)__builtin_nan("");  // skipped by acc_minmax
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v[u][j], lo, hi);
      }
    }
    if (blockIdx.x == 0)
      for (size_t i = (ngroups << 2) + threadIdx.x; i < n; i += kBlock) acc_minmax<V, K>(x[i], lo, hi);
  } else {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthreads = (size_t)gridDim.x * kBlock;
    for (size_t i = tid; i < n; i += nthreads) acc_minmax<V, K>(x[i], lo, hi);
  }
  block_minmax(lo, hi);
  if (threadIdx.x == 0) {
    K* p = reinterpret_cast<K*>(partials);
    p[blockIdx.x] = lo;
    p[gridDim.x + blockIdx.x] = hi;
  }
}

// The min/max partials every workgroup of the encode kernel folds (<= 1024
// pairs, L2-resident), in two steps: load (into registers, kMinmaxGrid /
// kBlock pairs a thread) before the first tile's loads, fold after them.  The
// order matters: loads return in issue order, and C3's partials, loaded behind
// 2048 workgroups' first tiles (32 MB), arrived 5.7 us (median) into a 12 us
// kernel, holding every workgroup's quantiser that long.  (Scalar loads, which
// a CU pair's scalar cache would serve from one fetch, were slower still: the
// scalar path took 12-38 us to deliver 8 KB to 2048 workgroups.)  The fold
// returns min/max in the reference's FilterConfig representation (float),
// fixing_float.h:57-64.
template <typename V>
struct Partials {
  typedef typename KeyOf<V>::K K;
  static constexpr int kPer = (kMinmaxGrid + kBlock - 1) / kBlock;
  K lo[kPer], hi[kPer];
  int n = 1 << 30;  // records loaded unconditionally: lanes at or past n hold 0
  __device__ __forceinline__ void load(const void* partials, int nparts) {
    const K* p = reinterpret_cast<const K*>(partials);
    if (sizeof(K) == 4) {
      // unconditional buffer loads, no exec-masked branches: a record past
      // nparts reads 0, the max identity; the min's lanes select theirs
      const int bytes = nparts * 4;
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(const_cast<K*>(p), 0, bytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rh =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<K*>(p + nparts), 0, bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int off = ((int)threadIdx.x + k * kBlock) * 4;
        lo[k] = (K)__builtin_amdgcn_raw_buffer_load_b32(rl, off, 0, 0);
        hi[k] = (K)__builtin_amdgcn_raw_buffer_load_b32(rh, off, 0, 0);
      }
      n = nparts;  // (the min's identity is selected in fold: a select here
                   // waited for these loads before the tile's were issued)
      return;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = (int)threadIdx.x + k * kBlock;
      lo[k] = i < nparts ? p[i] : KeyOf<V>::kLoId;
      hi[k] = i < nparts ? p[nparts + i] : KeyOf<V>::kHiId;
    }
  }
  __device__ __forceinline__ void fold(float& mn_f, float& mx_f) const {
    K l = lo[0], h = hi[0];
#pragma unroll
    for (int k = 1; k < kPer; ++k) {
      l = lo[k] < l ? lo[k] : l;
      h = hi[k] > h ? hi[k] : h;
    }
    if (n < kPer * kBlock) {  // (uniform) fewer partials than lanes' slots
      l = KeyOf<V>::kLoId;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const K a = (int)threadIdx.x + k * kBlock < n ? lo[k] : KeyOf<V>::kLoId;
        l = a < l ? a : l;
      }
    }
    block_minmax<K, true>(l, h);
    if (sizeof(V) == 4) {
      // all-NaN / empty: l stays at the identity, which decodes to a NaN
      float lo_v = key_f32((uint32_t)l), hi_v = key_f32((uint32_t)h);
      mn_f = lo_v;
      mx_f = (float)((double)hi_v + 1e-6);
    } else {
      double lo_v = key_f64((uint64_t)l), hi_v = key_f64((uint64_t)h);
      mn_f = (float)lo_v;
      mx_f = (float)(hi_v + 1e-6);
    }
  }
};

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
  uint32_t a_thr, c_thr;    // scalar path (full 32-bit): nthreads elements
  const uint32_t* lcg_bits; // bit k = !bit16(x_k), x_k the k-th state of the mod-2^17 cycle from 0
  uint32_t lcg_pos;         // position of the seed on that cycle: seed = x_pos (mod 2^17)
  double ratio;
  float* range_out;         // side-info float[2] (device), may be null
  int* status_out;          // CHECK_GT(bin,0) outcome (device), may be null
  float* range_host;        // {min, max, status} into host-mapped memory, may be null
  PubSlot* pub;             // host-mapped publish slot, may be null
  uint32_t ticket;
  // 1: workgroup b takes the tiles of workgroup grid - 1 - b, the array's end
  // first -- what a strided min/max pass read last (the Infinity Cache's)
  uint32_t reverse;
};

// s -> a*s + c, composed k times.
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
    reinterpret_cast<uint32_t*>(out)[g] = w;
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

// ---- codes written into a stored snappy stream (COMPRESSING next) ----------
// FfJob::flags bit 2: the job's codes go to the layout of psf_internal.h's
// StoredLayout -- fragment k's 64 KiB at hdr + 65539 k + 3, its literal tag
// before it, the varint header first -- so COMPRESSING leaves a stream whose
// fragments all come out stored where it is (snappy.hip K-place).  A group's
// code dword(s) land misaligned by (hdr + 3k + 3) mod 4: one unaligned
// global store (gfx950 runs in unaligned mode: as fast as the aligned stream,
// tools/ustore_probe.hip); the tags and the header are constants, written by
// the job's first workgroup while it encodes.
constexpr uint32_t kFlagStored = 4u;
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;
typedef uint64_t __attribute__((aligned(1))) u64_unaligned;

// the header / tag bytes before fragment k's payload
__device__ __forceinline__ void stored_put_prefix(uint8_t* __restrict__ out, const StoredLayout& L, uint32_t k) {
  const uint64_t p0 = k ? stored_frag_tag(L, k) : 0, p1 = stored_frag_data(L, k);
  for (uint64_t P = p0; P < p1; ++P) out[P] = stored_prefix_byte(L, k, P);
}

// payload byte b (the ragged tail), one thread
__device__ __forceinline__ void stored_put_byte(uint8_t* __restrict__ out, const StoredLayout& L, uint32_t b,
                                                uint8_t v) {
  out[stored_pos(L, b)] = v;
}

// the 4 * NB code bytes of group g (NB 1 or 2: a group never straddles a fragment)
template <int NB>
__device__ __forceinline__ void store_codes_stored(uint8_t* __restrict__ out, const StoredLayout& L, size_t g,
                                                   uint32_t w0, uint32_t w1) {
  const uint32_t b = (uint32_t)(g * 4 * NB);
  uint8_t* p = out + stored_pos(L, b);
  if (NB == 1) *reinterpret_cast<u32_unaligned*>(p) = w0;
  else *reinterpret_cast<u64_unaligned*>(p) = (uint64_t)w0 | ((uint64_t)w1 << 32);
}
template <int NB>
__device__ __forceinline__ void store_codes_stored(uint8_t* __restrict__ out, const StoredLayout& L, size_t g,
                                                   const uint64_t r[4]) {
  uint32_t w0, w1 = 0;
  if (NB == 1) {
    w0 = (uint32_t)(r[0] & 0xFF) | ((uint32_t)(r[1] & 0xFF) << 8) | ((uint32_t)(r[2] & 0xFF) << 16) |
         ((uint32_t)(r[3] & 0xFF) << 24);
  } else {
    w0 = (uint32_t)(r[0] & 0xFFFF) | ((uint32_t)(r[1] & 0xFFFF) << 16);
    w1 = (uint32_t)(r[2] & 0xFFFF) | ((uint32_t)(r[3] & 0xFFFF) << 16);
  }
  store_codes_stored<NB>(out, L, g, w0, w1);
}

// The quantiser.  Reference (fixing_float.h:80-82):
//   tmp = (proj - min_v) / bin * ratio;  r = (uint64)floor(tmp) + boolrand
// Only floor(tmp) matters, so the f64 division is skipped unless it can change
// the floor:
//  * f64 fast path (nb <= 3): t' = d * (ratio/bin) differs from tmp by
//    < 5e-16 * tmp <= 8.4e-9; floor(t') == floor(tmp) whenever frac(t') is
//    farther than kGuard64 = 2^-26 from an integer.
//  * f32 fast path (f32 values, nb == 1): d, ratio/bin and the product in
//    f32 carry <= 3 * 2^-24 relative error together, so |t' - tmp| <= 4.6e-5
//    for tmp <= 254.0001 and the guard is kGuard32 = 2^-14 = 6.1e-5.
//    (tests/test_oracle.py checks both bounds on adversarial inputs.)
// Anything inside a guard band, NaN inputs (the min/max clamp sends them to a
// band edge) and an infinite bin take the reference's exact double sequence.
constexpr double kGuard64 = 1.4901161193847656e-08;  // 2^-26
constexpr float kGuard32 = 6.103515625e-05f;         // 2^-14

struct QuantParams {
  double min_v, max_v, bin, ratio, scale;
  float min_f, max_f, scale_f;
  bool fast;  // bin finite (an infinite bin makes inf/inf NaNs the fast path misses)
};

// the reference's exact sequence, NaN -> 0 (x86 cast)
__device__ __forceinline__ uint32_t quant_exact(double x, const QuantParams& q) {
  const double proj = x > q.max_v ? q.max_v : (x < q.min_v ? q.min_v : x);
  const double tmp = (proj - q.min_v) / q.bin * q.ratio;
  return (tmp == tmp) ? (uint32_t)floor(tmp) : 0u;
}

// Branch-free fast floor for nb <= 3; `ok` is false when the value sits in a
// guard band (or is NaN / the bin is infinite) and needs quant_exact.
template <typename V, int NB>
__device__ __forceinline__ uint32_t quant_fast(V xv, const QuantParams& q, bool& ok) {
  if (NB == 1 && sizeof(V) == 4) {
    const float x = (float)xv;
    // clamp in one v_med3 (min < max here); NaNs go to the exact path
    const float t = (__builtin_amdgcn_fmed3f(x, q.min_f, q.max_f) - q.min_f) * q.scale_f;
    const float f = floorf(t);
    // frac in (g, 1-g) as one compare: |frac - 1/2| < 1/2 - g (conservative
    // where 1/2 - frac rounds; those values just take the exact path)
    ok = q.fast & (fabsf((t - f) - 0.5f) < 0.5f - kGuard32) & (x == x);  // no branches
    return (uint32_t)f;
  }
  const double x = (double)xv;
  const double t = (fmin(fmax(x, q.min_v), q.max_v) - q.min_v) * q.scale;
  const double f = floor(t);
  ok = q.fast & (fabs((t - f) - 0.5) < 0.5 - kGuard64);  // NaN t: false
  return (uint32_t)f;
}

// 4 groups x 4 values of one lane: fast floors, then one (rare) divergent
// pass over the values that need the exact sequence.
template <typename V, int NB>
__device__ __forceinline__ void quant_tile(const V v[4][4], const QuantParams& q, uint32_t fl[4][4]) {
  if (NB >= 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double x = (double)v[u][j];
        const double proj = x > q.max_v ? q.max_v : (x < q.min_v ? q.min_v : x);
        fl[u][j] = (uint32_t)x86_d2u64(floor((proj - q.min_v) / q.bin * q.ratio));
      }
    return;
  }
  // one flag per lane (the per-value flags combine in scalar masks); a lane
  // with any value in a guard band redoes its 16 values exactly (rare)
  bool all_ok = true;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bool ok;
      fl[u][j] = quant_fast<V, NB>(v[u][j], q, ok);
      all_ok = all_ok & ok;
    }
  if (__builtin_expect(!all_ok, 0)) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) fl[u][j] = quant_exact((double)v[u][j], q);
  }
}

template <typename V, int NB>
__device__ __forceinline__ uint64_t quant_floor(V xv, const QuantParams& q) {
  if (NB >= 4) {  // degenerate int-shift ratios: always the exact sequence
    const double x = (double)xv;
    const double proj = x > q.max_v ? q.max_v : (x < q.min_v ? q.min_v : x);
    return x86_d2u64(floor((proj - q.min_v) / q.bin * q.ratio));
  }
  if (!q.fast) return quant_exact((double)xv, q);
  if (NB == 1 && sizeof(V) == 4) {
    const float x = (float)xv;
    const float t = (fminf(fmaxf(x, q.min_f), q.max_f) - q.min_f) * q.scale_f;
    const float f = floorf(t);
    const float fr = t - f;
    if (__builtin_expect(fr > kGuard32 && fr < 1.0f - kGuard32, 1)) return (uint32_t)f;
    return quant_exact((double)xv, q);
  }
  const double x = (double)xv;
  const double t = (fmin(fmax(x, q.min_v), q.max_v) - q.min_v) * q.scale;
  const double f = floor(t);
  const double fr = t - f;
  if (__builtin_expect(fr > kGuard64 && fr < 1.0 - kGuard64, 1)) return (uint32_t)f;
  return quant_exact(x, q);
}

// full 32-bit state step (scalar and tail paths)
__device__ __forceinline__ uint64_t lcg_bit(uint32_t& s) {
  s = kLcgA * s + kLcgC;
  return ((s >> 16) & 1u) == 0u ? 1u : 0u;
}

// The rare exact pass of a lane whose band test failed: the values of its
// valid groups that sit in a guard band (quant_fast's test) get the
// reference's double sequence.  One rolled loop over the lane's 16 values,
// each read from its register by the wave-uniform loop index: sixteen unrolled tests and
// exact sequences held the tile kernels at 73-79 VGPRs (6 waves per SIMD)
// and cost C3's encode 1 us.
__device__ __forceinline__ void redo_f32_nb1(const float v[4][4], const QuantParams& q, uint32_t valid,
                                             uint32_t w[4]) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  const f32x16 vv = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3],
                     v[2][0], v[2][1], v[2][2], v[2][3], v[3][0], v[3][1], v[3][2], v[3][3]};
#pragma unroll 1
  for (uint32_t k = 0; k < 16; ++k) {  // k uniform: vv[k] is an indexed register read
    if (!((valid >> (k >> 2)) & 1u)) continue;
    const float xv = vv[k];
    bool ok;
    (void)quant_fast<float, 1>(xv, q, ok);
    if (ok) continue;
    const uint32_t c = quant_exact((double)xv, q);
    const uint32_t sh = 8u * (k & 3u);
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if ((k >> 2) == u) w[u] = (w[u] & ~(0xFFu << sh)) | (c << sh);
  }
}

// f32 values, num_bytes = 1: one lane's tile (4 groups x 4 values; `valid`
// bit u: group u is in the array, all four but in an array's partial last
// tile).  Fast floor in f32 (the guard band of quant_fast), with the band
// test folded into two lane-wide accumulators of frac = t - floor(t)
// compared as u32 bit patterns (frac >= 0, so the order is the float order,
// and a NaN frac sorts above 1): the lane is fast when g < min frac and max
// frac < 1 - g.  NaN and infinite values need no test of their own: med3
// returns min_f or max_f for them, whose t is 0 or within 1e-4 of ratio,
// inside the band.  Codes <= ratio = 254, so the packed LCG bits add without
// carries.  A lane that fails takes redo_f32_nb1 (xg: the values of v in
// memory, group u's at xg + 4 u kBlock).
template <bool kStored = false>
__device__ __forceinline__ void encode_tile_f32_nb1(const float v[4][4], const float* xg, const QuantParams& q,
                                                    const uint32_t b4[4], uint32_t* __restrict__ out,
                                                    const StoredLayout* L = nullptr, size_t gs = 0,
                                                    uint32_t valid = 0xFu) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 mn2 = {q.min_f, q.min_f}, sc2 = {q.scale_f, q.scale_f};
  uint32_t lo = 0x7F800000u, hi = 0u;
  uint32_t w[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint32_t acc = 0, ulo = 0x7F800000u, uhi = 0u;
#pragma unroll
    for (int j = 0; j < 4; j += 2) {  // value pairs: packed f32 sub/mul (exact per element)
      const f32x2 c = {__builtin_amdgcn_fmed3f(v[u][j], q.min_f, q.max_f),
                       __builtin_amdgcn_fmed3f(v[u][j + 1], q.min_f, q.max_f)};
      const f32x2 t = (c - mn2) * sc2;
      const f32x2 f = {floorf(t.x), floorf(t.y)};
      const f32x2 fr = t - f;
      const uint32_t a = __float_as_uint(fr.x), b = __float_as_uint(fr.y);
      ulo = __builtin_elementwise_min(__builtin_elementwise_min(ulo, a), b);
      uhi = __builtin_elementwise_max(__builtin_elementwise_max(uhi, a), b);
      acc = __builtin_amdgcn_cvt_pk_u8_f32(f.x, j, acc);
      acc = __builtin_amdgcn_cvt_pk_u8_f32(f.y, j + 1, acc);
    }
    if ((valid >> u) & 1u) {
      lo = __builtin_elementwise_min(lo, ulo);
      hi = __builtin_elementwise_max(hi, uhi);
    }
    w[u] = acc;
  }
  const bool fast = q.fast && (lo > __float_as_uint(kGuard32)) && (hi < __float_as_uint(1.0f - kGuard32));
  if (__builtin_expect(!fast, 0)) redo_f32_nb1(v, q, valid, w);  // rare (~0.4 % of lanes)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (!((valid >> u) & 1u)) continue;
    const uint32_t c = w[u] + ((b4[u] * 0x204081u) & 0x01010101u);
    if (kStored) store_codes_stored<1>(reinterpret_cast<uint8_t*>(out), *L, gs + u * kBlock, c, 0u);
    else out[u * kBlock] = c;
  }
}

// One tile of this lane (groups gb, gb+256, gb+512, gb+768 of the array x;
// `valid` as above): LCG bits from the cycle table -- group g (elements 4g..4g+3) uses
// the states s_{4g+1..4g+4} = x_{pos+4g+1..4}, four consecutive table bits
// (one 8-byte L1/L2-hit load and a funnel shift) -- then quantise, add, pack,
// store.
template <typename V, int NB, bool kStored = false>
__device__ __forceinline__ void encode_full_tile(const V v[4][4], const V* x, const QuantParams& q,
                                                 const EncodeParams& p, uint8_t* __restrict__ out, size_t gb,
                                                 size_t gs, const StoredLayout* L = nullptr, uint32_t valid = 0xFu) {
  uint32_t b4[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t k = (p.lcg_pos + 1u + 4u * (uint32_t)(gb + u * kBlock)) & kMask17;
    const uint2 w = *reinterpret_cast<const uint2*>(p.lcg_bits + (k >> 5));
    b4[u] = __builtin_amdgcn_alignbit(w.y, w.x, k & 31u) & 0xFu;
  }
  if (NB == 1 && sizeof(V) == 4) {
    const float* xg = reinterpret_cast<const float*>(x) + 4 * gb;
    if (kStored) encode_tile_f32_nb1<true>(reinterpret_cast<const float(*)[4]>(v), xg, q, b4,
                                           reinterpret_cast<uint32_t*>(out), L, gs, valid);
    else encode_tile_f32_nb1(reinterpret_cast<const float(*)[4]>(v), xg, q, b4,
                             reinterpret_cast<uint32_t*>(out) + gs, nullptr, 0, valid);
    return;
  }
  uint32_t fl[4][4];
  quant_tile<V, NB>(v, q, fl);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (!((valid >> u) & 1u)) continue;
    uint64_t r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = (uint64_t)(uint32_t)(fl[u][j] + ((b4[u] >> j) & 1u));
    if constexpr (kStored && (NB == 1 || NB == 2)) store_codes_stored<NB>(out, *L, gs + u * kBlock, r);
    else store_codes<NB>(out, gs + u * kBlock, r);
  }
}

// An array's partial last tile (groups past the end masked off): every load
// issued before any use (they used to go out one group at a time behind a
// 64-bit LCG jump, and C3's last workgroup finished 2 us after the rest), the
// LCG bits from the cycle table as in a full tile.
template <typename V, int NB, bool kStored = false>
__device__ __forceinline__ void encode_partial_tile(const V* __restrict__ x, bool aligned, size_t ngroups,
                                                    const QuantParams& q, const EncodeParams& p,
                                                    uint8_t* __restrict__ out, size_t gb,
                                                    const StoredLayout* L = nullptr) {
  V v[4][4];
  uint32_t valid = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const size_t g = gb + u * kBlock;
    if (g < ngroups) {
      valid |= 1u << u;
      if (aligned) Vec4<V>::load(x + 4 * g, v[u]);
      else Vec4<V>::loadu(x + 4 * g, v[u]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[u][j] = (V)q.min_f;
    }
  }
  encode_full_tile<V, NB, kStored>(v, x, q, p, out, gb, gb, L, valid);
}

// A workgroup's first full tile, loaded unconditionally through a buffer
// descriptor over it (no records when the workgroup has no full tile: the
// loads return zeros, which nothing reads).  Behind a branch, the loads made
// the compiler's wait for the partials (issued before them) a vmcnt(0) at the
// branch's join, i.e. a wait for the tile as well.  Non-temporal, as
// Vec4::load.
template <typename V>
__device__ __forceinline__ void prefetch_tile(const V* x, size_t t0, size_t tf, V v[4][4]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const bool have = t0 < tf;
  const V* base = x + (have ? 4 * t0 * kTileGroups : 0);
  const int bytes = have ? (int)(4 * kTileGroups * sizeof(V)) : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<V*>(base), 0, bytes, 0x00020000);
  constexpr int kNt = 2;  // gfx950 cache policy bit: nt
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int off = (int)((threadIdx.x + u * kBlock) * 4 * sizeof(V));
    if (sizeof(V) == 4) {
      const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kNt);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[u][j] = (V)__uint_as_float(a[j]);
    } else {
      const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kNt);
      const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, kNt);
      v[u][0] = (V)__longlong_as_double((long long)((uint64_t)a[1] << 32 | a[0]));
      v[u][1] = (V)__longlong_as_double((long long)((uint64_t)a[3] << 32 | a[2]));
      v[u][2] = (V)__longlong_as_double((long long)((uint64_t)b[1] << 32 | b[0]));
      v[u][3] = (V)__longlong_as_double((long long)((uint64_t)b[3] << 32 | b[2]));
    }
  }
}

template <typename V, int NB, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_encode(const V* __restrict__ x, size_t n,
                                                     uint8_t* __restrict__ out, EncodeParams p) {
  PSF_STAMP(ts0);
  // tiles of this workgroup; the partials' loads, then the first full
  // tile's, are issued before the min/max fold so that their latency hides
  // behind each other (Partials, prefetch_tile)
  const size_t ngroups = n >> 2;
  const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
  const size_t nfull = ngroups / kTileGroups;
  size_t t0 = 0, t1 = 0;
  if (kVec) {
    // (workgroup b keeps tile run b: the decode's workgroup b, dealt to the
    // same XCD, then reads its codes from that XCD's L2.  Rotating the runs by
    // one, to start the array's partial tile first, cost C3's decode 7.1 ->
    // 8.4 us for a 0.4 us gain of the encode.)
    tile_range(ntiles, t0, t1, p.reverse ? gridDim.x - 1 - blockIdx.x : blockIdx.x);
  }
  const size_t tf = t1 < nfull ? t1 : nfull;  // full tiles are [t0, tf)
  Partials<V> parts;
  // (f32: loaded unconditionally -- no records without partials -- so that
  // the loads share the tile's block and nothing consumes them before the
  // tile's loads are out)
  if (sizeof(V) == 4) parts.load(p.partials ? p.partials : (const void*)x, p.partials ? p.nparts : 0);
  else if (p.partials != nullptr) parts.load(p.partials, p.nparts);
  __builtin_amdgcn_sched_barrier(0);  // the partials' loads stay ahead of the tile's
  V first[4][4];
  if (kVec) prefetch_tile<V>(x, t0, tf, first);

  float mn_f = p.preset_min, mx_f = p.preset_max;
  if (p.partials != nullptr) {
    float cmn, cmx;
    parts.fold(cmn, cmx);
    if (!p.has_min) mn_f = cmn;
    if (!p.has_max) mx_f = cmx;
  }
  QuantParams q;
  q.min_v = (double)mn_f;
  q.max_v = (double)mx_f;
  q.bin = q.max_v - q.min_v;
  q.ratio = p.ratio;
  q.scale = q.ratio / q.bin;
  q.min_f = mn_f;
  q.max_f = mx_f;
  q.scale_f = (float)q.scale;
  q.fast = q.bin < __builtin_huge_val();
  PSF_STAMP(ts1);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int status = (q.bin > 0) ? kOk : kErrBin;
    if (p.range_out) { p.range_out[0] = mn_f; p.range_out[1] = mx_f; }
    if (p.status_out) *p.status_out = status;
    if (p.range_host) {  // read by the host after a stream sync
      p.range_host[0] = mn_f;
      p.range_host[1] = mx_f;
      reinterpret_cast<int32_t*>(p.range_host)[2] = status;
    }
    if (p.pub) {  // side-info to the host while the grid keeps streaming
      pub_store(&p.pub->range[0], mn_f);
      pub_store(&p.pub->range[1], mx_f);
      pub_store(&p.pub->status, (int32_t)status);
      publish_ticket(p.pub, p.ticket);
    }
  }
  if (!(q.bin > 0)) return;  // CHECK_GT(bin, 0), fixing_float.h:71

  if (kVec) {
    if (t0 < tf) {
      encode_full_tile<V, NB>(first, x, q, p, out, t0 * kTileGroups + threadIdx.x, t0 * kTileGroups + threadIdx.x);
      for (size_t t = t0 + 1; t < tf; ++t) {
        const size_t gb = t * kTileGroups + threadIdx.x;
        V v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) Vec4<V>::load(x + 4 * (gb + u * kBlock), v[u]);
        encode_full_tile<V, NB>(v, x, q, p, out, gb, gb);
      }
    }
    // the partial last tile of the array, if this workgroup owns it
    for (size_t t = (t0 > tf ? t0 : tf); t < t1; ++t)
      encode_partial_tile<V, NB>(x, true, ngroups, q, p, out, t * kTileGroups + threadIdx.x);
    // ragged tail (< 4 values): one thread
    const size_t tail = ngroups << 2;
    if (blockIdx.x == 0 && threadIdx.x == 0 && tail < n) {
      uint32_t st = lcg_jump(p.seed, tail);
      for (size_t i = tail; i < n; ++i) {
        uint64_t r = quant_floor<V, NB>(x[i], q) + lcg_bit(st);
        for (int j = 0; j < NB; ++j) { out[i * NB + j] = (uint8_t)(r & 0xFF); r >>= 8; }
      }
    }
  } else {
    // unaligned buffers: scalar grid-stride path, one value per lane per step
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthreads = (size_t)gridDim.x * kBlock;
    uint32_t s = lcg_jump(p.seed, tid);
    for (size_t i = tid; i < n; i += nthreads) {
      uint32_t st = s;
      uint64_t r = quant_floor<V, NB>(x[i], q) + lcg_bit(st);
      for (int j = 0; j < NB; ++j) { out[i * NB + j] = (uint8_t)(r & 0xFF); r >>= 8; }
      s = p.a_thr * s + p.c_thr;
    }
  }
  PSF_TRACE_END(ts0, ts1);
}

// ------------------------------------------------------------- decode ------
struct DecodeParams {
  const float* range;     // device float[2] or null -> use (mn, mx)
  float mn, mx;
  double ratio;
};

// dequant / dequant_q: ff_dequant.h

struct __attribute__((aligned(4))) CodeWords3 { uint32_t a, b, d; };  // one group of four nb=3 codes

__device__ __forceinline__ void unpack_codes3(uint32_t a, uint32_t b, uint32_t d, uint64_t r[4]) {
  r[0] = a & 0xFFFFFF;
  r[1] = (a >> 24) | ((b & 0xFFFF) << 8);
  r[2] = (b >> 16) | ((d & 0xFF) << 16);
  r[3] = d >> 8;
}


template <int NB>
__device__ __forceinline__ void load_codes(const uint8_t* __restrict__ code, size_t g, uint64_t r[4]) {
  if (NB == 2) {
    uint2 w = reinterpret_cast<const uint2*>(code)[g];
    r[0] = w.x & 0xFFFF; r[1] = w.x >> 16; r[2] = w.y & 0xFFFF; r[3] = w.y >> 16;
  } else {
    const CodeWords3 c = reinterpret_cast<const CodeWords3*>(code)[g];
    unpack_codes3(c.a, c.b, c.d, r);
  }
}

// One tile (kTileGroups groups of four values) of the decode.  All four code
// loads are issued before any dequantise: lanes past the array's last group
// load that group again (in bounds, branch-free) and skip the store, so the
// loads of a partial tile are not serialised behind per-group branches.
template <typename V, int NB>
__device__ __forceinline__ void decode_tile(const uint8_t* __restrict__ code, V* __restrict__ out, size_t gb,
                                            size_t ngroups, const V* lut, double ratio,
                                            double bin, double min_v) {
  const double inv = 1.0 / ratio;  // IEEE division: RN(1/ratio)
  if (NB == 1) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(code);
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      w[u] = c32[g < ngroups ? g : ngroups - 1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      if (g < ngroups) {
        V v[4] = {lut[w[u] & 0xFF], lut[(w[u] >> 8) & 0xFF], lut[(w[u] >> 16) & 0xFF], lut[w[u] >> 24]};
        Vec4<V>::store(out + 4 * g, v);
      }
    }
  } else {
    uint64_t r[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      load_codes<NB>(code, g < ngroups ? g : ngroups - 1, r[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      if (g < ngroups) {
        V v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = dequant_q<V>(r[u][j], ratio, inv, bin, min_v);
        Vec4<V>::store(out + 4 * g, v);
      }
    }
  }
}

template <typename V, int NB, bool kVec>
__global__ __launch_bounds__(kBlock) void ff_decode(const uint8_t* __restrict__ code, size_t n,
                                                     V* __restrict__ out, DecodeParams p) {
  // nb = 1: the first tile's code words go out before the range read and the
  // table build, whose latency they then hide (LDS-only barrier: the table's
  // __syncthreads would wait for them)
  uint32_t w0[4];
  size_t t0 = 0, t1 = 0;
  const size_t ngroups = n >> 2;
  if (kVec && NB == 1) {
    const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
    tile_range(ntiles, t0, t1);
    if (t0 < t1) {
      const uint32_t* c32 = reinterpret_cast<const uint32_t*>(code);
      const size_t gb = t0 * kTileGroups + threadIdx.x;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t g = gb + u * kBlock;
        w0[u] = c32[g < ngroups ? g : ngroups - 1];
      }
    }
  }
  float mn_f = p.mn, mx_f = p.mx;
  if (p.range) { mn_f = p.range[0]; mx_f = p.range[1]; }
  const double min_v = (double)mn_f, max_v = (double)mx_f;
  const double bin = max_v - min_v;
  const double ratio = p.ratio;

  if (kVec && NB <= 3) {
    const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
    if (NB != 1) tile_range(ntiles, t0, t1);
    __shared__ V lut[256];
    if (NB == 1) {
      // 256-entry table, same formula => bit-identical to the per-element path
      lut[threadIdx.x] = dequant<V>((uint64_t)threadIdx.x, ratio, bin, min_v);
      lds_barrier();
      if (t0 < t1) {  // the prefetched first tile
        const size_t gb = t0 * kTileGroups + threadIdx.x;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const size_t g = gb + u * kBlock;
          if (g < ngroups) {
            V v[4] = {lut[w0[u] & 0xFF], lut[(w0[u] >> 8) & 0xFF], lut[(w0[u] >> 16) & 0xFF], lut[w0[u] >> 24]};
            Vec4<V>::store(out + 4 * g, v);
          }
        }
        ++t0;
      }
    }
    for (size_t t = t0; t < t1; ++t)
      decode_tile<V, NB>(code, out, t * kTileGroups + threadIdx.x, ngroups, lut, ratio, bin, min_v);
    if (blockIdx.x == 0) {
      for (size_t i = (ngroups << 2) + threadIdx.x; i < n; i += kBlock) {
        uint64_t r = 0;
        for (int j = 0; j < NB; ++j) r |= (uint64_t)code[i * NB + j] << (8 * j);
        out[i] = dequant<V>(r, ratio, bin, min_v);
      }
    }
    return;
  }

  // generic byte path (nb >= 4, or unaligned buffers)
  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t nthreads = (size_t)gridDim.x * kBlock;
  for (size_t i = tid; i < n; i += nthreads) {
    uint64_t r = 0;
    for (int j = 0; j < NB; ++j) r |= (uint64_t)code[i * NB + j] << (8 * j);
    out[i] = dequant<V>(r, ratio, bin, min_v);
  }
}

// ------------------------------------------------- batched (many arrays) ---
// Many small messages (the async-SGD minibatches, the C4 slices) make the
// per-array launches latency-bound.  The batched kernels take a table of up
// to kFfBatchMax arrays in their kernel arguments; a workgroup finds its array
// by its index in the batch grid and runs the same tile code as the
// single-array kernels on its share of that array's tiles.  Aligned f32/f64
// arrays with num_bytes 1..3 only (the launcher routes the rest to the
// single-array kernels).
struct FfJob {
  const void* x;
  void* out;                 // codes (encode) / values (decode)
  union {
    struct { uint32_t seed, lcg_pos; } e;  // encode: LCG seed and its position on the mod-2^17 cycle
    const float* range;                    // decode: device {min, max} written by the encode, or null
  } u;
  uint32_t n;                // elements (ff_batchable admits n < 2^32 only)
  float mn, mx;              // encode: preset range; decode: the received range
  uint32_t ticket;           // encode: publish ticket
  uint16_t mm_nwg;           // encode: min/max workgroups (0: both preset)
  uint16_t lazy;             // encode: index k of {min, max, status} at range_base / ring_base + 4k, or kNoLazy
  uint32_t flags;            // encode: bit 0 has_min, bit 1 has_max, bits 16-31 publish slot + 1 (0: none)
};
static_assert(sizeof(FfJob) == 48, "FfJob layout");
constexpr uint16_t kNoLazy = 0xFFFFu;
// Two table sizes: up to 64 arrays (4 KiB of kernel arguments, the C1-sized
// batches whose launches are latency-bound) and up to kFfBatchMax = 512 (a
// whole C4 step's slices in one launch per kernel; HIP on ROCm 7 takes
// kernel arguments up to 32 KiB, tools/kernarg_probe.hip).
constexpr int kBatchSmall = 64;
template <int CAP>
struct FfBatchT {
  // a job's workgroups are [first[i], first[i + 1]) (the last ends at the
  // grid); mm_first likewise for the min/max kernel, where a job without a
  // min/max pass has an empty range.  Unused entries ~0u.
  uint32_t first[CAP];
  uint32_t mm_first[CAP];
  FfJob job[CAP];
  int njobs;
  uint32_t total;           // workgroups of the encode / decode grid
  uint32_t mm_total;        // workgroups of the min/max kernel (partials count)
  void* partials;           // K lo[mm_total], K hi[mm_total]
  PubSlot* pub;             // slot base
  float* range_base;        // encode: device {min, max, status} records of the lazy jobs
  float* ring_base;         // encode: the same records in host-mapped memory
  const uint32_t* lcg_bits;
  uint32_t mm_reverse;     // min/max workgroups dispatched in reverse array order
  uint32_t mm_total_done;  // (host) the min/max pass already ran in a merged launch
  double ratio;
};
static_assert(sizeof(FfBatchT<kBatchSmall>) <= 4096, "the small batch fits 4 KiB of kernel arguments");
static_assert(sizeof(FfBatchT<kFfBatchMax>) <= 32000, "the large batch fits the kernel-argument segment");
static_assert(kMinmaxGrid <= 0xFFFF, "FfJob::mm_nwg is 16 bits");
static_assert(kBatchSmall == kFusedArrays, "one ready counter per array of a small batch");


// the job whose [first, first + count) workgroup range holds b: a fully
// unrolled count over the contiguous first-workgroup table (wide scalar loads
// issued together, no dependent loop); the large table in two levels (every
// 16th entry, then the 16 entries of that group)
template <int CAP>
__device__ __forceinline__ int batch_job(const FfBatchT<CAP>& B, uint32_t b, bool mm) {
  const uint32_t* f = mm ? B.mm_first : B.first;
  if (CAP <= kBatchSmall) {
    int j = -1;
#pragma unroll
    for (int i = 0; i < CAP; ++i) j += f[i] <= b ? 1 : 0;
    return j;
  }
  int c = -1;
#pragma unroll
  for (int i = 0; i < CAP / 16; ++i) c += f[16 * i] <= b ? 1 : 0;
  const uint32_t* g = f + 16 * c;
  int j = 16 * c - 1;
#pragma unroll
  for (int i = 0; i < 16; ++i) j += g[i] <= b ? 1 : 0;
  return j;
}

// workgroups of job j in the encode / decode grid
template <int CAP>
__device__ __forceinline__ uint32_t batch_nwg(const FfBatchT<CAP>& B, int j) {
  return (j + 1 < B.njobs ? B.first[j + 1] : B.total) - B.first[j];
}

__device__ __forceinline__ void tile_range_of(size_t ntiles, uint32_t wg, uint32_t nwg, size_t& t0,
                                              size_t& t1) {
  const size_t per = (ntiles + nwg - 1) / nwg;
  t0 = (size_t)wg * per;
  t1 = t0 + per < ntiles ? t0 + per : ntiles;
}

// the batched kernels' bodies take their workgroup index: a merged launch
// (ff_dec_mm_batch) runs a decode batch and a min/max batch side by side
// ---- the in-launch hand-off of ff_fused_batch: an array's min/max items
// (its share of the min/max grid) are claimed and folded by the array's own
// encode workgroups, which then wait until every item is folded.  Per-XCD L2s
// are not coherent and a CU's L1 is never refreshed by another CU's stores
// (MI355X_MICROARCH.md, inter-workgroup visibility): each partial is stored
// write-through (an agent-scope atomic store, `sc1`), the storing wave drains
// its stores, then one lane adds to the array's ready counter (agent scope);
// a waiting workgroup polls that counter with `sc1` loads, joins a barrier and
// loads the partials `sc1`.  Every item is claimed by a workgroup that is
// already running before anyone waits for it (a workgroup claims once, before
// it waits), so no dispatch order can deadlock it.  Per array one 128-byte line of counters: [0] claims, [1]
// items folded, [2] workgroups done -- the last one done zeroes the line for
// the next launch on the stream.  Bounded: a wait that outlasts kHandoffTicks
// gives up and the array reports kErrHip.
#ifdef PSF_FUSED_DEBUG
constexpr uint64_t kHandoffTicks = 20000000ull;
#else
constexpr uint64_t kHandoffTicks = 200000000ull;  // 2 s of the 100 MHz wall clock
#endif
// the bound in force (psf_debug_set_handoff_ticks lowers it, so a test can
// drive the late path)
__device__ uint64_t g_handoff_ticks = kHandoffTicks;
constexpr uint32_t kFusedLine = 32;               // u32 per array's counter line
__device__ __forceinline__ bool wait_ready(const uint32_t* c, uint32_t want) {
  const uint64_t t0 = wall_clock64();
  const uint64_t lim = g_handoff_ticks;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
    if (wall_clock64() - t0 > lim) return false;
    __builtin_amdgcn_s_sleep(8);
  }
  return true;
}

// min/max partial bb (of job jb) of a batch; ready: ff_fused_batch's counter
// of folded items (null: a plain launch, the kernel boundary publishes it)
template <typename V, int CAP>
__device__ __forceinline__ void minmax_item(const FfBatchT<CAP>& B, int jb, uint32_t bb, uint32_t* ready) {
  typedef typename KeyOf<V>::K K;
  const FfJob& J = B.job[jb];
  const V* __restrict__ x = static_cast<const V*>(J.x);
  const size_t n = J.n;
  const uint32_t wg = bb - B.mm_first[jb];
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int r = (int)((reinterpret_cast<uintptr_t>(x) & 15) / sizeof(V));
  const V* xa = x - r;
  K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
  const size_t ngroups = n >> 2;
  const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
  size_t t0, t1;
  tile_range_of(ntiles, wg, J.mm_nwg, t0, t1);
  const size_t nfull = ngroups / kTileGroups;
  const size_t tf = t1 < nfull ? t1 : nfull;
  for (size_t t = t0; t < tf; ++t) {  // full tiles: all four loads in flight before the folds
    const size_t gb = t * kTileGroups + threadIdx.x;
    V v[4][4];
    if (al) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#ifdef PSF_MM_KEEP
        Vec4<V>::load_keep(x + 4 * (gb + u * kBlock), v[u]);
#else
        Vec4<V>::load(x + 4 * (gb + u * kBlock), v[u]);
#endif
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#ifdef PSF_MM_KEEP
        Vec4<V>::loadu_keep(x + 4 * (gb + u * kBlock), v[u]);
#else
        Shifted<V>::load(x, xa, r, gb + u * kBlock, v[u]);
#endif
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v[u][j], lo, hi);
  }
  for (size_t t = (t0 > tf ? t0 : tf); t < t1; ++t) {  // the partial last tile: loads before any use
    const size_t gb = t * kTileGroups + threadIdx.x;
    V v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      if (g < ngroups) {
        if (al) Vec4<V>::load(x + 4 * g, v[u]);
        else Vec4<V>::loadu(x + 4 * g, v[u]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = (V)__builtin_nan("");  // skipped by acc_minmax
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v[u][j], lo, hi);
  }
  if (wg == 0)
    for (size_t i = (ngroups << 2) + threadIdx.x; i < n; i += kBlock) acc_minmax<V, K>(x[i], lo, hi);
  block_minmax(lo, hi);
  if (threadIdx.x == 0) {
    K* pp = reinterpret_cast<K*>(B.partials);
    if (ready) {
      __hip_atomic_store(&pp[bb], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&pp[B.mm_total + bb], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      pp[bb] = lo;
      pp[B.mm_total + bb] = hi;
    }
  }
}
// The fused hand-off's own-tile path: min/max items bb and, with two, bb + 1
// are full tiles this workgroup already holds in registers (v, v2): one
// block reduction for both (and the job's ragged tail when bb is the job's
// first item), published as minmax_item publishes an item -- the run's
// min/max in bb's slot, the identity in bb + 1's -- and both counted ready.
template <typename V, int CAP>
__device__ __forceinline__ void minmax_run_regs(const FfBatchT<CAP>& B, int jb, uint32_t bb, uint32_t nitems,
                                                const V v[4][4], const V v2[4][4], uint32_t* ready) {
  typedef typename KeyOf<V>::K K;
  const FfJob& J = B.job[jb];
  K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v[u][j], lo, hi);
  if (nitems == 2)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_minmax<V, K>(v2[u][j], lo, hi);
  if (bb == B.mm_first[jb]) {
    const V* __restrict__ x = static_cast<const V*>(J.x);
    for (size_t i = ((J.n >> 2) << 2) + threadIdx.x; i < J.n; i += kBlock) acc_minmax<V, K>(x[i], lo, hi);
  }
  block_minmax(lo, hi);
  if (threadIdx.x == 0) {
    K* pp = reinterpret_cast<K*>(B.partials);
    __hip_atomic_store(&pp[bb], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&pp[B.mm_total + bb], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (nitems == 2) {
      __hip_atomic_store(&pp[bb + 1], KeyOf<V>::kLoId, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&pp[B.mm_total + bb + 1], KeyOf<V>::kHiId, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ready, nitems, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <typename V, int CAP>
__device__ __forceinline__ void minmax_batch_body(const FfBatchT<CAP>& B, uint32_t block) {
  // mm_reverse: workgroups dispatched last-array-first, so the arrays the
  // encode reads first are the ones read last here (still in the Infinity
  // Cache when the encode starts)
  const uint32_t bb = B.mm_reverse ? B.mm_total - 1 - block : block;
  minmax_item<V, CAP>(B, batch_job(B, bb, true), bb, nullptr);
}
template <typename V, int CAP>
__global__ __launch_bounds__(kBlock) void ff_minmax_batch(FfBatchT<CAP> B) {
  minmax_batch_body<V, CAP>(B, blockIdx.x);
}

// kStored: the instantiation launched when a job of the batch writes a
// stored stream (its extra registers stay out of the plain one's occupancy)
// fused: ff_fused_batch's counter lines (this array's min/max items are folded
// by its encode workgroups in the same launch); returns the job
template <typename V, int NB, int CAP, bool kStored>
__device__ __forceinline__ int encode_batch_body(const FfBatchT<CAP>& B, uint32_t block, uint32_t* fused,
                                                 int32_t* sticky = nullptr) {
  const int jb = batch_job(B, block, false);
  const FfJob& J = B.job[jb];
  const V* __restrict__ x = static_cast<const V*>(J.x);
  uint8_t* __restrict__ out = static_cast<uint8_t*>(J.out);
  const size_t n = J.n;
  const uint32_t wg = block - B.first[jb];
  const uint32_t nwg = batch_nwg(B, jb);
  const uint32_t mm_wg0 = B.mm_first[jb];
  const size_t ngroups = n >> 2;
  const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
  const size_t nfull = ngroups / kTileGroups;
  size_t t0, t1;
  tile_range_of(ntiles, wg, nwg, t0, t1);
  const size_t tf = t1 < nfull ? t1 : nfull;
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int r = (int)((reinterpret_cast<uintptr_t>(x) & 15) / sizeof(V));
  const V* xa = x - r;
  // the first full tile's loads go out before the partials fold, which they
  // do not depend on
  V v[4][4];
  auto load_tile = [&](size_t t) {
    const size_t gb = t * kTileGroups + threadIdx.x;
    if (al) {
#pragma unroll
      for (int u = 0; u < 4; ++u) Vec4<V>::load(x + 4 * (gb + u * kBlock), v[u]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) Shifted<V>::load(x, xa, r, gb + u * kBlock, v[u]);
    }
  };
  if (t0 < tf) load_tile(t0);
  float mn_f = J.mn, mx_f = J.mx;
  bool late = false;  // the in-launch hand-off gave up (never expected)
  // the fused hand-off gave this workgroup exactly its own (full) tiles as
  // min/max items: their values stay in registers for the encode (v, v2)
  bool own = false;
  V v2[4][4];
  if (J.mm_nwg) {
    typedef typename KeyOf<V>::K K;
    K* pp = reinterpret_cast<K*>(B.partials);
    K lo = KeyOf<V>::kLoId, hi = KeyOf<V>::kHiId;
    if (fused) {
      uint32_t* c = fused + kFusedLine * jb;
      __shared__ uint32_t s_item, s_late;
      const uint32_t per = ((uint32_t)J.mm_nwg + nwg - 1) / nwg;
      auto items = [&](uint32_t i0, uint32_t i1) {
        for (uint32_t item = i0; item < i1; ++item) minmax_item<V, CAP>(B, jb, mm_wg0 + item, &c[1]);
      };
      if ((size_t)J.mm_nwg == ntiles && nwg <= 32) {
        // one item a tile, so workgroup w's run of items is its own tiles:
        // runs are claimed by bit in c[0], this workgroup's own run first
        // (its values then stay in registers for the encode), then every run
        // not claimed yet (so no item waits on a workgroup that has not
        // started; the runs of the ones that have are theirs by then)
        if (threadIdx.x == 0) s_item = __hip_atomic_fetch_or(&c[0], 1u << wg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const bool mine = ((__builtin_amdgcn_readfirstlane(s_item) >> wg) & 1u) == 0;
        __syncthreads();  // (s_item is written again below)
        PSF_STAMP_AT(6);
        if (mine) {
          own = t0 < t1 && t1 <= tf && t1 - t0 <= 2;
          if (own) {
            if (t1 - t0 == 2) {
              V v0[4][4];  // (load_tile fills v)
#pragma unroll
              for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) v0[u][j] = v[u][j];
              load_tile(t0 + 1);
#pragma unroll
              for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  v2[u][j] = v[u][j];
                  v[u][j] = v0[u][j];
                }
            }
            minmax_run_regs<V, CAP>(B, jb, mm_wg0 + (uint32_t)t0, (uint32_t)(t1 - t0), v, v2, &c[1]);
          } else {
            items(min(wg * per, (uint32_t)J.mm_nwg), min(wg * per + per, (uint32_t)J.mm_nwg));
          }
        }
        PSF_STAMP_AT(7);
        const uint32_t all = nwg == 32 ? ~0u : (1u << nwg) - 1u;
        if (threadIdx.x == 0) s_item = __hip_atomic_fetch_or(&c[0], all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (uint32_t left = all & ~__builtin_amdgcn_readfirstlane(s_item); left; left &= left - 1) {
          const uint32_t r = (uint32_t)__builtin_ctz(left);
          items(min(r * per, (uint32_t)J.mm_nwg), min(r * per + per, (uint32_t)J.mm_nwg));
        }
      } else {
        // one claim per workgroup of a run of ceil(items / workgroups) items
        // (every item then belongs to a workgroup that is running: the first
        // ones to start take them all); the run's bounds read into scalar
        // registers, so its loop is uniform for the compiler too
        if (threadIdx.x == 0) s_item = __hip_atomic_fetch_add(&c[0], per, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t i0 = __builtin_amdgcn_readfirstlane(s_item);
        items(i0, i0 + per < (uint32_t)J.mm_nwg ? i0 + per : (uint32_t)J.mm_nwg);
      }
      PSF_STAMP_AT(4);
      if (threadIdx.x == 0) s_late = wait_ready(&c[1], J.mm_nwg) ? 0u : 1u;
#ifdef PSF_FUSED_DEBUG
      if (threadIdx.x == 0 && s_late != 0)
        printf("fused: job %d wg %u timed out: claims %u ready %u done %u want %u\n", jb, wg, c[0], c[1], c[2], (uint32_t)J.mm_nwg);
#endif
      __syncthreads();
      PSF_STAMP_AT(5);
      late = __builtin_amdgcn_readfirstlane(s_late) != 0;
      for (uint32_t i = threadIdx.x; i < J.mm_nwg; i += kBlock) {
        const K a = __hip_atomic_load(&pp[mm_wg0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const K b = __hip_atomic_load(&pp[B.mm_total + mm_wg0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
      }
    } else {
      for (uint32_t i = threadIdx.x; i < J.mm_nwg; i += kBlock) {
        const K a = pp[mm_wg0 + i], b = pp[B.mm_total + mm_wg0 + i];
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
      }
    }
    block_minmax(lo, hi);
    float cmn, cmx;
    if (sizeof(V) == 4) {
      const float lo_v = key_f32((uint32_t)lo), hi_v = key_f32((uint32_t)hi);
      cmn = lo_v;
      cmx = (float)((double)hi_v + 1e-6);
    } else {
      const double lo_v = key_f64((uint64_t)lo), hi_v = key_f64((uint64_t)hi);
      cmn = (float)lo_v;
      cmx = (float)(hi_v + 1e-6);
    }
    if (!(J.flags & 1u)) mn_f = cmn;
    if (!(J.flags & 2u)) mx_f = cmx;
  }
  QuantParams q;
  q.min_v = (double)mn_f;
  q.max_v = (double)mx_f;
  q.bin = q.max_v - q.min_v;
  q.ratio = B.ratio;
  q.scale = q.ratio / q.bin;
  q.min_f = mn_f;
  q.max_f = mx_f;
  q.scale_f = (float)q.scale;
  q.fast = q.bin < __builtin_huge_val();
  PSF_STAMP_AT(1);
  if (wg == 0 && threadIdx.x == 0) {
    const int status = late ? kErrHip : (q.bin > 0) ? kOk : kErrBin;
    if (J.lazy != kNoLazy) {
      float* r = B.range_base + 4 * (uint32_t)J.lazy;  // read by a later decode on this stream
      r[0] = mn_f;
      r[1] = mx_f;
      reinterpret_cast<int32_t*>(r)[2] = status;
      if (B.ring_base) {  // read by the host when it settles the FilterConfig
        float* h = B.ring_base + 4 * (uint32_t)J.lazy;
        h[0] = mn_f;
        h[1] = mx_f;
        reinterpret_cast<int32_t*>(h)[2] = status;
      }
    }
    if (J.flags >> 16) {
      PubSlot* ps = B.pub + ((J.flags >> 16) - 1);
      pub_store(&ps->range[0], mn_f);
      pub_store(&ps->range[1], mx_f);
      pub_store(&ps->status, (int32_t)status);
      publish_ticket(ps, J.ticket);
    }
  }
  if (late && sticky && threadIdx.x == 0) pub_store(sticky, (int32_t)kErrHip);  // Context::sync throws
  if (!(q.bin > 0) || late) return jb;  // CHECK_GT(bin, 0), fixing_float.h:71

  // the next full tile: from registers on the own-tile path, else loaded
  auto next_tile = [&](size_t t) {
    if (own && t == t0 + 1) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = v2[u][j];
    } else {
      load_tile(t);
    }
  };
  EncodeParams p{};  // the per-launch constants the tile code reads
  p.lcg_bits = B.lcg_bits;
  p.lcg_pos = J.u.e.lcg_pos;
  const bool stored = kStored && (NB == 1 || NB == 2) && (J.flags & kFlagStored);
  const StoredLayout L = stored_layout((uint32_t)(n * NB));
  if constexpr (kStored && (NB == 1 || NB == 2)) {
    if (stored) {
      if (wg == 0)  // every fragment's tag, and the header
        for (uint32_t k = threadIdx.x; k <= L.last; k += kBlock) stored_put_prefix(out, L, k);
      for (size_t t = t0; t < tf; ++t) {
        if (t != t0) next_tile(t);
        const size_t gb = t * kTileGroups + threadIdx.x;
        encode_full_tile<V, NB, true>(v, x, q, p, out, gb, gb, &L);
      }
    }
  }
  if (!stored) {
    for (size_t t = t0; t < tf; ++t) {
      if (t != t0) next_tile(t);
      encode_full_tile<V, NB>(v, x, q, p, out, t * kTileGroups + threadIdx.x, t * kTileGroups + threadIdx.x);
    }
  }
  for (size_t t = (t0 > tf ? t0 : tf); t < t1; ++t) {
    const size_t gb = t * kTileGroups + threadIdx.x;
    if constexpr (kStored && (NB == 1 || NB == 2)) {
      if (stored) encode_partial_tile<V, NB, true>(x, al, ngroups, q, p, out, gb, &L);
      else encode_partial_tile<V, NB>(x, al, ngroups, q, p, out, gb);
    } else {
      encode_partial_tile<V, NB>(x, al, ngroups, q, p, out, gb);
    }
  }
  const size_t tail = ngroups << 2;
  if (wg == 0 && threadIdx.x == 0 && tail < n) {
    uint32_t st = lcg_jump(J.u.e.seed, tail);
    for (size_t i = tail; i < n; ++i) {
      uint64_t r = quant_floor<V, NB>(x[i], q) + lcg_bit(st);
      for (int j = 0; j < NB; ++j) {
        if (kStored && stored) stored_put_byte(out, L, (uint32_t)(i * NB + j), (uint8_t)(r & 0xFF));
        else out[i * NB + j] = (uint8_t)(r & 0xFF);
        r >>= 8;
      }
    }
  }
  return jb;
}

template <typename V, int NB, int CAP, bool kStored>
__global__ __launch_bounds__(kBlock) void ff_encode_batch(FfBatchT<CAP> B) {
  encode_batch_body<V, NB, CAP, kStored>(B, blockIdx.x, nullptr);
}

template <typename V, int NB, int CAP>
__device__ __forceinline__ void decode_batch_body(const FfBatchT<CAP>& B, uint32_t block) {
  const int jb = batch_job(B, block, false);
  const FfJob& J = B.job[jb];
  const uint8_t* __restrict__ code = static_cast<const uint8_t*>(J.x);
  V* __restrict__ out = static_cast<V*>(J.out);
  const size_t n = J.n;
  const uint32_t wg = block - B.first[jb];
  const size_t ngroups = n >> 2;
  const size_t ntiles = (ngroups + kTileGroups - 1) / kTileGroups;
  size_t t0, t1;
  tile_range_of(ntiles, wg, batch_nwg(B, jb), t0, t1);
  // nb = 1: the first tile's code words before the range read and the table
  // build (as ff_decode)
  uint32_t w0[4];
  if (NB == 1 && t0 < t1) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(code);
    const size_t gb = t0 * kTileGroups + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t g = gb + u * kBlock;
      w0[u] = c32[g < ngroups ? g : ngroups - 1];
    }
  }
  float mn_f = J.mn, mx_f = J.mx;
  if (J.u.range) { mn_f = J.u.range[0]; mx_f = J.u.range[1]; }
  const double min_v = (double)mn_f, max_v = (double)mx_f;
  const double bin = max_v - min_v;
  const double ratio = B.ratio;
  __shared__ V lut[256];
  if (NB == 1) {
    lut[threadIdx.x] = dequant<V>((uint64_t)threadIdx.x, ratio, bin, min_v);
    lds_barrier();
    if (t0 < t1) {
      const size_t gb = t0 * kTileGroups + threadIdx.x;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t g = gb + u * kBlock;
        if (g < ngroups) {
          V v[4] = {lut[w0[u] & 0xFF], lut[(w0[u] >> 8) & 0xFF], lut[(w0[u] >> 16) & 0xFF], lut[w0[u] >> 24]};
          Vec4<V>::store(out + 4 * g, v);
        }
      }
      ++t0;
    }
  }
  for (size_t t = t0; t < t1; ++t)
    decode_tile<V, NB>(code, out, t * kTileGroups + threadIdx.x, ngroups, lut, ratio, bin, min_v);
  if (wg == 0) {
    for (size_t i = (ngroups << 2) + threadIdx.x; i < n; i += kBlock) {
      uint64_t r = 0;
      for (int j = 0; j < NB; ++j) r |= (uint64_t)code[i * NB + j] << (8 * j);
      out[i] = dequant<V>(r, ratio, bin, min_v);
    }
  }
}
template <typename V, int NB, int CAP>
__global__ __launch_bounds__(kBlock) void ff_decode_batch(FfBatchT<CAP> B) {
  decode_batch_body<V, NB, CAP>(B, blockIdx.x);
}
// One launch for a decode batch and an independent min/max batch (the round
// trip driver's decode of one phase and the next phase's first encode pass:
// psf_nodes_roundtrip_opts): workgroups [0, D.total) decode, the rest fold.
template <typename V, int NB>
__global__ __launch_bounds__(kBlock) void ff_dec_mm_batch(FfBatchT<kBatchSmall> D, FfBatchT<kBatchSmall> M) {
  if (blockIdx.x < D.total) decode_batch_body<V, NB, kBatchSmall>(D, blockIdx.x);
  else minmax_batch_body<V, kBatchSmall>(M, blockIdx.x - D.total);
}
// One launch for a small batch's min/max and encode, with a pending decode
// batch of the same value type and num_bytes in front (the round trip
// driver's decode of one phase): workgroups [0, D.total) decode, the rest
// encode, each array's encode workgroups folding its min/max items first (the
// hand-off above); the last of an array's workgroups to finish zeroes its
// counter line.
template <typename V, int NB, bool kStored>
__global__ __launch_bounds__(kBlock) void ff_fused_batch(FfBatchT<kBatchSmall> D, FfBatchT<kBatchSmall> B, uint32_t* ctl,
                                                         int32_t* sticky) {
  PSF_STAMP(ts0);
  if (blockIdx.x < D.total) {
    decode_batch_body<V, NB, kBatchSmall>(D, blockIdx.x);
    PSF_TRACE_END(ts0, 0ull);
    return;
  }
  const int jb = encode_batch_body<V, NB, kBatchSmall, kStored>(B, blockIdx.x - D.total, ctl, sticky);
  if (B.job[jb].mm_nwg) {
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t* c = ctl + kFusedLine * jb;
      if (__hip_atomic_fetch_add(&c[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == batch_nwg(B, jb) - 1) {
        __hip_atomic_store(&c[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&c[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&c[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  PSF_TRACE_END(ts0, 0ull);
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

// Only bit 16 of the LCG state is ever observed, and (a*s + c) mod 2^17
// depends only on s mod 2^17, so the encoder reads its bits off the LCG modulo
// 2^17, which is one cycle of
// length 2^17 (a = 1 mod 4, c odd).  Host side: the cycle x_0 = 0,
// x_{k+1} = a x_k + c, the position of every residue on it, and per device a
// bit table T[k] = !bit16(x_k) for k < 2^17 + 64 (wrapped), 16 KiB.
namespace {
struct LcgCycle {
  std::vector<uint32_t> pos;   // pos[x] = k with x_k = x
  std::vector<uint32_t> bits;  // T, packed 32 per word, LSB first
  LcgCycle() : pos(1u << 17), bits(((1u << 17) + 64) / 32, 0u) {
    uint32_t x = 0;
    for (uint32_t k = 0; k < (1u << 17); ++k) {
      pos[x] = k;
      x = (kLcgA * x + kLcgC) & kMask17;
    }
    x = 0;
    for (uint32_t k = 0; k < (1u << 17) + 64; ++k) {
      if (((~x) >> 16) & 1u) bits[k >> 5] |= 1u << (k & 31);
      x = (kLcgA * x + kLcgC) & kMask17;
    }
  }
};
const LcgCycle& lcg_cycle() {
  static const LcgCycle c;
  return c;
}
std::mutex g_lcg_mu;
std::map<int, uint32_t*> g_lcg_dev;  // per device, allocated once, never freed
}  // namespace

static const uint32_t* lcg_bits_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> l(g_lcg_mu);
  auto it = g_lcg_dev.find(dev);
  if (it != g_lcg_dev.end()) return it->second;
  const LcgCycle& c = lcg_cycle();
  uint32_t* d = nullptr;
  if (hipMalloc(&d, c.bits.size() * sizeof(uint32_t)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, c.bits.data(), c.bits.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  g_lcg_dev[dev] = d;
  return d;
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

static int tile_grid(size_t n, int cap) {
  const size_t ntiles = ((n >> 2) + kTileGroups - 1) / kTileGroups;
  size_t g = ntiles < 1 ? 1 : ntiles;
  if (g > (size_t)cap) g = cap;
  return (int)g;
}

static bool enc_perm_mode();

// the LCG jump constants of an encode launch over `grid` workgroups
static void encode_lcg_params(EncodeParams& p, int grid) {
  lcg_affine_pow((uint64_t)grid * kBlock, p.a_thr, p.c_thr);
  p.lcg_pos = lcg_cycle().pos[p.seed & kMask17];
}

template <typename V, int NB, bool kVec>
static void launch_encode(const V* x, size_t n, uint8_t* out, EncodeParams p, hipStream_t st) {
  const int grid = kVec ? tile_grid(n, kStreamGrid) : ff_grid(n);
  // after a strided min/max pass over an array larger than the Infinity
  // Cache (smaller ones stay on chip whatever the order, and the reversed
  // order cost C3's 40 MB arrays 9 %: encode 15.8 -> 17.8 us, tools/ab_perm_c13.sh)
  p.reverse = kVec && p.partials && enc_perm_mode() && (double)n * sizeof(V) > 256.0 * (1 << 20) ? 1u : 0u;
  encode_lcg_params(p, grid);
  psf_launch((ff_encode<V, NB, kVec>), dim3(grid), dim3(kBlock), 0, st, x, n, out, p);
}

template <typename V, bool kVec>
static int dispatch_encode_nb(const V* x, size_t n, int nb, uint8_t* out, EncodeParams p,
                              hipStream_t st) {
  p.lcg_bits = lcg_bits_device();
  if (!p.lcg_bits) return kErrHip;
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
                        hipStream_t st, Profiler* prof, PubSlot* pub, uint32_t ticket, float* range_host) {
  EncodeParams p{};
  p.range_host = range_host;
  p.pub = pub;
  p.ticket = ticket;
  p.has_min = preset.has_min;
  p.has_max = preset.has_max;
  p.preset_min = preset.min_value;
  p.preset_max = preset.max_value;
  p.seed = seed;
  p.ratio = ff_ratio(nb);
  p.range_out = range_out;
  p.status_out = status_out;
  // 16-byte aligned values, 4-byte (nb=2: 8-byte) aligned codes
  const bool vec = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & (nb == 2 ? 7 : 3)) == 0);
  if (!(preset.has_min && preset.has_max)) {
    const int grid = vec ? tile_grid(n, kMinmaxGrid) : (ff_grid(n) < kMinmaxGrid ? ff_grid(n) : kMinmaxGrid);
    ProfScope ps(prof, kKMinmax, st, (double)n * sizeof(V), true);
    if (vec)
      psf_launch((ff_minmax_partials<V, true>), dim3(grid), dim3(kBlock), 0, st, x, n, partials,
                         1u);  // strided at every size: C3 (40 MB) 3756 -> 3837 GiB/s
    else
      psf_launch((ff_minmax_partials<V, false>), dim3(grid), dim3(kBlock), 0, st, x, n, partials, 0u);
    p.partials = partials;
    p.nparts = grid;
    if (launch_status() != kOk) return kErrHip;
  }
  ProfScope ps(prof, kKEncode, st, (double)n * (sizeof(V) + nb), true);
  int s = vec ? dispatch_encode_nb<V, true>(x, n, nb, out, p, st)
              : dispatch_encode_nb<V, false>(x, n, nb, out, p, st);
  return s == kOk ? launch_status() : s;
}

int ff_encode_launch(const void* x, size_t n, int value_type, int nb, const FixedPoint& preset,
                     uint32_t seed, void* out, void* partials, float* range_out, int* status_out,
                     hipStream_t st, Profiler* prof, PubSlot* pub, uint32_t ticket, float* range_host) {
  if (nb <= 0 || nb >= 8) return kErrNbytes;
  if (n == 0) return kOk;
  if (value_type == kFloat)
    return encode_typed<float>(static_cast<const float*>(x), n, nb, preset, seed,
                               static_cast<uint8_t*>(out), partials, range_out, status_out, st, prof,
                               pub, ticket, range_host);
  if (value_type == kDouble)
    return encode_typed<double>(static_cast<const double*>(x), n, nb, preset, seed,
                                static_cast<uint8_t*>(out), partials, range_out, status_out, st, prof,
                                pub, ticket, range_host);
  return kErrArg;
}

template <typename V, int NB, bool kVec>
static void launch_decode(const uint8_t* code, size_t n, V* out, const DecodeParams& p,
                          hipStream_t st) {
  // arrays of >= 2 x kDecodeGridBig tiles (2^28 values) decode on twice the
  // stream grid, 2 tiles per workgroup: decode 193-194 -> 189 us at 2^28
  // (tools/ab_c2.sh, r02); the encode and smaller arrays measured no gain
  // from it (2^27 on one tile per workgroup: -2.5 %)
  const size_t tiles = ((n >> 2) + kTileGroups - 1) / kTileGroups;
  const int cap = tiles >= 2 * (size_t)kDecodeGridBig ? kDecodeGridBig : kStreamGrid;
  const int grid = (kVec && NB <= 3) ? tile_grid(n, cap) : ff_grid(n);
  psf_launch((ff_decode<V, NB, kVec>), dim3(grid), dim3(kBlock), 0, st, code, n, out, p);
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
  ProfScope ps(prof, kKDecode, st, (double)n * (nb + vsz), true);
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


// ------------------------------------------------------ batched launchers ---
bool ff_batchable(const void* x, const void* out, size_t n, int nb, int value_type, bool encode) {
  if (nb < 1 || nb > 3 || n == 0 || n >= (1ull << 32)) return false;
  const uintptr_t xa = reinterpret_cast<uintptr_t>(x), oa = reinterpret_cast<uintptr_t>(out);
  const uintptr_t code_align = nb == 2 ? 7 : 3;
  // encode: values element-aligned (slices of a value array, message.h:141-143,
  // start at any element; the batched kernels load unaligned groups element
  // by element), codes aligned for the packed stores
  const uintptr_t elem_align = value_type == kDouble ? 7 : 3;
  return encode ? ((xa & elem_align) == 0 && (oa & code_align) == 0)
                : ((oa & 15) == 0 && (xa & code_align) == 0);
}

template <typename V, int NB, int CAP>
static void launch_encode_batch(FfBatchT<CAP>& B, uint32_t enc_total, hipStream_t st, Profiler* prof,
                                double bytes_mm, double bytes_enc) {
  if (B.mm_total && !B.mm_total_done) {
    ProfScope ps(prof, kKMinmax, st, bytes_mm, true);
    psf_launch((ff_minmax_batch<V, CAP>), dim3(B.mm_total), dim3(kBlock), 0, st, B);
  }
  ProfScope pe(prof, kKEncode, st, bytes_enc, true);
  bool stored = false;
  for (int i = 0; i < B.njobs; ++i) stored |= (B.job[i].flags & kFlagStored) != 0;
  if (stored && (NB == 1 || NB == 2))
    psf_launch((ff_encode_batch<V, NB, CAP, true>), dim3(enc_total), dim3(kBlock), 0, st, B);
  else
    psf_launch((ff_encode_batch<V, NB, CAP, false>), dim3(enc_total), dim3(kBlock), 0, st, B);
}

static size_t tiles_of(size_t n) { return ((n >> 2) + kTileGroups - 1) / kTileGroups; }

// the batched min/max pass's grid (shared by its arrays by tiles): larger than
// the single-array one -- 4096 measured 9 % faster than 1024 on C4's 512 x 1 MiB
// slices (8192: 4 % more), where 1024 is best for one 1 GiB array (tools/ab_c4.sh, r02)
#ifndef PSF_BATCH_MINMAX_GRID
#define PSF_BATCH_MINMAX_GRID 16384  // r06: 16384 against 8192 on C4, min/max 86.8 -> 83.3 us (4786 -> 4803 GiB/s; 32768: 91.6)
#endif
constexpr int kBatchMinmaxGrid = PSF_BATCH_MINMAX_GRID;
#ifndef PSF_BATCH_STREAM_GRID
#define PSF_BATCH_STREAM_GRID 16384  // the batched encode grid: 16384 measured 4 % faster than 8192 on C4
#endif
constexpr int kBatchStreamGrid = PSF_BATCH_STREAM_GRID;
static_assert(kBatchMinmaxGrid <= 0xFFFF, "FfJob::mm_nwg is 16 bits");

// fewest tiles per workgroup in the batched min/max and encode grids
#ifndef PSF_BATCH_MM_TPW
#define PSF_BATCH_MM_TPW 1
#endif
#ifndef PSF_BATCH_ENC_TPW
#define PSF_BATCH_ENC_TPW 2  // 2 measured 10 % faster than 1 on 64 x 1 MiB batches (r02)
#endif
#ifndef PSF_BATCH_DEC_TPW
#define PSF_BATCH_DEC_TPW 1  // one tile per workgroup measured best for decode
#endif
constexpr size_t kBatchMmTpw = PSF_BATCH_MM_TPW, kBatchEncTpw = PSF_BATCH_ENC_TPW, kBatchDecTpw = PSF_BATCH_DEC_TPW;
// at most this many min/max workgroups per array: every encode workgroup of
// the array folds all of its partials before it quantises, so a few large
// arrays (C5: 8 x 2^24 values, 1024 partials each from the 8192 grid) pay for
// the fold in every one of their ~2048 encode workgroups (C5, tools/ab_ff.sh:
// 128 per array gives encode 116 us against 131 at 1024, min/max 84 -- the
// 1024-workgroup total the single-array kernel uses for one 1 GiB array; C4's
// 512 small arrays get 16 each and are unaffected)
#ifndef PSF_BATCH_MM_PER_ARRAY
#define PSF_BATCH_MM_PER_ARRAY 128
#endif
constexpr uint32_t kBatchMmPerArray = PSF_BATCH_MM_PER_ARRAY;

// Workgroups of one array in a batched launch: its share (by tiles) of the
// grid the single-array kernel would use, at least one.  A batch of large
// arrays then runs several tiles per workgroup as the single kernels do
// instead of one workgroup per tile (C4: 32 x 2^21 values).
static int share_grid(size_t n, size_t tiles_total, int cap) {
  const size_t t = tiles_of(n);
  size_t c = tiles_total ? ((size_t)cap * t + tiles_total - 1) / tiles_total : (size_t)cap;
  if (c < 1) c = 1;
  if (c > (size_t)cap) c = cap;
  return tile_grid(n, (int)c);
}

// an upper bound of the min/max workgroups of ff_encode_batch_launch (each
// array's share_grid is at most its tile_grid)
size_t ff_batch_partials_bytes(const FfArray* arrs, int count) {
  size_t wgs = 0;
  for (int i = 0; i < count; ++i)
    if (!(arrs[i].preset.has_min && arrs[i].preset.has_max)) wgs += tile_grid(arrs[i].n, kBatchMinmaxGrid);
  return 2 * sizeof(uint64_t) * (wgs + 1);
}

// PSF_MM_REVERSE (A/B knob, tools/): 1 always, 0 never; unset: never
static bool mm_reverse_mode(double bytes_mm) {
  static const int mode = [] {
    const char* e = getenv("PSF_MM_REVERSE");
    return e && *e ? atoi(e) : 0;
  }();
  (void)bytes_mm;
  return mode == 1;
}

// PSF_ENC_PERM (A/B knob, tools/ab_perm.sh): 0 keeps the min/max pass in
// contiguous runs per workgroup and the encode in tile order.  On (default):
// the strided min/max pass sweeps the array front to back (2^28: 159 -> 156
// us) and the encode starts from the end it read last; the Infinity Cache
// share that buys is small (encode 220 -> 222 us at 2^28, the 2^27 line
// 1743 -> 1768 GiB/s; profiles/r04_ab_perm.txt).  (Interleaving the encode
// over the min/max runs' last chunks instead cost it 219 -> 237 us.)
static bool enc_perm_mode() {
  static const bool on = [] {
    const char* e = getenv("PSF_ENC_PERM");
    return !(e && *e == '0');
  }();
  return on;
}

template <int CAP>
static int fill_decode_batch(FfBatchT<CAP>& B, int value_type, int nb, const FfDecArray* arrs, int count,
                             double* bytes_out, size_t tpw = 1);

// PSF_FF_FUSED (A/B knob, tools/): 0 keeps a small batch's min/max and
// encode in two launches
static bool fused_mode() {
  static const bool on = [] {
    const char* e = getenv("PSF_FF_FUSED");
    return !(e && *e == '0');
  }();
  return on;
}
// ff_fused_batch only for batches of at most this many encode workgroups:
// its waiting workgroups hold their slots (and poll), which a launch-bound
// batch of small arrays (C1: 832) does not notice and one of large arrays
// does (C5, 8 x 2^24 values, 16384 workgroups: 1.08 ms against 0.20 in two
// launches, tools/ab_fused.sh r04).  1024 keeps the grid about within one
// round of resident workgroups (5 per CU at its registers); sizes between
// (C4's 64 slices per rank at N = 8: 2048) are unmeasured and keep two launches.
constexpr uint32_t kFusedMaxEncWgs = 1024;
// tiles per decode workgroup inside ff_fused_batch: 4 (C1, tools/ab_fused_tpw.sh
// r04: the fused kernel 28.1-28.8 us at 1, 27.4-28.5 at 2, 25.6-26.7 at 4,
// 25.6-26.1 at 8; fewer, longer decode workgroups leave the encode ones their
// slots sooner); A/B knob PSF_FUSED_DEC_TPW
static size_t fused_dec_tpw() {
  static const size_t v = [] {
    const char* e = getenv("PSF_FUSED_DEC_TPW");
    const int t = e ? atoi(e) : 0;
    return t >= 1 && t <= 16 ? (size_t)t : (size_t)4;
  }();
  return v;
}

template <typename V, int NB>
static void launch_fused(const FfBatchT<kBatchSmall>& D, const FfBatchT<kBatchSmall>& B, dim3 grid, hipStream_t st,
                         FfFusedCtl* fc, bool stored) {
  if constexpr (NB == 1 || NB == 2) {
    if (stored) {
      psf_launch((ff_fused_batch<V, NB, true>), grid, dim3(kBlock), 0, st, D, B, fc->ctl, fc->sticky);
      return;
    }
  }
  psf_launch((ff_fused_batch<V, NB, false>), grid, dim3(kBlock), 0, st, D, B, fc->ctl, fc->sticky);
}

template <int CAP>
static int encode_batch_cap(int value_type, int nb, const FfArray* arrs, int count, void* partials,
                            PubSlot* pub_base, hipStream_t st, Profiler* prof, const FfDecArray* dec, int ndec,
                            int dec_nb, FfFusedCtl* fused) {
  static FfBatchT<CAP> B;  // host staging of the kernel arguments (launches are serialised per thread)
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  memset(&B, 0, sizeof(B));
  for (int i = 0; i < CAP; ++i) B.first[i] = B.mm_first[i] = ~0u;
  B.njobs = count;
  B.partials = partials;
  B.pub = pub_base;
  B.lcg_bits = lcg_bits_device();
  if (!B.lcg_bits) return kErrHip;
  B.ratio = ff_ratio(nb);
  uint32_t mm = 0, enc = 0;
  double bytes_mm = 0, bytes_enc = 0;
  const size_t vsz = value_type == kFloat ? 4 : 8;
  size_t tiles_mm = 0, tiles_all = 0;
  for (int i = 0; i < count; ++i) {
    tiles_all += tiles_of(arrs[i].n);
    if (!(arrs[i].preset.has_min && arrs[i].preset.has_max)) tiles_mm += tiles_of(arrs[i].n);
  }
  // the lazy jobs' records are 16-byte entries of one device array and one
  // host-mapped ring (one RangeBatch per encode call, filters.cc): kept as a
  // base pointer each plus a per-job index
  for (int i = 0; i < count; ++i) {
    if (arrs[i].range && (!B.range_base || arrs[i].range < B.range_base)) {
      B.range_base = arrs[i].range;
      B.ring_base = arrs[i].range_host;
    }
  }
  for (int i = 0; i < count; ++i) {
    const FfArray& a = arrs[i];
    FfJob& J = B.job[i];
    if (a.n >= (1ull << 32) || a.slot < -1 || a.slot >= 0xFFFF) return kErrArg;
    J.x = a.x;
    J.out = a.out;
    J.n = (uint32_t)a.n;
    J.mn = a.preset.min_value;
    J.mx = a.preset.max_value;
    J.flags = (a.preset.has_min ? 1u : 0u) | (a.preset.has_max ? 2u : 0u) | ((uint32_t)(a.slot + 1) << 16);
    if (a.stored) {
      if ((nb != 1 && nb != 2) || (reinterpret_cast<uintptr_t>(a.out) & 3)) return kErrArg;
      J.flags |= kFlagStored;
    }
    J.u.e.seed = a.seed;
    J.u.e.lcg_pos = lcg_cycle().pos[a.seed & kMask17];
    J.ticket = a.ticket;
    J.lazy = kNoLazy;
    if (a.range) {
      const ptrdiff_t k = a.range - B.range_base;
      if (k % 4 || k / 4 >= kNoLazy) return kErrArg;
      const bool ring_ok = B.ring_base ? a.range_host == B.ring_base + k : a.range_host == nullptr;
      if (!ring_ok) return kErrArg;
      J.lazy = (uint16_t)(k / 4);
    } else if (a.range_host) {
      return kErrArg;
    }
    uint32_t mm_nwg =
        (a.preset.has_min && a.preset.has_max) ? 0u : (uint32_t)share_grid(a.n, tiles_mm, kBatchMinmaxGrid);
    if (mm_nwg > 1) mm_nwg = std::min<uint32_t>(mm_nwg, (uint32_t)((tiles_of(a.n) + kBatchMmTpw - 1) / kBatchMmTpw));
    mm_nwg = std::min(mm_nwg, kBatchMmPerArray);
    J.mm_nwg = (uint16_t)mm_nwg;
    B.mm_first[i] = mm;
    mm += mm_nwg;
    B.first[i] = enc;
    enc += std::min<uint32_t>((uint32_t)share_grid(a.n, tiles_all, kBatchStreamGrid),
                              (uint32_t)std::max<size_t>(1, (tiles_of(a.n) + kBatchEncTpw - 1) / kBatchEncTpw));
    if (mm_nwg) bytes_mm += (double)a.n * vsz;
    bytes_enc += (double)a.n * (vsz + nb);
  }
  B.total = enc;
  B.mm_total = mm;
  B.mm_reverse = mm_reverse_mode(bytes_mm) ? 1u : 0u;
  if constexpr (CAP == kBatchSmall) {
    // min/max, encode and the pending decode (same num_bytes) in one launch
    if (fused && fused->ctl && B.mm_total > 0 && enc <= kFusedMaxEncWgs &&
        (ndec <= 0 || (ndec <= kBatchSmall && dec_nb == nb)) && fused_mode()) {
      static FfBatchT<kBatchSmall> D;
      double bytes_dec = 0;
      if (ndec > 0) {
        const int fs = fill_decode_batch<kBatchSmall>(D, value_type, dec_nb, dec, ndec, &bytes_dec, fused_dec_tpw());
        if (fs != kOk) return fs;
      } else {
        memset(&D, 0, sizeof(D));
      }
      bool stored = false;
      for (int i = 0; i < count; ++i) stored |= (B.job[i].flags & kFlagStored) != 0;
      const dim3 grid(D.total + enc);  // (the min/max items run in the encode workgroups)
      {
        ProfScope pf(prof, kKFused, st, bytes_dec + bytes_mm + bytes_enc, true);
        if (value_type == kFloat) {
          switch (nb) {
            case 1: launch_fused<float, 1>(D, B, grid, st, fused, stored); break;
            case 2: launch_fused<float, 2>(D, B, grid, st, fused, stored); break;
            default: launch_fused<float, 3>(D, B, grid, st, fused, stored); break;
          }
        } else {
          switch (nb) {
            case 1: launch_fused<double, 1>(D, B, grid, st, fused, stored); break;
            case 2: launch_fused<double, 2>(D, B, grid, st, fused, stored); break;
            default: launch_fused<double, 3>(D, B, grid, st, fused, stored); break;
          }
        }
      }
      return launch_status();
    }
  }
  if (ndec > 0) {
    // the pending decode batch: in the min/max launch when both are small
    // (one launch instead of two), else on its own first
    const bool merge = CAP == kBatchSmall && ndec <= kBatchSmall && B.mm_total > 0 && dec_nb >= 1 && dec_nb <= 3;
    if (!merge) {
      const int ds = ff_decode_batch_launch(value_type, dec_nb, dec, ndec, st, prof);
      if (ds != kOk) return ds;
    } else if constexpr (CAP == kBatchSmall) {
      static FfBatchT<kBatchSmall> D;
      double bytes_dec = 0;
      const int fs = fill_decode_batch<kBatchSmall>(D, value_type, dec_nb, dec, ndec, &bytes_dec, kBatchDecTpw);
      if (fs != kOk) return fs;
      const FfBatchT<kBatchSmall>& M = B;
      const dim3 grid(D.total + M.mm_total);
      {
        ProfScope pm(prof, kKDecodeMinmax, st, bytes_dec + bytes_mm, true);
        if (value_type == kFloat) {
          switch (dec_nb) {
            case 1: psf_launch((ff_dec_mm_batch<float, 1>), grid, dim3(kBlock), 0, st, D, M); break;
            case 2: psf_launch((ff_dec_mm_batch<float, 2>), grid, dim3(kBlock), 0, st, D, M); break;
            default: psf_launch((ff_dec_mm_batch<float, 3>), grid, dim3(kBlock), 0, st, D, M); break;
          }
        } else {
          switch (dec_nb) {
            case 1: psf_launch((ff_dec_mm_batch<double, 1>), grid, dim3(kBlock), 0, st, D, M); break;
            case 2: psf_launch((ff_dec_mm_batch<double, 2>), grid, dim3(kBlock), 0, st, D, M); break;
            default: psf_launch((ff_dec_mm_batch<double, 3>), grid, dim3(kBlock), 0, st, D, M); break;
          }
        }
      }
      B.mm_total_done = 1;  // the encode launch below skips the min/max pass
    }
  }
  if (value_type == kFloat) {
    switch (nb) {
      case 1: launch_encode_batch<float, 1, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
      case 2: launch_encode_batch<float, 2, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
      default: launch_encode_batch<float, 3, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
    }
  } else {
    switch (nb) {
      case 1: launch_encode_batch<double, 1, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
      case 2: launch_encode_batch<double, 2, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
      default: launch_encode_batch<double, 3, CAP>(B, enc, st, prof, bytes_mm, bytes_enc); break;
    }
  }
  return launch_status();
}

int ff_encode_batch_launch(int value_type, int nb, const FfArray* arrs, int count, void* partials,
                           PubSlot* pub_base, hipStream_t st, Profiler* prof, const FfDecArray* dec, int ndec,
                           int dec_nb, FfFusedCtl* fused) {
  if (count <= 0) return ndec > 0 ? ff_decode_batch_launch(value_type, dec_nb, dec, ndec, st, prof) : kOk;
  if (count > kFfBatchMax) return kErrArg;
  if (value_type != kFloat && value_type != kDouble) return kErrArg;
  return count <= kBatchSmall ? encode_batch_cap<kBatchSmall>(value_type, nb, arrs, count, partials, pub_base, st, prof,
                                                              dec, ndec, dec_nb, fused)
                              : encode_batch_cap<kFfBatchMax>(value_type, nb, arrs, count, partials, pub_base, st, prof,
                                                              dec, ndec, dec_nb, nullptr);
}

// a decode batch's kernel arguments
template <int CAP>
static int fill_decode_batch(FfBatchT<CAP>& B, int value_type, int nb, const FfDecArray* arrs, int count,
                             double* bytes_out, size_t tpw) {
  memset(&B, 0, sizeof(B));
  for (int i = 0; i < CAP; ++i) B.first[i] = B.mm_first[i] = ~0u;
  B.njobs = count;
  B.ratio = ff_ratio(nb);
  uint32_t wg = 0;
  double bytes = 0;
  const size_t vsz = value_type == kFloat ? 4 : 8;
  for (int i = 0; i < count; ++i) {
    if (arrs[i].n >= (1ull << 32)) return kErrArg;
    FfJob& J = B.job[i];
    J.x = arrs[i].code;
    J.out = arrs[i].out;
    J.n = (uint32_t)arrs[i].n;
    J.mn = arrs[i].mn;
    J.mx = arrs[i].mx;
    J.u.range = arrs[i].range;
    B.first[i] = wg;
    wg += std::min<uint32_t>((uint32_t)tile_grid(arrs[i].n, kStreamGrid),
                             (uint32_t)std::max<size_t>(1, (tiles_of(arrs[i].n) + tpw - 1) / tpw));
    bytes += (double)arrs[i].n * (vsz + nb);
  }
  B.total = wg;
  *bytes_out = bytes;
  return kOk;
}

template <int CAP>
static int decode_batch_cap(int value_type, int nb, const FfDecArray* arrs, int count, hipStream_t st,
                            Profiler* prof) {
  static FfBatchT<CAP> B;
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  double bytes = 0;
  const int fs = fill_decode_batch<CAP>(B, value_type, nb, arrs, count, &bytes, kBatchDecTpw);
  if (fs != kOk) return fs;
  const uint32_t wg = B.total;
  ProfScope ps(prof, kKDecode, st, bytes, true);
  if (value_type == kFloat) {
    switch (nb) {
      case 1: psf_launch((ff_decode_batch<float, 1, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
      case 2: psf_launch((ff_decode_batch<float, 2, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
      default: psf_launch((ff_decode_batch<float, 3, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
    }
  } else {
    switch (nb) {
      case 1: psf_launch((ff_decode_batch<double, 1, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
      case 2: psf_launch((ff_decode_batch<double, 2, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
      default: psf_launch((ff_decode_batch<double, 3, CAP>), dim3(wg), dim3(kBlock), 0, st, B); break;
    }
  }
  return launch_status();
}

int ff_decode_batch_launch(int value_type, int nb, const FfDecArray* arrs, int count, hipStream_t st,
                           Profiler* prof) {
  if (count <= 0) return kOk;
  if (count > kFfBatchMax) return kErrArg;
  return count <= kBatchSmall ? decode_batch_cap<kBatchSmall>(value_type, nb, arrs, count, st, prof)
                              : decode_batch_cap<kFfBatchMax>(value_type, nb, arrs, count, st, prof);
}

}  // namespace psf

// diagnostic: the in-launch hand-off's bound in 100 MHz ticks on the current
// device (0 = the default); a tiny bound drives ff_fused_batch's late path
extern "C" int psf_debug_set_handoff_ticks(uint64_t ticks) {
  const uint64_t v = ticks ? ticks : psf::kHandoffTicks;
  return hipMemcpyToSymbol(HIP_SYMBOL(psf::g_handoff_ticks), &v, sizeof(v)) == hipSuccess ? 0 : -1;
}
