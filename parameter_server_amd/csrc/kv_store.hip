// Server-side consumers of a received message, fused with the FIXING_FLOAT
// dequantise.  The reference runs them after
// RemoteNode::DecodeMessage has materialised the decoded value array; here the
// codes are dequantised in registers with the decode's exact arithmetic
// (fixing_float.h:89-101, bit-identical to ff_decode) and consumed at once, so
// the n*sizeof(V) decoded array is never written or re-read.
//
//   ordered_match   ParallelOrderedMatch (src/util/parallel_ordered_match.h:7-83)
//                   as KVVector::SetValue / GetValue call it
//                   (src/parameter/kv_vector.h:182-183,205-207,237): for every
//                   src key also in dst (both sorted),
//                   dst_val[j*k+i] op= src_val[s*k+i].
//   kvmap_*         KVMap<Key, float, FTRLEntry, SGDState>
//                   (src/parameter/kv_map.h:69-91,
//                   src/app/linear_method/async_sgd.h:89-154): the async-SGD
//                   server's model as an open-addressing hash table in HBM;
//                   SetValue = FTRLEntry::Set per key, GetValue = w per key.
//
// Compiled with -ffp-contract=off like every codec file: the reference's float
// expressions are evaluated operation by operation (g++/x86-64 SSE, no FMA).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "psf_internal.h"

namespace psf {

// ----------------------------------------------------- value sources ------
// Element e of a FIXING_FLOAT code array of nb bytes, dequantised exactly as
// ff_decode does (r accumulated as an integer, one double divide/multiply/add).
struct CodeSrc {
  const uint8_t* code;
  int nb;
  double ratio, bin, min_v;
};

template <typename V>
__device__ __forceinline__ V dequant_code(const CodeSrc& c, size_t e) {
  uint64_t r = 0;
  for (int j = 0; j < c.nb; ++j) r |= (uint64_t)c.code[e * c.nb + j] << (8 * j);
  const double d = (double)r;
  return (V)(d / c.ratio * c.bin + c.min_v);  // fixing_float.h:97
}

template <typename V>
__device__ __forceinline__ void assign_op(V& right, V left, int op) {  // assign_op.h:10-26
  switch (op) {
    case 0: right = left; break;
    case 1: right += left; break;
    case 2: right -= left; break;
    case 3: right *= left; break;
    case 4: right /= left; break;
  }
}

// first index in [lo, hi) with a[idx] >= key / > key
__device__ __forceinline__ size_t lower_bound_u64(const uint64_t* a, size_t lo, size_t hi, uint64_t key) {
  while (lo < hi) {
    const size_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ size_t upper_bound_u64(const uint64_t* a, size_t lo, size_t hi, uint64_t key) {
  while (lo < hi) {
    const size_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Wave-cooperative bound: every lane of the wave calls it with the same
// arguments; 64 pivots per step narrow [lo, hi) 64-fold, so a search over 10^8
// keys takes 5 dependent loads instead of 27.  Returns the first index in
// [lo, hi) with a[idx] >= key (upper: > key), or hi.
__device__ __forceinline__ size_t wave_bound(const uint64_t* a, size_t lo, size_t hi, uint64_t key,
                                             bool upper) {
  const int lane = threadIdx.x & 63;
  while (hi - lo > 64) {
    const size_t step = (hi - lo + 63) / 64;
    const size_t idx = lo + (size_t)lane * step;
    const bool less = idx < hi && (upper ? a[idx] <= key : a[idx] < key);
    const int c = __popcll(__ballot(less));  // pivots below key: a prefix (sorted)
    const size_t nlo = c > 0 ? lo + (size_t)(c - 1) * step + 1 : lo;
    size_t nhi = lo + (size_t)c * step;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
  }
  const size_t idx = lo + lane;
  const bool less = idx < hi && (upper ? a[idx] <= key : a[idx] < key);
  return lo + (size_t)__popcll(__ballot(less));
}

// ------------------------------------------------------ ordered match ------
// Pairing rule (parallel_ordered_match.h:20-34): both cursors advance on a
// match, so the r-th copy of key K in src pairs with the r-th copy of K in
// dst.  For unique keys (every KVVector key array) r = 0.
//
// A workgroup owns kMatchChunk consecutive src keys.  Thread 0 narrows dst to
// the window [lower_bound(first), upper_bound(last)); the window is streamed
// through LDS in chunks of kMatchLds keys (coalesced loads), and every src key
// binary-searches the one chunk that holds its lower_bound -- the chunk whose
// last key is >= it and whose predecessor's last key is < it.
constexpr int kMatchPer = 4;
constexpr int kMatchChunk = kBlock * kMatchPer;
constexpr int kMatchLds = 4096;  // dst keys staged per chunk (32 KiB)

struct MatchParams {
  const uint64_t* src_key;
  size_t nsrc;
  const void* src_val;   // V[nsrc*k] (plain source)
  CodeSrc codes;         // FIXING_FLOAT source (codes.code != null)
  const uint64_t* dst_key;
  size_t ndst;
  void* dst_val;         // V[ndst*k]
  int64_t* match;        // k > 1: per-src dst row (or -1), consumed by match_apply
  int k, op;
  unsigned long long* matched;  // += matched keys (device counter)
};

template <typename V, bool kCodes>
__device__ __forceinline__ V src_value(const MatchParams& p, size_t e) {
  if (kCodes) return dequant_code<V>(p.codes, e);
  return static_cast<const V*>(p.src_val)[e];
}

template <typename V, bool kCodes>
__global__ __launch_bounds__(kBlock) void ordered_match_kernel(MatchParams p) {
  __shared__ uint64_t s_dst[kMatchLds];
  __shared__ size_t s_win[2];
  __shared__ unsigned s_cnt;
  const size_t c0 = (size_t)blockIdx.x * kMatchChunk;
  const size_t c1 = c0 + kMatchChunk < p.nsrc ? c0 + kMatchChunk : p.nsrc;
  // wave 0: window start, wave 1: window end (two 64-ary searches in parallel)
  if (threadIdx.x < 128) {
    const bool upper = threadIdx.x >= 64;
    const size_t b = wave_bound(p.dst_key, 0, p.ndst, p.src_key[upper ? c1 - 1 : c0], upper);
    if ((threadIdx.x & 63) == 0) s_win[upper ? 1 : 0] = b;
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const size_t w0 = s_win[0], w1 = s_win[1];
  uint64_t key[kMatchPer];
  size_t pos[kMatchPer];  // global lower_bound of key in dst (w1: beyond the window)
#pragma unroll
  for (int u = 0; u < kMatchPer; ++u) {
    const size_t s = c0 + (size_t)u * kBlock + threadIdx.x;
    key[u] = s < c1 ? p.src_key[s] : ~0ull;
    pos[u] = w1;
  }
  for (size_t b0 = w0; b0 < w1; b0 += kMatchLds) {
    const size_t b1 = b0 + kMatchLds < w1 ? b0 + kMatchLds : w1;
    {  // all loads in flight before the LDS stores (one memory latency per chunk)
      uint64_t t[kMatchLds / kBlock];
#pragma unroll
      for (int q = 0; q < kMatchLds / kBlock; ++q) {
        const size_t j = b0 + (size_t)q * kBlock + threadIdx.x;
        t[q] = j < b1 ? p.dst_key[j] : 0;
      }
#pragma unroll
      for (int q = 0; q < kMatchLds / kBlock; ++q) s_dst[q * kBlock + threadIdx.x] = t[q];
    }
    __syncthreads();
    const uint64_t last = s_dst[b1 - b0 - 1];
    const bool first = b0 == w0;
    const uint64_t prev = first ? 0 : p.dst_key[b0 - 1];
#pragma unroll
    for (int u = 0; u < kMatchPer; ++u) {
      if (key[u] <= last && (first || key[u] > prev)) {
        size_t lo = 0, hi = b1 - b0;
        while (lo < hi) {
          const size_t mid = (lo + hi) >> 1;
          if (s_dst[mid] < key[u]) lo = mid + 1; else hi = mid;
        }
        pos[u] = b0 + lo;
      }
    }
    __syncthreads();
  }
  unsigned cnt = 0;
#pragma unroll
  for (int u = 0; u < kMatchPer; ++u) {
    const size_t s = c0 + (size_t)u * kBlock + threadIdx.x;
    if (s >= c1) break;
    // rank of this copy of the key among equal src keys (0 for unique keys)
    size_t r = 0;
    if (s > 0 && p.src_key[s - 1] == key[u]) r = s - lower_bound_u64(p.src_key, 0, s, key[u]);
    const size_t j = pos[u] + r;
    const bool hit = j < w1 && p.dst_key[j] == key[u];
    if (p.k == 1) {
      if (hit) assign_op<V>(static_cast<V*>(p.dst_val)[j], src_value<V, kCodes>(p, s), p.op);
    } else {
      p.match[s] = hit ? (int64_t)j : -1;
    }
    cnt += hit ? 1u : 0u;
  }
  // matched keys (ParallelOrderedMatch's *n is this times k)
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0 && s_cnt) atomicAdd(p.matched, (unsigned long long)s_cnt);
}

// k > 1: one lane per value element; rows are contiguous in src and dst.
template <typename V, bool kCodes>
__global__ __launch_bounds__(kBlock) void match_apply_kernel(MatchParams p) {
  const size_t total = p.nsrc * (size_t)p.k;
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += stride) {
    const size_t s = e / (size_t)p.k;
    const int64_t j = p.match[s];
    if (j < 0) continue;
    const size_t i = e - s * (size_t)p.k;
    assign_op<V>(static_cast<V*>(p.dst_val)[(size_t)j * p.k + i], src_value<V, kCodes>(p, e), p.op);
  }
}

static unsigned grid_for(size_t n) {
  size_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > (size_t)kMaxGrid * 4) g = (size_t)kMaxGrid * 4;
  return (unsigned)g;
}

template <typename V, bool kCodes>
static int launch_match(const MatchParams& p, hipStream_t st, Profiler* prof) {
  const double vsz = (double)sizeof(V);
  const double src_bytes = kCodes ? (double)p.codes.nb : vsz;
  // src keys + src values + the dst key window + a read-modify-write of each
  // matched dst element (counted for every src element: an upper bound)
  const double alg = (double)p.nsrc * (8.0 + p.k * src_bytes + p.k * 2.0 * vsz) + (double)p.ndst * 8.0;
  ProfScope ps(prof, kKMatch, st, alg);
  const size_t blocks = (p.nsrc + kMatchChunk - 1) / kMatchChunk;
  hipLaunchKernelGGL((ordered_match_kernel<V, kCodes>), dim3((unsigned)blocks), dim3(kBlock), 0, st, p);
  if (p.k > 1)
    hipLaunchKernelGGL((match_apply_kernel<V, kCodes>), dim3(grid_for(p.nsrc * (size_t)p.k)), dim3(kBlock),
                       0, st, p);
  return launch_status();
}

int ordered_match_launch(const uint64_t* src_key, size_t nsrc, const void* src_val, const void* code,
                         int nb, float mn, float mx, const uint64_t* dst_key, size_t ndst, void* dst_val,
                         int k, int value_type, int op, int64_t* match_scratch,
                         unsigned long long* d_matched, hipStream_t st, Profiler* prof) {
  if (k <= 0 || op < 0 || op > 4) return kErrArg;
  if (value_type != kFloat && value_type != kDouble) return kErrArg;
  if (nsrc == 0 || ndst == 0) return kOk;
  MatchParams p{};
  p.src_key = src_key;
  p.nsrc = nsrc;
  p.src_val = src_val;
  p.dst_key = dst_key;
  p.ndst = ndst;
  p.dst_val = dst_val;
  p.match = match_scratch;
  p.k = k;
  p.op = op;
  p.matched = d_matched;
  if (code) {
    if (nb <= 0 || nb >= 8) return kErrNbytes;
    p.codes = CodeSrc{static_cast<const uint8_t*>(code), nb, ff_ratio(nb), (double)mx - (double)mn,
                      (double)mn};
    return value_type == kFloat ? launch_match<float, true>(p, st, prof)
                                : launch_match<double, true>(p, st, prof);
  }
  return value_type == kFloat ? launch_match<float, false>(p, st, prof)
                              : launch_match<double, false>(p, st, prof);
}

// --------------------------------------------------- KVMap (FTRL) ---------
// Slot layout: 32 B, so the probe and the entry it finds share one cache line
// (4 slots per 128 B line).  key == kEmptyKey marks a free slot (the key
// 2^64-1 lies outside every server range: Range::All() is [0, 2^64-1),
// range.h:92-95).  A free slot's payload is zero = FTRLEntry's default state.
struct alignas(32) KvSlot {
  unsigned long long key;
  float w, z, sqrt_n, pad;
  float pad2[2];
};
static_assert(sizeof(KvSlot) == 32, "slot size");
constexpr unsigned long long kEmptyKey = ~0ull;

__device__ __forceinline__ uint64_t kv_hash(uint64_t k) {  // murmur3 fmix64
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

struct FtrlParams {
  float alpha, beta;       // LearningRate<float>: V(conf_.alpha()), V(conf_.beta())
  int lr_decay;            // LearningRateConfig::DECAY (else CONSTANT)
  float lambda1, lambda2;  // ElasticNet<float>
};

// SGDState counters (async_sgd.h:118-125) plus table bookkeeping; mirrored by
// KvMapFtrl::Stats on the host.
struct KvStats {
  long long nnz_delta;
  double weight_sum, delta_sum;
  unsigned long long inserted;
  int status;
  int pad;
};

// FTRLEntry::Set (async_sgd.h:137-151) with LearningRate::eval
// (learning_rate.h:15-22) and ElasticNet::proximal (penalty.h:51-56), float
// arithmetic one operation at a time.
__device__ __forceinline__ float ftrl_set(KvSlot& e, float grad, const FtrlParams& f, int& bad_eta) {
  const float w_old = e.w;
  const float sn = e.sqrt_n;
  const float sum = sn * sn + grad * grad;
  const float sqrt_n_new = __builtin_sqrtf(sum);
  const float sigma = (sqrt_n_new - sn) / f.alpha;
  const float t = grad - sigma * w_old;
  const float z = e.z + t;
  const float eta = f.lr_decay ? f.alpha / (sqrt_n_new + f.beta) : f.alpha;
  const float zz = -z * eta;  // proximal(-z*eta, eta)
  bad_eta |= !(eta > 0.0f) ? 1 : 0;  // CHECK_GT(eta, 0), penalty.h:52
  const float leta = f.lambda1 * eta;
  float w;
  if (zz <= leta && zz >= -leta) {
    w = 0.0f;
  } else {
    const float den = 1.0f + f.lambda2 * eta;
    w = zz > 0.0f ? (zz - leta) / den : (zz + leta) / den;
  }
  e.z = z;
  e.sqrt_n = sqrt_n_new;
  e.w = w;
  return w_old;
}

struct KvPushParams {
  KvSlot* table;
  uint64_t mask;  // capacity - 1 (power of two)
  const uint64_t* keys;
  size_t n;
  const float* grad;  // plain source
  CodeSrc codes;      // FIXING_FLOAT source (codes.code != null)
  FtrlParams f;
  KvStats* stats;
};

template <bool kCodes>
__global__ __launch_bounds__(kBlock) void kvmap_push_kernel(KvPushParams p) {
  __shared__ float s_lut[256];
  if (kCodes && p.codes.nb == 1) {  // the decode's 256-entry table, same formula
    const double d = (double)threadIdx.x;
    s_lut[threadIdx.x] = (float)(d / p.codes.ratio * p.codes.bin + p.codes.min_v);
    __syncthreads();
  }
  long long nnz = 0;
  double wsum = 0.0, dsum = 0.0;
  unsigned ins = 0;
  int bad = 0, full = 0;
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < p.n; i += stride) {
    const unsigned long long key = p.keys[i];
    float g;
    if (kCodes) g = p.codes.nb == 1 ? s_lut[p.codes.code[i]] : dequant_code<float>(p.codes, i);
    else g = p.grad[i];
    uint64_t h = kv_hash(key) & p.mask;
    KvSlot* e = nullptr;
    for (uint64_t probe = 0; probe <= p.mask; ++probe) {
      KvSlot* s = p.table + h;
      const unsigned long long cur = __hip_atomic_load(&s->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == key) { e = s; break; }
      if (cur == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&s->key, kEmptyKey, key);
        if (prev == kEmptyKey) { e = s; ++ins; break; }
        if (prev == key) { e = s; break; }
      }
      h = (h + 1) & p.mask;
    }
    if (!e) { full = 1; continue; }
    const float w_old = ftrl_set(*e, g, p.f, bad);
    const float w_new = e->w;
    // SGDState::UpdateWeight (async_sgd.h:106-116)
    if (w_new == 0.0f && w_old != 0.0f) --nnz;
    else if (w_new != 0.0f && w_old == 0.0f) ++nnz;
    wsum += (double)(w_new * w_new);
    const float delta = w_new - w_old;
    dsum += (double)(delta * delta);
  }
  for (int o = 32; o > 0; o >>= 1) {
    nnz += __shfl_xor(nnz, o, 64);
    wsum += __shfl_xor(wsum, o, 64);
    dsum += __shfl_xor(dsum, o, 64);
    ins += __shfl_xor(ins, o, 64);
    bad |= __shfl_xor(bad, o, 64);
    full |= __shfl_xor(full, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (nnz) atomicAdd(reinterpret_cast<unsigned long long*>(&p.stats->nnz_delta), (unsigned long long)nnz);
    if (wsum != 0.0) atomicAdd(&p.stats->weight_sum, wsum);
    if (dsum != 0.0) atomicAdd(&p.stats->delta_sum, dsum);
    if (ins) atomicAdd(&p.stats->inserted, (unsigned long long)ins);
    if (bad) atomicExch(&p.stats->status, kErrCheck);
    if (full) atomicExch(&p.stats->status, kErrUnsupported);
  }
}

// KVMap::GetValue (kv_map.h:69-77): w of each key; an absent key reads as a
// default entry's w (0).  The reference also inserts that default entry; it
// changes nothing a later call can observe (Set starts from the same zero
// state, WriteToFile skips zero weights), so the lookup does not insert.
__global__ __launch_bounds__(kBlock) void kvmap_get_kernel(const KvSlot* __restrict__ table, uint64_t mask,
                                                           const uint64_t* __restrict__ keys, size_t n,
                                                           float* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const unsigned long long key = keys[i];
    uint64_t h = kv_hash(key) & mask;
    float w = 0.0f;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      const unsigned long long cur = table[h].key;
      if (cur == key) { w = table[h].w; break; }
      if (cur == kEmptyKey) break;
      h = (h + 1) & mask;
    }
    out[i] = w;
  }
}

__device__ __forceinline__ float kv_lookup(const KvSlot* __restrict__ table, uint64_t mask, unsigned long long key) {
  uint64_t h = kv_hash(key) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long cur = table[h].key;
    if (cur == key) return table[h].w;
    if (cur == kEmptyKey) break;
    h = (h + 1) & mask;
  }
  return 0.0f;
}

// The same over a batch of key arrays (a pull step's responses): element i of
// the concatenation belongs to the last job whose `first` is <= i.  A
// workgroup takes chunks of kGetPer x kBlock consecutive elements and finds
// the chunk's first job once (a uniform search); each lane then steps to the
// next job where its element crosses a boundary.  Four lookups per lane are
// in flight at once: each first probe is one 16-byte load of {key, w}, and
// only a probe that lands on another key walks on (linear probing).
constexpr int kGetPer = 16;
#ifndef PSF_GET_INFLIGHT
#define PSF_GET_INFLIGHT 8  // lookups in flight per lane (A/B knob: 4 / 8 / 16 gave 2008 / 1970 / 2814 us at C4pull, r06h)
#endif
constexpr int kGetFly = PSF_GET_INFLIGHT;
static_assert(kGetPer % kGetFly == 0, "whole rounds of lookups per chunk");
__global__ __launch_bounds__(kBlock) void kvmap_get_batch_kernel(const KvSlot* __restrict__ table, uint64_t mask,
                                                                 const KvGetJob* __restrict__ jobs, int njobs,
                                                                 uint64_t total) {
  const uint64_t chunk = (uint64_t)kBlock * kGetPer;
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base < total; base += (uint64_t)gridDim.x * chunk) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].first <= base) lo = mid;
      else hi = mid - 1;
    }
    int j = lo;
    uint64_t jend = jobs[j].first + jobs[j].n;
#pragma unroll 1
    for (int k = 0; k < kGetPer; k += kGetFly) {
      unsigned long long key[kGetFly];
      float* dst[kGetFly];
#pragma unroll
      for (int u = 0; u < kGetFly; ++u) {
        const uint64_t i = base + (uint64_t)(k + u) * kBlock + threadIdx.x;
        dst[u] = nullptr;
        key[u] = kEmptyKey;
        if (i < total) {
          while (i >= jend) {
            ++j;
            jend = jobs[j].first + jobs[j].n;
          }
          const uint64_t e = i - jobs[j].first;
          key[u] = jobs[j].keys[e];
          dst[u] = jobs[j].out + e;
        }
      }
      uint64_t h[kGetFly];
      uint4 sl[kGetFly];
#pragma unroll
      for (int u = 0; u < kGetFly; ++u) {
        h[u] = kv_hash(key[u]) & mask;
        sl[u] = *reinterpret_cast<const uint4*>(&table[h[u]]);  // {key, w, z}
      }
#pragma unroll
      for (int u = 0; u < kGetFly; ++u) {
        if (!dst[u]) continue;
        const unsigned long long cur = (unsigned long long)sl[u].x | ((unsigned long long)sl[u].y << 32);
        float w = 0.0f;
        if (cur == key[u]) w = __uint_as_float(sl[u].z);
        else if (cur != kEmptyKey) w = kv_lookup(table, mask, key[u]);  // (rare: a collision)
        *dst[u] = w;
      }
    }
  }
}

// Re-insert every occupied slot of `from` into the empty table `to` (growth).
__global__ __launch_bounds__(kBlock) void kvmap_rehash_kernel(const KvSlot* __restrict__ from, size_t nfrom,
                                                              KvSlot* to, uint64_t mask) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < nfrom; i += stride) {
    const KvSlot s = from[i];
    if (s.key == kEmptyKey) continue;
    uint64_t h = kv_hash(s.key) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      if (atomicCAS(&to[h].key, kEmptyKey, s.key) == kEmptyKey) {
        to[h].w = s.w;
        to[h].z = s.z;
        to[h].sqrt_n = s.sqrt_n;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

__global__ __launch_bounds__(kBlock) void kvmap_init_kernel(KvSlot* t, size_t n) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    KvSlot s;
    s.key = kEmptyKey;
    s.w = s.z = s.sqrt_n = s.pad = 0.0f;
    s.pad2[0] = s.pad2[1] = 0.0f;
    t[i] = s;
  }
}

size_t kvmap_slot_bytes() { return sizeof(KvSlot); }
size_t kvmap_stats_bytes() { return sizeof(KvStats); }

int kvmap_init_launch(void* table, size_t cap, hipStream_t st) {
  hipLaunchKernelGGL(kvmap_init_kernel, dim3(grid_for(cap)), dim3(kBlock), 0, st,
                     static_cast<KvSlot*>(table), cap);
  return launch_status();
}

int kvmap_rehash_launch(const void* from, size_t nfrom, void* to, size_t cap_to, hipStream_t st) {
  hipLaunchKernelGGL(kvmap_rehash_kernel, dim3(grid_for(nfrom)), dim3(kBlock), 0, st,
                     static_cast<const KvSlot*>(from), nfrom, static_cast<KvSlot*>(to),
                     (uint64_t)cap_to - 1);
  return launch_status();
}

int kvmap_push_launch(void* table, size_t cap, const uint64_t* keys, size_t n, const float* grad,
                      const void* code, int nb, float mn, float mx, float alpha, float beta,
                      int lr_decay, float lambda1, float lambda2, void* stats, hipStream_t st,
                      Profiler* prof) {
  if (n == 0) return kOk;
  KvPushParams p{};
  p.table = static_cast<KvSlot*>(table);
  p.mask = (uint64_t)cap - 1;
  p.keys = keys;
  p.n = n;
  p.grad = grad;
  p.f = FtrlParams{alpha, beta, lr_decay, lambda1, lambda2};
  p.stats = static_cast<KvStats*>(stats);
  // key + gradient (or code) + one 32-byte slot read and written per key
  const double alg = (double)n * (8.0 + (code ? nb : 4) + 64.0);
  ProfScope ps(prof, kKKvPush, st, alg);
  if (code) {
    if (nb <= 0 || nb >= 8) return kErrNbytes;
    p.codes = CodeSrc{static_cast<const uint8_t*>(code), nb, ff_ratio(nb), (double)mx - (double)mn,
                      (double)mn};
    hipLaunchKernelGGL(kvmap_push_kernel<true>, dim3(grid_for(n)), dim3(kBlock), 0, st, p);
  } else {
    hipLaunchKernelGGL(kvmap_push_kernel<false>, dim3(grid_for(n)), dim3(kBlock), 0, st, p);
  }
  return launch_status();
}

int kvmap_get_launch(const void* table, size_t cap, const uint64_t* keys, size_t n, float* out,
                     hipStream_t st, Profiler* prof) {
  if (n == 0) return kOk;
  ProfScope ps(prof, kKKvGet, st, (double)n * (8.0 + 32.0 + 4.0));
  hipLaunchKernelGGL(kvmap_get_kernel, dim3(grid_for(n)), dim3(kBlock), 0, st,
                     static_cast<const KvSlot*>(table), (uint64_t)cap - 1, keys, n, out);
  return launch_status();
}


int kvmap_get_batch_launch(const void* table, size_t cap, const KvGetJob* d_jobs, int njobs, uint64_t total,
                           hipStream_t st, Profiler* prof) {
  if (njobs <= 0 || total == 0) return kOk;
  ProfScope ps(prof, kKKvGet, st, (double)total * (8.0 + 32.0 + 4.0));
  const uint64_t chunks = (total + (uint64_t)kBlock * kGetPer - 1) / ((uint64_t)kBlock * kGetPer);
  const unsigned grid = (unsigned)std::min<uint64_t>(chunks, (uint64_t)kMaxGrid * 4);
  hipLaunchKernelGGL(kvmap_get_batch_kernel, dim3(grid), dim3(kBlock), 0, st,
                     static_cast<const KvSlot*>(table), (uint64_t)cap - 1, d_jobs, njobs, total);
  return launch_status();
}
}  // namespace psf
