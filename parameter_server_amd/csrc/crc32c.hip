// CRC-32C (Castagnoli) on the device -- the KEY_CACHING signature
// (reference src/filter/key_caching.h:18,43 -> util/crc32c.cc:292-335: init ~0,
// final ~0, reflected polynomial 0x82F63B78).
//
// The reference walks the bytes serially (slicing-by-4).  Here every lane CRCs
// its own contiguous chunk against a 1 KiB LDS byte table, then moves its chunk
// CRC to the end of the message with the GF(2) "append n zero bytes" operator
// (multiplication by x^(8n) mod P, zlib's crc32_combine algebra):
//     crc(A1..Ak) = XOR_i  shift(crc(A_i), |A_{i+1}..A_k|)
// The per-lane contributions are XOR-reduced (order-independent, hence
// deterministic) in the wave, then across waves, then across workgroups with
// atomicXor into a zeroed word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psf_internal.h"

namespace psf {

constexpr uint32_t kCrcPoly = 0x82F63B78u;

struct X2nTable { uint32_t v[32]; };  // x^(2^k) mod P, k = 0..31

__host__ __device__ static inline uint32_t multmodp(uint32_t a, uint32_t b) {
  // a*b mod P, bit 31 = x^0 (reflected)
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kCrcPoly : (b >> 1);
  }
  return p;
}

__device__ static inline uint32_t x2nmodp(uint64_t n, unsigned k, const X2nTable& t) {
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp(t.v[k & 31], p);
    n >>= 1;
    ++k;
  }
  return p;
}

__global__ __launch_bounds__(kBlock) void crc32c_chunks(const uint8_t* __restrict__ d, size_t n,
                                                         size_t chunk, uint32_t* __restrict__ out,
                                                         X2nTable tbl, PubSlot* pub, uint32_t ticket) {
  __shared__ uint32_t table[256];
  __shared__ uint32_t wave_acc[kBlock / 64];
  {
    uint32_t c = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kCrcPoly & (0u - (c & 1u)));
    table[threadIdx.x] = c;
  }
  __syncthreads();

  const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t begin = t * chunk;
  uint32_t contrib = 0;
  if (begin < n) {
    const size_t end = begin + chunk < n ? begin + chunk : n;
    uint32_t l = 0xFFFFFFFFu;
    size_t i = begin;
    // 4-byte steps when the chunk start is aligned (chunk is a multiple of 4)
    if (((reinterpret_cast<uintptr_t>(d + begin)) & 3) == 0) {
      for (; i + 4 <= end; i += 4) {
        uint32_t w = *reinterpret_cast<const uint32_t*>(d + i);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          l = table[(l ^ (w >> (8 * b))) & 0xFF] ^ (l >> 8);
        }
      }
    }
    for (; i < end; ++i) l = table[(l ^ d[i]) & 0xFF] ^ (l >> 8);
    const uint32_t c = l ^ 0xFFFFFFFFu;
    contrib = multmodp(x2nmodp(n - end, 3, tbl), c);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
  if ((threadIdx.x & 63) == 0) wave_acc[threadIdx.x >> 6] = contrib;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) acc ^= wave_acc[w];
    if (gridDim.x == 1) {  // whole message in this workgroup: final value
      *out = acc;
      if (pub) publish_crc(pub, acc, ticket);
    } else {
      atomicXor(out, acc);
    }
  }
}

// ---- single-workgroup path (KEY_CACHING: <= 2 KiB, latency-bound) ----------
// Lane t CRCs the 8 bytes [n - 8(256-t), n - 8(255-t)) (clipped at 0, so the
// short chunk is lane 0's), then a shift-and-XOR tree combines neighbours; every
// right-hand block at level j is 8*2^j bytes long, so the operator x^(64*2^j)
// is a compile-time constant, applied as eight nibble-table lookups.
constexpr uint32_t multmodp_c(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kCrcPoly : (b >> 1);
  }
  return p;
}
struct NibbleOps {
  uint32_t t[8][8][16];  // [level j][nibble q][value v] = (v << 4q) * x^(64*2^j) mod P
};
constexpr NibbleOps make_nibble_ops() {
  NibbleOps o{};
  uint32_t k = 1u << 31;  // x^0
  uint32_t x8 = 1u << 23;  // x^8
  // x^64 = (x^8)^8
  uint32_t x64 = 1u << 31;
  for (int i = 0; i < 8; ++i) x64 = multmodp_c(x64, x8);
  k = x64;
  for (int j = 0; j < 8; ++j) {
    for (int q = 0; q < 8; ++q)
      for (uint32_t v = 0; v < 16; ++v) o.t[j][q][v] = multmodp_c(v << (4 * q), k);
    k = multmodp_c(k, k);  // x^(64*2^(j+1))
  }
  return o;
}
__constant__ NibbleOps kNibbleOps = make_nibble_ops();

__device__ __forceinline__ uint32_t shift_op(const uint32_t (*t)[16], uint32_t a) {
  uint32_t r = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) r ^= t[q][(a >> (4 * q)) & 15];
  return r;
}

// CRC32C of d[0:n), n <= kCrcSingleBlock, by the whole workgroup; the value
// is valid in thread 0
__device__ __forceinline__ uint32_t crc_small_block(const uint8_t* __restrict__ d, uint32_t n) {
  __shared__ uint32_t table[256];
  __shared__ uint32_t ops[8][8][16];
  __shared__ uint32_t wave_acc[kBlock / 64];
  const uint32_t t = threadIdx.x;
  // the 8 bytes of this lane (issued first: the longest latency)
  const int64_t e = (int64_t)n - 8 * (int64_t)(kBlock - 1 - t);
  const int64_t b = e - 8;
  uint8_t bytes[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bytes[i] = (b + i >= 0 && b + i < e) ? d[b + i] : 0;
  {
    uint32_t c = t;
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kCrcPoly & (0u - (c & 1u)));
    table[t] = c;
    const uint32_t* src = &kNibbleOps.t[0][0][0];
    uint32_t* dst = &ops[0][0][0];
    for (uint32_t i = t; i < 8 * 8 * 16; i += kBlock) dst[i] = src[i];
  }
  __syncthreads();
  uint32_t v = 0;  // crc32c of this lane's bytes ("" -> 0)
  if (e > 0) {
    uint32_t l = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (b + i >= 0) l = table[(l ^ bytes[i]) & 0xFF] ^ (l >> 8);
    v = l ^ 0xFFFFFFFFu;
  }
  // crc(L || R) = shift(crc(L), |R|) ^ crc(R), |R| = 8 * 2^j at level j
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const uint32_t r = __shfl_down(v, 1u << j, 64);
    if ((t & ((2u << j) - 1)) == 0) v = shift_op(ops[j], v) ^ r;
  }
  if ((t & 63) == 0) wave_acc[t >> 6] = v;
  __syncthreads();
  uint32_t acc = 0;
  if (t == 0) {
    acc = wave_acc[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) acc = shift_op(ops[6], acc) ^ wave_acc[w];  // 512-byte blocks
  }
  return acc;
}

__global__ __launch_bounds__(kBlock) void crc32c_small(const uint8_t* __restrict__ d, uint32_t n,
                                                        uint32_t* __restrict__ out, PubSlot* pub,
                                                        uint32_t ticket) {
  const uint32_t acc = crc_small_block(d, n);
  if (threadIdx.x == 0) {
    *out = acc;
    if (pub) publish_crc(pub, acc, ticket);
  }
}

// many short messages (KEY_CACHING signatures of a batch): workgroup b CRCs
// job b and publishes it to pub[job.slot]
struct CrcBatch {
  const uint8_t* d[kCrcBatchMax];
  uint32_t n[kCrcBatchMax];
  int32_t slot[kCrcBatchMax];
  uint32_t ticket[kCrcBatchMax];
};
__global__ __launch_bounds__(kBlock) void crc32c_small_batch(CrcBatch B, PubSlot* pub) {
  const uint32_t b = blockIdx.x;
  const uint32_t acc = crc_small_block(B.d[b], B.n[b]);
  if (threadIdx.x == 0) {
    publish_crc(pub + B.slot[b], acc, B.ticket[b]);
  }
}

// SliceKOFVMessage's split positions (message.h:107-147) fused with the
// KEY_CACHING signature of every slice (key_caching.h:18), for many messages
// in one launch: workgroup (m, i) finds pos[i] and pos[i + 1] of message m
// (two lanes, one binary search each over the sorted keys), then CRCs the
// first min(2048, slice bytes) key bytes of slice i.  Inputs and results live
// in host-mapped memory: the host reads them once the launch's event has
// completed, with no copy and no stream synchronisation.
template <typename K>
__global__ __launch_bounds__(kBlock) void slice_sig_kernel(SliceSigParams P) {
  __shared__ uint64_t s_pos[2];
  const int ns = P.nslices, nb = ns + 1;
  const int m = blockIdx.x / ns, i = blockIdx.x % ns;
  const K* keys = reinterpret_cast<const K*>(P.desc[2 * m]);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 2) {  // wave w: lower_bound of bound i + w, a 64-ary search (log64 n dependent loads)
    const size_t n = (size_t)P.desc[2 * m + 1];
    const K v = (K)P.bounds[(size_t)m * nb + i + w];
    size_t lo = 0, len = n;  // the first index with keys[idx] >= v lies in [lo, lo + len]
    while (len > 64) {
      // pivots p_k = lo + (k+1) len / 65, strictly increasing; keys[p_k] < v
      // holds for k < c and fails from c on (sorted keys)
      const size_t pk = lo + ((size_t)(lane + 1) * len) / 65;
      const int c = __popcll(__ballot(keys[pk] < v));
      const size_t below = c ? lo + ((size_t)c * len) / 65 + 1 : lo;  // p_{c-1} + 1
      const size_t above = c < 64 ? lo + ((size_t)(c + 1) * len) / 65 : lo + len;  // p_c
      lo = below;
      len = above - below;
    }
    const bool lt = (size_t)lane < len && keys[lo + lane] < v;
    const size_t pos = lo + (size_t)__popcll(__ballot(lt));  // the whole wave votes
    if (lane == 0) s_pos[w] = pos;
  }
  __syncthreads();
  const uint64_t lo = s_pos[0], hi = s_pos[1] > lo ? s_pos[1] : lo;
  const uint64_t bytes = (hi - lo) * sizeof(K);
  const uint32_t len = bytes < kCrcSingleBlock ? (uint32_t)bytes : (uint32_t)kCrcSingleBlock;
  uint32_t crc = 0;
  if (len) crc = crc_small_block(reinterpret_cast<const uint8_t*>(keys + lo), len);
  if (threadIdx.x == 0) {
    uint64_t* pos = P.pos + (size_t)m * nb;
    if (i == 0) pos[0] = s_pos[0];
    pos[i + 1] = s_pos[1];
    P.sig[(size_t)m * ns + i] = crc;
  }
}

int slice_sig_launch(const SliceSigParams& p, int key_bytes, hipStream_t st) {
  if (p.nslices <= 0 || p.nmsg <= 0) return kOk;
  const size_t grid = (size_t)p.nslices * (size_t)p.nmsg;
  if (grid > 0x7fffffffu) return kErrArg;
  if (key_bytes == 8)
    hipLaunchKernelGGL(slice_sig_kernel<uint64_t>, dim3((unsigned)grid), dim3(kBlock), 0, st, p);
  else if (key_bytes == 4)
    hipLaunchKernelGGL(slice_sig_kernel<uint32_t>, dim3((unsigned)grid), dim3(kBlock), 0, st, p);
  else
    return kErrArg;
  return launch_status();
}

int crc32c_batch_launch(const void* const* d, const uint32_t* n, const int* slot, const uint32_t* ticket,
                        int count, PubSlot* pub, hipStream_t st, Profiler* prof) {
  if (count <= 0) return kOk;
  if (count > kCrcBatchMax) return kErrArg;
  CrcBatch B{};
  double bytes = 0;
  for (int i = 0; i < count; ++i) {
    if (n[i] == 0 || n[i] > kCrcSingleBlock) return kErrArg;
    B.d[i] = static_cast<const uint8_t*>(d[i]);
    B.n[i] = n[i];
    B.slot[i] = slot[i];
    B.ticket[i] = ticket[i];
    bytes += n[i];
  }
  ProfScope ps(prof, kKCrc, st, bytes);
  hipLaunchKernelGGL(crc32c_small_batch, dim3(count), dim3(kBlock), 0, st, B, pub);
  return launch_status();
}

static X2nTable make_x2n_table() {
  X2nTable t;
  uint32_t p = 1u << 30;  // x^1
  t.v[0] = p;
  for (int k = 1; k < 32; ++k) t.v[k] = p = multmodp(p, p);
  return t;
}

int crc32c_launch(const void* d, size_t n, uint32_t* out, hipStream_t st, Profiler* prof,
                  PubSlot* pub, uint32_t ticket) {
  static const X2nTable tbl = make_x2n_table();
  if (n == 0) return kErrArg;  // crc32c("") == 0: callers answer that on the host
  if (n <= kCrcSingleBlock) {
    ProfScope ps(prof, kKCrc, st, (double)n);
    hipLaunchKernelGGL(crc32c_small, dim3(1), dim3(kBlock), 0, st, static_cast<const uint8_t*>(d),
                       (uint32_t)n, out, pub, ticket);
    return launch_status();
  }
  if (hipMemsetAsync(out, 0, sizeof(uint32_t), st) != hipSuccess) return kErrHip;
  // >= 8 bytes per lane, chunks a multiple of 4 bytes, at most kMaxGrid blocks
  size_t lanes = (n + 7) / 8;
  size_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks > (size_t)kMaxGrid) blocks = kMaxGrid;
  size_t total = blocks * kBlock;
  size_t chunk = (n + total - 1) / total;
  chunk = (chunk + 3) & ~(size_t)3;
  blocks = ((n + chunk - 1) / chunk + kBlock - 1) / kBlock;
  ProfScope ps(prof, kKCrc, st, (double)n);
  hipLaunchKernelGGL(crc32c_chunks, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                     static_cast<const uint8_t*>(d), n, chunk, out, tbl, nullptr, 0u);
  return launch_status();
}

}  // namespace psf
