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
      if (pub) {
        pub->crc = acc;
        publish_ticket(pub, ticket);
      }
    } else {
      atomicXor(out, acc);
    }
  }
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
    size_t chunk = ((n + kBlock - 1) / kBlock + 3) & ~(size_t)3;
    ProfScope ps(prof, kKCrc, st, (double)n);
    hipLaunchKernelGGL(crc32c_chunks, dim3(1), dim3(kBlock), 0, st, static_cast<const uint8_t*>(d),
                       n, chunk, out, tbl, pub, ticket);
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
