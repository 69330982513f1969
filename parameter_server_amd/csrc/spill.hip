// Device side of the cross-range spill: one launch gathers
// every frame a rank sends in a step -- the Task/record blob staged from the
// host and the encoded key / value frames already in HBM -- into the
// contiguous per-peer send buffer the all-to-all-v moves.  This replaces the
// reference's loop of per-server zero-copy sends (executor.cc:135-146,
// van.cc:122-191), where the frames stay separate ZeroMQ parts.
//
// Work split: every copy is cut into kSpillChunk-byte chunks, one workgroup
// per chunk (a 4 KiB wave-row per iteration, 16 B per lane when the source is
// 16-byte aligned); a workgroup finds its copy by binary search over the
// copies' first-chunk indices.  Destinations are 256-byte aligned.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psf_internal.h"

namespace psf {

template <typename W>
__device__ __forceinline__ void copy_words(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           uint64_t len) {
  const uint64_t nw = len / sizeof(W);
  const W* s = reinterpret_cast<const W*>(src);
  W* d = reinterpret_cast<W*>(dst);
  for (uint64_t i = threadIdx.x; i < nw; i += blockDim.x) d[i] = s[i];
  for (uint64_t i = nw * sizeof(W) + threadIdx.x; i < len; i += blockDim.x) dst[i] = src[i];
}

__global__ void __launch_bounds__(kBlock) spill_gather_kernel(const SpillCopy* __restrict__ copies, int n,
                                                              uint8_t* __restrict__ dst) {
  const uint64_t b = blockIdx.x;
  int lo = 0, hi = n - 1;  // last copy whose first chunk <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (copies[mid].chunk0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const SpillCopy c = copies[lo];
  const uint64_t off = (b - c.chunk0) * kSpillChunk;
  if (off >= c.len) return;
  const uint64_t len = c.len - off < kSpillChunk ? c.len - off : kSpillChunk;
  const uint8_t* s = c.src + off;
  uint8_t* d = dst + c.dst_off + off;
  const uintptr_t a = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d);
  if ((a & 15) == 0) copy_words<uint4>(s, d, len);
  else if ((a & 7) == 0) copy_words<uint2>(s, d, len);
  else if ((a & 3) == 0) copy_words<uint32_t>(s, d, len);
  else copy_words<uint8_t>(s, d, len);
}

int spill_gather_launch(const SpillCopy* d_copies, int n, uint64_t nchunks, void* dst, hipStream_t st) {
  if (n <= 0 || nchunks == 0) return kOk;
  if (nchunks > 0x7fffffffull) return kErrArg;
  hipLaunchKernelGGL(spill_gather_kernel, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_copies, n,
                     static_cast<uint8_t*>(dst));
  return launch_status();
}

}  // namespace psf
