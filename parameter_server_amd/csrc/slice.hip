// Device side of SliceKOFVMessage (reference src/system/message.h:107-147):
// the split positions pos[i] = lower_bound(keys, bound[i]) of a sorted key
// array at the <= (servers + 1) range boundaries.  One lane per boundary does a
// branch-free binary search over the HBM-resident keys (log2(n) dependent loads).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psf_internal.h"

namespace psf {

template <typename K>
__global__ void lower_bound_kernel(const K* __restrict__ keys, size_t n, const uint64_t* bounds,
                                   int nb, uint64_t* pos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const K v = (K)bounds[i];
  size_t lo = 0, len = n;
  while (len > 0) {  // first index with keys[idx] >= v
    const size_t half = len >> 1;
    const size_t mid = lo + half;
    if (keys[mid] < v) {
      lo = mid + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  pos[i] = lo;
}

int lower_bound_launch(const void* keys, size_t n, int key_bytes, const uint64_t* d_bounds, int nb,
                       uint64_t* d_pos, hipStream_t st) {
  if (nb <= 0) return kOk;
  const int threads = 64;
  const int blocks = (nb + threads - 1) / threads;
  if (key_bytes == 8)
    hipLaunchKernelGGL((lower_bound_kernel<uint64_t>), dim3(blocks), dim3(threads), 0, st,
                       static_cast<const uint64_t*>(keys), n, d_bounds, nb, d_pos);
  else if (key_bytes == 4)
    hipLaunchKernelGGL((lower_bound_kernel<uint32_t>), dim3(blocks), dim3(threads), 0, st,
                       static_cast<const uint32_t*>(keys), n, d_bounds, nb, d_pos);
  else
    return kErrArg;
  return launch_status();
}

// many messages at once: lane i handles bound i % nb of message i / nb;
// desc[m] = {key pointer, key count}
template <typename K>
__global__ void lower_bound_batch_kernel(const uint64_t* __restrict__ desc, const uint64_t* bounds, int nb,
                                         int nmsg, uint64_t* pos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * nmsg) return;
  const int m = i / nb;
  const K* keys = reinterpret_cast<const K*>(desc[2 * m]);
  const size_t n = (size_t)desc[2 * m + 1];
  const K v = (K)bounds[i];
  size_t lo = 0, len = n;
  while (len > 0) {
    const size_t half = len >> 1;
    const size_t mid = lo + half;
    if (keys[mid] < v) {
      lo = mid + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  pos[i] = lo;
}

int lower_bound_batch_launch(const uint64_t* d_desc, int key_bytes, const uint64_t* d_bounds, int nb, int nmsg,
                             uint64_t* d_pos, hipStream_t st) {
  if (nb <= 0 || nmsg <= 0) return kOk;
  const int threads = 64;
  const int blocks = (nb * nmsg + threads - 1) / threads;
  if (key_bytes == 8)
    hipLaunchKernelGGL((lower_bound_batch_kernel<uint64_t>), dim3(blocks), dim3(threads), 0, st, d_desc, d_bounds,
                       nb, nmsg, d_pos);
  else if (key_bytes == 4)
    hipLaunchKernelGGL((lower_bound_batch_kernel<uint32_t>), dim3(blocks), dim3(threads), 0, st, d_desc, d_bounds,
                       nb, nmsg, d_pos);
  else
    return kErrArg;
  return launch_status();
}

}  // namespace psf
