// NOISE filter (reference src/filter/add_noise.h:11-39) for gfx950.
//
// The reference adds std::normal_distribution<V>(mean, std) samples in place,
// drawing from a FRESH std::default_random_engine (libstdc++ minstd_rand0,
// seed 1) per value array -- so every message receives the same standard-normal
// sequence z_0, z_1, ... (only `* std + mean` differs).  libpsf therefore:
//
//  1. builds z once per context and dtype, on the device, with a parallel
//     Marsaglia polar method reproducing libstdc++'s draw order exactly:
//       attempt j consumes uniform draws 2j, 2j+1 (f32: generate_canonical<
//       float,24> = 1 engine draw per uniform; f64: 2 draws per uniform);
//       accepted attempts (0 < r2 <= 1) yield y*mult then x*mult.
//     noise_count   -- each lane jumps the engine (16807^k mod 2^31-1) to its
//                      first attempt and counts acceptances per workgroup
//     noise_scan    -- exclusive scan of the workgroup counts (one workgroup)
//     noise_emit    -- lanes re-walk their attempts and write their normals at
//                      2 * (global rank of the accepted attempt)
//  2. per message runs noise_apply: v[i] += z[i] * std + mean (no FMA), in place.
//
// Exactness: the engine, the uniforms, x, y, r2 and the acceptance test are
// exact IEEE operations, identical to libstdc++'s.  mult = sqrt(-2 log(r2)/r2)
// uses correctly rounded sqrt/division and glibc's own log algorithms --
// logf for f32 (glibc_logf.h), log for f64 (glibc_log.h, including the fused
// multiply-adds of the FMA build the reference's host runs) -> NOISE is
// bit-exact for both types.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_log.h"
#include "glibc_logf.h"
#include "psf_internal.h"

namespace psf {

constexpr uint32_t kMinstdP = 2147483647u;  // 2^31 - 1
constexpr uint32_t kMinstdA = 16807u;
constexpr int kAttemptsPerLane = 16;

__host__ __device__ inline uint32_t mulmod_p(uint32_t a, uint32_t b) {
  uint64_t x = (uint64_t)a * b;
  uint64_t r = (x & kMinstdP) + (x >> 31);
  r = (r & kMinstdP) + (r >> 31);
  return r >= kMinstdP ? (uint32_t)(r - kMinstdP) : (uint32_t)r;
}
__host__ __device__ inline uint32_t powmod_p(uint32_t a, uint64_t k) {
  uint32_t r = 1;
  while (k) {
    if (k & 1) r = mulmod_p(r, a);
    a = mulmod_p(a, a);
    k >>= 1;
  }
  return r;
}

// one engine draw: x <- 16807 x mod p (seed 1: the state after k draws is 16807^k)
__device__ __forceinline__ uint32_t draw(uint32_t& x) {
  x = mulmod_p(x, kMinstdA);
  return x;
}

// Correctly rounded sqrtf.  gfx950's v_sqrt_f32 (behind __fsqrt_rn and sqrtf)
// is off by one ulp on ~15 % of inputs, while the reference's sqrtss is exact.
// Take the double-precision root rounded to float, then settle between it and
// its neighbours with the midpoints: a midpoint of two adjacent floats has 25
// significant bits, so its square is exact in double, and no float input can
// equal it (no ties).
__device__ __forceinline__ float sqrt_rn(float q) {
  if (!(q > 0.0f) || q == __builtin_huge_valf()) return __fsqrt_rn(q);  // 0, inf, NaN, <0
  float s = (float)__dsqrt_rn((double)q);
  const double dq = (double)q;
  const float lo = __uint_as_float(__float_as_uint(s) - 1u);
  const double mlo = ((double)lo + (double)s) * 0.5;
  if (dq < mlo * mlo) return lo;
  const float hi = __uint_as_float(__float_as_uint(s) + 1u);
  const double mhi = ((double)s + (double)hi) * 0.5;
  if (dq > mhi * mhi) return hi;
  return s;
}

template <typename V> struct Polar;
template <> struct Polar<float> {
  static constexpr int kDrawsPerAttempt = 2;
  // generate_canonical<float, 24> over minstd_rand0: (x - 1) / float(2^31 - 2)
  __device__ static float uniform(uint32_t& x) {
    float ret = (float)(draw(x) - 1u) / 2147483648.0f;
    return ret >= 1.0f ? __uint_as_float(0x3F7FFFFFu) : ret;
  }
  // one attempt; returns accepted, and the two normals in the reference's order
  __device__ static bool attempt(uint32_t& x, float& z0, float& z1) {
    const float a = (float)((double)(2.0f * uniform(x)) - 1.0);
    const float b = (float)((double)(2.0f * uniform(x)) - 1.0);
    const float r2 = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (r2 > 1.0f || r2 == 0.0f) return false;
    const float lg = glibc_logf(r2);  // the reference's libm logf, bit for bit
    const float mult = sqrt_rn(__fdiv_rn(__fmul_rn(-2.0f, lg), r2));
    z0 = __fmul_rn(b, mult);
    z1 = __fmul_rn(a, mult);
    return true;
  }
};
template <> struct Polar<double> {
  static constexpr int kDrawsPerAttempt = 4;
  // generate_canonical<double, 53>: two draws, sum/tmp with tmp = r*r
  __device__ static double uniform(uint32_t& x) {
    const double r = 2147483646.0;
    double sum = (double)(draw(x) - 1u);
    sum = __dadd_rn(sum, __dmul_rn((double)(draw(x) - 1u), r));
    double ret = sum / __dmul_rn(r, r);
    return ret >= 1.0 ? __longlong_as_double(0x3FEFFFFFFFFFFFFFll) : ret;
  }
  __device__ static bool attempt(uint32_t& x, double& z0, double& z1) {
    const double a = __dadd_rn(__dmul_rn(2.0, uniform(x)), -1.0);
    const double b = __dadd_rn(__dmul_rn(2.0, uniform(x)), -1.0);
    const double r2 = __dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b));
    if (r2 > 1.0 || r2 == 0.0) return false;
    const double lg = glibc_log(r2);  // the reference's libm log, bit for bit
    const double mult = __dsqrt_rn(__ddiv_rn(__dmul_rn(-2.0, lg), r2));
    z0 = __dmul_rn(b, mult);
    z1 = __dmul_rn(a, mult);
    return true;
  }
};

template <typename V>
__device__ __forceinline__ uint32_t lane_state(uint64_t first_attempt) {
  return powmod_p(kMinstdA, first_attempt * Polar<V>::kDrawsPerAttempt);
}

template <typename V>
__global__ __launch_bounds__(kBlock) void noise_count(uint64_t attempts, uint32_t* block_counts) {
  __shared__ uint32_t s_cnt[kBlock / 64];
  const uint64_t lane = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t a0 = lane * kAttemptsPerLane;
  uint32_t cnt = 0;
  if (a0 < attempts) {
    uint32_t x = lane_state<V>(a0);
    const int na = (int)(attempts - a0 < (uint64_t)kAttemptsPerLane ? attempts - a0 : kAttemptsPerLane);
    for (int k = 0; k < na; ++k) {
      V z0, z1;
      cnt += Polar<V>::attempt(x, z0, z1) ? 1u : 0u;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += s_cnt[w];
    block_counts[blockIdx.x] = t;
  }
}

// exclusive scan of nb counts into offsets[0..nb), total in offsets[nb]; one workgroup
__global__ __launch_bounds__(kBlock) void noise_scan(const uint32_t* counts, int nb, uint64_t* offsets) {
  __shared__ uint64_t s[kBlock];
  uint64_t carry = 0;
  for (int base = 0; base < nb; base += kBlock) {
    const int i = base + threadIdx.x;
    uint64_t v = i < nb ? counts[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {  // Hillis-Steele inclusive scan
      uint64_t t = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) offsets[i] = carry + s[threadIdx.x] - v;
    const uint64_t tot = s[kBlock - 1];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) offsets[nb] = carry;
}

template <typename V>
__global__ __launch_bounds__(kBlock) void noise_emit(uint64_t attempts, const uint64_t* offsets,
                                                      V* z, uint64_t nz) {
  __shared__ uint32_t s_cnt[kBlock];
  const uint64_t lane = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t a0 = lane * kAttemptsPerLane;
  const int na = a0 >= attempts ? 0
               : (int)(attempts - a0 < (uint64_t)kAttemptsPerLane ? attempts - a0 : kAttemptsPerLane);
  // pass 1: this lane's acceptance count, then the in-workgroup exclusive prefix
  uint32_t x0 = na ? lane_state<V>(a0) : 1u;
  uint32_t x = x0, cnt = 0;
  for (int k = 0; k < na; ++k) {
    V z0, z1;
    cnt += Polar<V>::attempt(x, z0, z1) ? 1u : 0u;
  }
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = 1; o < kBlock; o <<= 1) {
    uint32_t t = threadIdx.x >= (unsigned)o ? s_cnt[threadIdx.x - o] : 0;
    __syncthreads();
    s_cnt[threadIdx.x] += t;
    __syncthreads();
  }
  uint64_t rank = offsets[blockIdx.x] + s_cnt[threadIdx.x] - cnt;
  // pass 2: emit
  x = x0;
  for (int k = 0; k < na; ++k) {
    V z0, z1;
    if (Polar<V>::attempt(x, z0, z1)) {
      const uint64_t p = 2 * rank;
      if (p < nz) z[p] = z0;
      if (p + 1 < nz) z[p + 1] = z1;
      ++rank;
    }
  }
}

// v[i] += z[i] * sd + mean  (add_noise.h:36, `ret * stddev + mean` then +=; no FMA)
template <typename V>
__global__ __launch_bounds__(kBlock) void noise_apply(V* __restrict__ v, const V* __restrict__ z,
                                                       size_t n, V mean, V sd) {
  const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t T = (size_t)gridDim.x * kBlock;
  for (size_t i = t; i < n; i += T) {
    const V nz = z[i] * sd + mean;
    v[i] = v[i] + nz;
  }
}

// ---------------------------------------------------------------- host ----
template <typename V>
static int build_table(V* z, uint64_t nz, void* scratch, size_t scratch_bytes, hipStream_t st,
                       uint64_t* total_out_host) {
  // attempts for nz normals: ceil(nz/2) acceptances at p = pi/4, +6 sigma + slack
  const double need = (double)((nz + 1) / 2);
  uint64_t attempts = (uint64_t)(need / 0.7853981633974483 + 6.0 * sqrt(need) + 4096.0);
  const uint64_t lanes = (attempts + kAttemptsPerLane - 1) / kAttemptsPerLane;
  const uint64_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks * sizeof(uint32_t) + (blocks + 1) * sizeof(uint64_t) > scratch_bytes) return kErrArg;
  uint32_t* counts = static_cast<uint32_t*>(scratch);
  uint64_t* offsets = reinterpret_cast<uint64_t*>(static_cast<char*>(scratch) +
                                                  ((blocks * sizeof(uint32_t) + 15) & ~(size_t)15));
  hipLaunchKernelGGL((noise_count<V>), dim3((unsigned)blocks), dim3(kBlock), 0, st, attempts, counts);
  hipLaunchKernelGGL(noise_scan, dim3(1), dim3(kBlock), 0, st, counts, (int)blocks, offsets);
  hipLaunchKernelGGL((noise_emit<V>), dim3((unsigned)blocks), dim3(kBlock), 0, st, attempts, offsets, z, nz);
  if (launch_status() != kOk) return kErrHip;
  if (hipMemcpyAsync(total_out_host, offsets + blocks, sizeof(uint64_t), hipMemcpyDeviceToHost, st) != hipSuccess)
    return kErrHip;
  if (hipStreamSynchronize(st) != hipSuccess) return kErrHip;
  return kOk;
}

size_t noise_scratch_bytes(uint64_t nz) {
  const double need = (double)((nz + 1) / 2);
  uint64_t attempts = (uint64_t)(need / 0.7853981633974483 + 6.0 * sqrt(need) + 4096.0);
  const uint64_t blocks = ((attempts + kAttemptsPerLane - 1) / kAttemptsPerLane + kBlock - 1) / kBlock;
  return ((blocks * sizeof(uint32_t) + 15) & ~(size_t)15) + (blocks + 1) * sizeof(uint64_t) + 64;
}

int noise_build_table(int value_type, void* z, uint64_t nz, void* scratch, size_t scratch_bytes,
                      hipStream_t st, Profiler* prof) {
  uint64_t total = 0;
  ProfScope ps(prof, kKNoise, st, 0.0);
  int s = value_type == kFloat
              ? build_table<float>(static_cast<float*>(z), nz, scratch, scratch_bytes, st, &total)
          : value_type == kDouble
              ? build_table<double>(static_cast<double*>(z), nz, scratch, scratch_bytes, st, &total)
              : kErrArg;
  if (s != kOk) return s;
  return 2 * total >= nz ? kOk : kErrCheck;  // not enough accepted attempts (never at 6 sigma)
}

int noise_apply_launch(void* v, const void* z, size_t n, int value_type, float mean, float sd,
                       hipStream_t st, Profiler* prof) {
  if (n == 0) return kOk;
  size_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > (size_t)kMaxGrid) blocks = kMaxGrid;
  if (value_type == kFloat) {
    ProfScope ps(prof, kKNoise, st, 12.0 * n);
    hipLaunchKernelGGL((noise_apply<float>), dim3((unsigned)blocks), dim3(kBlock), 0, st,
                       static_cast<float*>(v), static_cast<const float*>(z), n, mean, sd);
  } else if (value_type == kDouble) {
    ProfScope ps(prof, kKNoise, st, 24.0 * n);
    hipLaunchKernelGGL((noise_apply<double>), dim3((unsigned)blocks), dim3(kBlock), 0, st,
                       static_cast<double*>(v), static_cast<const double*>(z), n, (double)mean,
                       (double)sd);
  } else {
    return kErrArg;
  }
  return launch_status();
}

}  // namespace psf
