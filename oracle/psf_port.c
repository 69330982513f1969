/*
 * ORACLE TEST INFRASTRUCTURE -- a plain-C restatement of the reference codec
 * arithmetic, used ONLY by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker / CPU baseline.  Never linked into libpsf.
 *
 * PARITY UNPINNED for FIXING_FLOAT (and the KEY_CACHING / COMPRESSING glue
 * restated in oracle/chain.py): the reference holds no vectors for them
 * (src/test/fixing_float_test.cc asserts nothing) and its filter headers need
 * glog / Eigen / the protobuf runtime, absent here, so it cannot be built.
 * tests/golden/ff_cases.* and scenarios.json are this restatement's own
 * record (tests/golden/make_golden.py).  Pinned to the reference itself:
 * CRC32C only (oracle/_ref/libcrc32c_ref.so, compiled from its crc32c.cc);
 * snappy to the 1.1.8 library, NOISE to libstdc++.
 *
 * Every function cites the reference lines it restates.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define PORT_OK 0
#define PORT_ERR_ARG -1     /* bad argument (dtype, null) */
#define PORT_ERR_NBYTES -2  /* CHECK_GT(nbytes,0) / CHECK_LT(nbytes,8), fixing_float.h:53-54 */
#define PORT_ERR_BIN -3     /* CHECK_GT(bin,0), fixing_float.h:71 */

#define DT_FLOAT 9   /* task.proto DataType::FLOAT */
#define DT_DOUBLE 10 /* task.proto DataType::DOUBLE */

/* boolrand, fixing_float.h:18-21: MSVC LCG on a 32-bit int (wraps mod 2^32). */
static inline int lcg_bit(uint32_t* s) {
  *s = 214013u * *s + 2531011u;
  return ((*s >> 16) & 1u) == 0;
}

/* s_k after k LCG steps from seed (s_0 = seed).  Test helper for jump-ahead. */
uint32_t port_lcg_state(int32_t seed, uint64_t k) {
  uint32_t a = 214013u, c = 2531011u, s = (uint32_t)seed;
  /* affine map composition by squaring: (a,c) applied k times */
  uint32_t A = 1u, C = 0u;
  while (k) {
    if (k & 1u) { A = a * A; C = a * C + c; }
    c = a * c + c; a = a * a; k >>= 1;
  }
  return A * s + C;
}

/* ratio, fixing_float.h:55: `static_cast<double>(1 << (nbytes*8)) - 2` on a
 * 32-bit int; x86 masks the shift count to 5 bits, so nb=4 gives -1 and
 * nb=5..7 behave as nb-4. */
double port_ff_ratio(int nb) {
  int32_t one_shifted = (int32_t)(1u << ((unsigned)(nb * 8) & 31u));
  return (double)one_shifted - 2.0;
}

/* static_cast<uint64>(floor(tmp)) as g++/x86-64 lowers it (cvttsd2si below
 * 2^63): negative values wrap through int64; NaN yields a value whose low 56
 * bits are zero (only those are ever emitted, nb < 8). */
static inline uint64_t x86_d2u64(double d) {
  if (d != d) return 0;
  if (d < 9223372036854775808.0) return (uint64_t)(int64_t)d;
  return (uint64_t)(int64_t)(d - 9223372036854775808.0) ^ 0x8000000000000000ull;
}

/* min/max exactly as fixing_float.h:57-64: min = (float)minCoeff,
 * max = (float)((double)maxCoeff + 1e-6).  Two points the reference leaves to
 * Eigen's (vectorised, order-dependent) reduction are fixed here and in the
 * HIP kernels alike (DESIGN.md "divergences"): NaNs are skipped, and -0.0
 * orders below +0.0 (only the sign bit of a zero min can differ; codes and
 * decoded values cannot). */
static void minmax_f32(const float* x, size_t n, float* mn, float* mx) {
  float lo = INFINITY, hi = -INFINITY;
  int any = 0;
  for (size_t i = 0; i < n; ++i) {
    float v = x[i];
    if (v != v) continue;
    any = 1;
    if (v < lo || (v == lo && signbit(v))) lo = v;
    if (v > hi) hi = v;
  }
  if (!any) { lo = NAN; hi = NAN; }
  *mn = lo;
  *mx = (float)((double)hi + 1e-6);
}
static void minmax_f64(const double* x, size_t n, float* mn, float* mx) {
  double lo = INFINITY, hi = -INFINITY;
  int any = 0;
  for (size_t i = 0; i < n; ++i) {
    double v = x[i];
    if (v != v) continue;
    any = 1;
    if (v < lo || (v == lo && signbit(v))) lo = v;
    if (v > hi) hi = v;
  }
  if (!any) { lo = NAN; hi = NAN; }
  *mn = (float)lo;
  *mx = (float)(hi + 1e-6);
}

/* FixingFloatFilter::convert<V> encode branch, fixing_float.h:50-88.
 * in: n elements of dtype; out: n*nb bytes.  (*mn,*mx) in/out: when has_* is
 * set they are the preset fixed_point range, otherwise they receive the
 * computed one (the side-info the filter stores in the FilterConfig). */
int port_ff_encode(const void* in, size_t n, int dtype, int nb, int has_min,
                   float* mn, int has_max, float* mx, int32_t seed,
                   uint8_t* out) {
  if (nb <= 0 || nb >= 8) return PORT_ERR_NBYTES;
  if (dtype != DT_FLOAT && dtype != DT_DOUBLE) return PORT_ERR_ARG;
  double ratio = port_ff_ratio(nb);
  if (!has_min || !has_max) {
    float cmn, cmx;
    if (dtype == DT_FLOAT) minmax_f32((const float*)in, n, &cmn, &cmx);
    else minmax_f64((const double*)in, n, &cmn, &cmx);
    if (!has_min) *mn = cmn;
    if (!has_max) *mx = cmx;
  }
  double min_v = (double)*mn, max_v = (double)*mx;
  double bin = max_v - min_v;
  if (!(bin > 0)) return PORT_ERR_BIN;
  uint32_t s = (uint32_t)seed;
  for (size_t i = 0; i < n; ++i) {
    double x = dtype == DT_FLOAT ? (double)((const float*)in)[i] : ((const double*)in)[i];
    double proj = x > max_v ? max_v : x < min_v ? min_v : x;
    double tmp = (proj - min_v) / bin * ratio;
    uint64_t r = x86_d2u64(floor(tmp)) + (uint64_t)lcg_bit(&s);
    for (int j = 0; j < nb; ++j) { *out++ = (uint8_t)(r & 0xFF); r >>= 8; }
  }
  return PORT_OK;
}

/* decode branch, fixing_float.h:89-101: r = sum byte_j << 8j (accumulated in
 * double), out = (V)(r / ratio * bin + min_v), no FMA. */
int port_ff_decode(const uint8_t* code, size_t code_bytes, int dtype, int nb,
                   float mn, float mx, void* out) {
  if (nb <= 0 || nb >= 8) return PORT_ERR_NBYTES;
  if (dtype != DT_FLOAT && dtype != DT_DOUBLE) return PORT_ERR_ARG;
  double ratio = port_ff_ratio(nb);
  double min_v = (double)mn, max_v = (double)mx;
  double bin = max_v - min_v;
  if (!(bin > 0)) return PORT_ERR_BIN;
  size_t n = code_bytes / (size_t)nb;
  for (size_t i = 0; i < n; ++i) {
    double r = 0;
    for (int j = 0; j < nb; ++j) r += (double)((uint64_t)(*code++) << (8 * j));
    double v = r / ratio * bin + min_v;
    if (dtype == DT_FLOAT) ((float*)out)[i] = (float)v;
    else ((double*)out)[i] = v;
  }
  return PORT_OK;
}

/* Checker for the device decode's quotient (ff_codec.hip dequant_q): counts
 * the codes r in [0, 2^(8nb)) where the fma-corrected reciprocal product
 * q0 = r * RN(1/ratio); q = fma(fma(-q0, ratio, r), RN(1/ratio), q0)
 * differs from the IEEE quotient r / ratio the reference computes
 * (fixing_float.h:97).  Not a restatement of the reference. */
long port_decode_quotient_mismatches(int nb) {
  if (nb <= 0 || nb > 3) return -1;
  const double ratio = port_ff_ratio(nb), inv = 1.0 / ratio;
  long bad = 0;
  for (uint32_t r = 0; r < (1u << (8 * nb)); ++r) {
    const double a = (double)r, q0 = a * inv;
    const double q = fma(fma(-q0, ratio, a), inv, q0);
    bad += q != a / ratio;
  }
  return bad;
}

/* CRC-32C (Castagnoli, reflected polynomial 0x82F63B78, init/final ~0) --
 * the function util/crc32c.cc:292-335 computes (slicing-by-4 there, a plain
 * byte table here; the value is alignment- and slicing-independent). */
static uint32_t crc_table[256];
static int crc_ready = 0;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    crc_table[i] = c;
  }
  crc_ready = 1;
}
uint32_t port_crc32c_extend(uint32_t crc, const void* p, size_t n) {
  if (!crc_ready) crc_init();
  const uint8_t* b = (const uint8_t*)p;
  uint32_t l = crc ^ 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) l = crc_table[(l ^ b[i]) & 0xFF] ^ (l >> 8);
  return l ^ 0xFFFFFFFFu;
}
uint32_t port_crc32c(const void* p, size_t n) { return port_crc32c_extend(0, p, n); }

/* KeyCachingFilter signature, key_caching.h:18,74: CRC32C of the first
 * min(bytes, 2048) key bytes. */
uint32_t port_key_signature(const void* key, size_t bytes) {
  return port_crc32c(key, bytes < 2048 ? bytes : 2048);
}

/* AddNoiseFilter, add_noise.h:29-39: std::default_random_engine (libstdc++
 * minstd_rand0, seed 1) feeding std::normal_distribution<float> (libstdc++
 * Marsaglia polar method through generate_canonical<float,24>), a fresh engine
 * per array, added in place. */
static uint32_t minstd_next(uint32_t* x) {
  *x = (uint32_t)(((uint64_t)*x * 16807u) % 2147483647u);
  return *x;
}
static float canon_f32(uint32_t* x) {
  float sum = (float)(minstd_next(x) - 1u);
  float tmp = 2147483648.0f;  /* float(2147483646.0L) */
  float ret = sum / tmp;
  if (ret >= 1.0f) ret = nextafterf(1.0f, 0.0f);
  return ret;
}
static double canon_f64(uint32_t* x) {
  /* generate_canonical<double,53>: m = ceil(53/30) = 2 draws */
  double r = 2147483646.0;
  double sum = (double)(minstd_next(x) - 1u);
  double tmp = r;
  sum += (double)(minstd_next(x) - 1u) * tmp;
  tmp *= r;
  double ret = sum / tmp;
  if (ret >= 1.0) ret = nextafter(1.0, 0.0);
  return ret;
}
int port_add_noise(void* data, size_t n, int dtype, float mean, float sd) {
  uint32_t x = 1u;
  int saved_ok = 0;
  if (dtype == DT_FLOAT) {
    float* v = (float*)data;
    float saved = 0.f;
    for (size_t i = 0; i < n; ++i) {
      float ret;
      if (saved_ok) { saved_ok = 0; ret = saved; }
      else {
        float a, b, r2;
        do {
          a = (float)((double)(2.0f * canon_f32(&x)) - 1.0);
          b = (float)((double)(2.0f * canon_f32(&x)) - 1.0);
          r2 = a * a + b * b;
        } while (r2 > 1.0f || r2 == 0.0f);
        float mult = sqrtf(-2.0f * logf(r2) / r2);
        saved = a * mult; saved_ok = 1;
        ret = b * mult;
      }
      v[i] += ret * sd + mean;
    }
    return PORT_OK;
  }
  if (dtype == DT_DOUBLE) {
    double* v = (double*)data;
    double saved = 0.0;
    for (size_t i = 0; i < n; ++i) {
      double ret;
      if (saved_ok) { saved_ok = 0; ret = saved; }
      else {
        double a, b, r2;
        do {
          a = 2.0 * canon_f64(&x) - 1.0;
          b = 2.0 * canon_f64(&x) - 1.0;
          r2 = a * a + b * b;
        } while (r2 > 1.0 || r2 == 0.0);
        double mult = sqrt(-2.0 * log(r2) / r2);
        saved = a * mult; saved_ok = 1;
        ret = b * mult;
      }
      v[i] += ret * (double)sd + (double)mean;
    }
    return PORT_OK;
  }
  return PORT_ERR_ARG;
}

/* ---- server-side consumers -------------------------- */

/* AssignOp, src/util/assign_op.h:10-26 (ASSIGN..DIVIDE) */
#define ASSIGN_OP(T, right, left, op)          \
  do {                                         \
    switch (op) {                              \
      case 0: (right) = (left); break;         \
      case 1: (right) += (left); break;        \
      case 2: (right) -= (left); break;        \
      case 3: (right) *= (left); break;        \
      case 4: (right) /= (left); break;        \
    }                                          \
  } while (0)

/* ParallelOrderedMatch, src/util/parallel_ordered_match.h:7-34 and 57-83, run
 * on one thread (the grainsize split only partitions dst): skip the src
 * prefix below dst[0] (lower_bound), then walk both sorted arrays with two
 * cursors, applying op on equal keys and advancing both.  Returns *n (matched
 * keys * k). */
size_t port_ordered_match(const uint64_t* sk, size_t ns, const void* sv, const uint64_t* dk, size_t nd,
                          void* dv, int k, int dtype, int op) {
  if (nd == 0 || ns == 0) return 0;
  size_t lo = 0, hi = ns;
  while (lo < hi) {
    size_t mid = lo + ((hi - lo) >> 1);
    if (sk[mid] < dk[0]) lo = mid + 1; else hi = mid;
  }
  size_t s = lo, d = 0, n = 0;
  while (d < nd && s < ns) {
    if (sk[s] < dk[d]) {
      ++s;
    } else {
      if (!(dk[d] < sk[s])) {
        for (int i = 0; i < k; ++i) {
          if (dtype == DT_FLOAT) ASSIGN_OP(float, ((float*)dv)[d * k + i], ((const float*)sv)[s * k + i], op);
          else ASSIGN_OP(double, ((double*)dv)[d * k + i], ((const double*)sv)[s * k + i], op);
        }
        ++s;
        n += (size_t)k;
      }
      ++d;
    }
  }
  return n;
}

/* FTRLEntry::Set, src/app/linear_method/async_sgd.h:137-151, with
 * LearningRate<float>::eval (learning_rate.h:15-22), ElasticNet<float>::proximal
 * (penalty.h:51-56) and SGDState::UpdateWeight (async_sgd.h:106-116), applied
 * serially to entries idx[0..n) of the state arrays (the caller maps keys to
 * entries, as the reference's unordered_map does).  float arithmetic, one
 * operation at a time.  Returns -1 where the reference's CHECK_GT(eta, 0)
 * fails, else 0. */
int port_ftrl_update(const int64_t* idx, size_t n, const float* grad, float* w, float* z, float* sqrt_n,
                     int lr_decay, float alpha, float beta, float lambda1, float lambda2, int64_t* nnz,
                     float* weight_sum, float* delta_sum) {
  for (size_t i = 0; i < n; ++i) {
    const int64_t e = idx[i];
    const float w_old = w[e];
    const float g = grad[i];
    const float sqrt_n_new = (float)sqrt((double)(sqrt_n[e] * sqrt_n[e] + g * g));
    const float sigma = (sqrt_n_new - sqrt_n[e]) / alpha;
    z[e] += g - sigma * w[e];
    sqrt_n[e] = sqrt_n_new;
    const float eta = lr_decay ? alpha / (sqrt_n[e] + beta) : alpha;
    const float zz = -z[e] * eta;
    if (!(eta > 0)) return -1;
    const float leta = lambda1 * eta;
    float nw;
    if (zz <= leta && zz >= -leta) nw = 0;
    else nw = zz > 0 ? (zz - leta) / (1 + lambda2 * eta) : (zz + leta) / (1 + lambda2 * eta);
    w[e] = nw;
    if (nw == 0 && w_old != 0) --*nnz;
    else if (nw != 0 && w_old == 0) ++*nnz;
    *weight_sum += nw * nw;
    const float delta = nw - w_old;
    *delta_sum += delta * delta;
  }
  return 0;
}
