// ORACLE TEST INFRASTRUCTURE -- never part of the shipped product.
//
// AddNoiseFilter::AddNoise (reference src/filter/add_noise.h:29-39) is two
// calls into libstdc++: a default-constructed std::default_random_engine,
// fresh for every value array, feeding std::normal_distribution<V>((V)mean,
// (V)std), one draw added to each element in order.  This shim makes those
// same libstdc++ calls, compiled with the reference's flags (Makefile +
// make/config.mk: g++ -std=c++0x -O3, no -march), so the C restatement
// (psf_port.c) and the NOISE kernel are checked against the library the
// reference itself calls -- its algorithm lives in libstdc++'s headers, the
// way COMPRESSING's lives in snappy 1.1.8.
#include <stddef.h>

#include <random>

template <typename V>
static void add_noise(V* d, size_t n, float mean, float sd) {
  std::default_random_engine generator;
  std::normal_distribution<V> distribution((V)mean, (V)sd);
  for (size_t i = 0; i < n; ++i) d[i] += distribution(generator);
}

// dtype: task.proto DataType, FLOAT = 9, DOUBLE = 10
extern "C" int noise_std(void* data, size_t n, int dtype, float mean, float sd) {
  if (dtype == 9) add_noise(static_cast<float*>(data), n, mean, sd);
  else if (dtype == 10) add_noise(static_cast<double*>(data), n, mean, sd);
  else return -1;
  return 0;
}
