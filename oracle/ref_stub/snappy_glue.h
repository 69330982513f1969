// ORACLE TEST INFRASTRUCTURE -- the SArray <-> snappy glue of the reference
// (src/util/shared_array_inl.h:232-255) restated for the stub SArray, shared by
// ref_harness.cc and adapter_harness.cc.  Links snappy 1.1.8 (/opt/conda).
#pragma once
#include "/opt/conda/include/snappy.h"

// snappy glue restated from shared_array_inl.h:232-255
namespace PS {
template <typename V> SArray<char> SArray<V>::CompressTo() const {
  if (empty()) return SArray<char>();
  size_t ssize = size_ * sizeof(V);
  size_t dsize = snappy::MaxCompressedLength(ssize);
  SArray<char> dest(dsize);
  snappy::RawCompress(reinterpret_cast<const char*>(data()), ssize, dest.data(), &dsize);
  dest.resize(dsize);
  return dest;
}
template <typename V> void SArray<V>::UncompressFrom(const char* src, size_t src_size) {
  if (src_size == 0) { clear(); return; }
  size_t dsize = 0;
  CHECK(snappy::GetUncompressedLength(src, src_size, &dsize));
  CHECK_EQ(dsize / sizeof(V) * sizeof(V), dsize);
  resize(dsize / sizeof(V));
  CHECK(snappy::RawUncompress(src, src_size, reinterpret_cast<char*>(data())));
}
template class SArray<char>;
}  // namespace PS

