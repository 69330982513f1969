// ORACLE TEST INFRASTRUCTURE -- not product code.
//
// A test double of the PS types that include/psf_ps_filter.h (the
// reference-side drop-in adapter) is written against, so that the adapter can
// be compiled and exercised here (oracle/adapter_harness.cc).  No reference
// source is compiled against this file: it mirrors the reference's interface
// (names and proto field semantics), written from
//   filter.h:9-24            Filter interface
//   filter.proto:3-35        FilterConfig / FixedFloatConfig fields + has-bits
//   task.proto:28-39,78-91   Task fields used by the filters, DataType enum
//   message.h:10-76          Message key/value, has_key/clear_key/set_key
//   range.h:11-131           Range<Key> equality + hash
//
// CHECK failures throw PsCheckError so the ctypes harness can report them
// instead of aborting the test process (the reference aborts via glog).
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <algorithm>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace PS {

typedef int8_t int8;
typedef uint8_t uint8;
typedef int32_t int32;
typedef uint32_t uint32;
typedef int64_t int64;
typedef uint64_t uint64;
typedef uint64 Key;
typedef std::lock_guard<std::mutex> Lock;

// ---------------------------------------------------------------- CHECK ----
struct PsCheckError : std::runtime_error {
  explicit PsCheckError(const std::string& s) : std::runtime_error(s) {}
};
class CheckFail {
 public:
  CheckFail(const char* file, int line, const char* what) {
    ss_ << file << ":" << line << " CHECK failed: " << what << " ";
  }
  ~CheckFail() noexcept(false) { throw PsCheckError(ss_.str()); }
  std::ostream& stream() { return ss_; }
 private:
  std::ostringstream ss_;
};
#define CHECK(c) if (c) ; else ::PS::CheckFail(__FILE__, __LINE__, #c).stream()
#define CHECK_EQ(a, b) CHECK((a) == (b))
#define CHECK_NE(a, b) CHECK((a) != (b))
#define CHECK_GT(a, b) CHECK((a) > (b))
#define CHECK_GE(a, b) CHECK((a) >= (b))
#define CHECK_LT(a, b) CHECK((a) < (b))
#define CHECK_LE(a, b) CHECK((a) <= (b))
template <typename T> T* CheckNotNull(T* p, const char* file, int line) {
  if (!p) ::PS::CheckFail(file, line, "not null");
  return p;
}
#define CHECK_NOTNULL(p) ::PS::CheckNotNull((p), __FILE__, __LINE__)

// ---------------------------------------------------------------- enums ----
enum DataType {
  OTHER = 0, INT8 = 1, INT16 = 2, INT32 = 3, INT64 = 4, UINT8 = 5,
  UINT16 = 6, UINT32 = 7, UINT64 = 8, FLOAT = 9, DOUBLE = 10, CHAR = 11
};

// ---------------------------------------------------------------- SArray ----
template <typename V> class SArray {
 public:
  SArray() {}
  explicit SArray(size_t n) { resize(n); }
  // zero-copy constructor (shared_array.h:57-59, reset in shared_array_inl.h:54-66)
  SArray(V* data, size_t size, bool deletable = true) {
    size_ = cap_ = size;
    if (deletable) ptr_.reset(reinterpret_cast<char*>(data), std::default_delete<char[]>());
    else ptr_.reset(reinterpret_cast<char*>(data), [](char*) {});
  }
  std::shared_ptr<char>& pointer() { return ptr_; }  // (the reference's is shared_ptr<void>)
  template <typename W> explicit SArray(const SArray<W>& o) {
    size_ = o.size() * sizeof(W) / sizeof(V);
    ptr_ = o.ptr();
  }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  void clear() { size_ = 0; ptr_.reset(); }
  void resize(size_t n) {
    if (n * sizeof(V) > cap_bytes()) {
      std::shared_ptr<char> p(new char[n * sizeof(V) + 1], std::default_delete<char[]>());
      if (size_) memcpy(p.get(), ptr_.get(), size_ * sizeof(V));
      ptr_ = p; cap_ = n * sizeof(V);
    }
    size_ = n;
  }
  V* data() const { return reinterpret_cast<V*>(ptr_.get()); }
  V& operator[](size_t i) const { return data()[i]; }
  V* begin() const { return data(); }
  V* end() const { return data() + size_; }
  const std::shared_ptr<char>& ptr() const { return ptr_; }

  // Eigen::Map<Array>::minCoeff/maxCoeff stand-in (first extreme element).
  struct EArray {
    const V* p; size_t n;
    V minCoeff() const { return *std::min_element(p, p + n); }
    V maxCoeff() const { return *std::max_element(p, p + n); }
  };
  EArray EigenArray() const { return EArray{data(), size_}; }

  SArray<char> CompressTo() const;
  void UncompressFrom(const char* src, size_t src_size);
  void UncompressFrom(const SArray<char>& src) { UncompressFrom(src.data(), src.size()); }

 private:
  size_t cap_bytes() const { return ptr_ ? cap_ : 0; }
  size_t size_ = 0;
  size_t cap_ = 0;
  std::shared_ptr<char> ptr_;
};

// ---------------------------------------------------------------- Range ----
struct PbRange {
  uint64 b = 0, e = 0;
  uint64 begin() const { return b; }
  uint64 end() const { return e; }
  void set_begin(uint64 v) { b = v; }
  void set_end(uint64 v) { e = v; }
};
template <class T> class Range {
 public:
  Range() {}
  Range(const PbRange& pb) : b_(pb.begin()), e_(pb.end()) {}
  Range(T b, T e) : b_(b), e_(e) {}
  T begin() const { return b_; }
  T end() const { return e_; }
  bool operator==(const Range& o) const { return b_ == o.b_ && e_ == o.e_; }
  static Range All() { return Range(0, (T)-1); }
  void To(PbRange* pb) const { pb->set_begin(b_); pb->set_end(e_); }
 private:
  T b_ = 0, e_ = 0;
};

// ------------------------------------------------------------ protos ----
struct FilterConfig_FixedFloatConfig {
  bool has_min_value() const { return has_min_; }
  bool has_max_value() const { return has_max_; }
  float min_value() const { return min_; }
  float max_value() const { return max_; }
  void set_min_value(float v) { min_ = v; has_min_ = true; }
  void set_max_value(float v) { max_ = v; has_max_ = true; }
  bool has_min_ = false, has_max_ = false;
  float min_ = -1.f, max_ = 1.f;   // proto defaults (filter.proto:22-25)
};

struct FilterConfig {
  enum Type { KEY_CACHING = 1, COMPRESSING = 2, FIXING_FLOAT = 3, NOISE = 4 };
  typedef FilterConfig_FixedFloatConfig FixedFloatConfig;

  Type type() const { return type_; }
  void set_type(Type t) { type_ = t; }
  bool clear_cache_if_done() const { return clear_cache_if_done_; }
  int32 num_bytes() const { return num_bytes_; }
  int fixed_point_size() const { return (int)fixed_point_.size(); }
  FixedFloatConfig* add_fixed_point() { fixed_point_.emplace_back(); return &fixed_point_.back(); }
  FixedFloatConfig* mutable_fixed_point(int i) { return &fixed_point_.at(i); }
  const FixedFloatConfig& fixed_point(int i) const { return fixed_point_.at(i); }
  float mean() const { return mean_; }
  float std() const { return std_; }
  bool has_signature() const { return has_signature_; }
  uint32 signature() const { return signature_; }
  void set_signature(uint32 s) { signature_ = s; has_signature_ = true; }
  void clear_signature() { signature_ = 0; has_signature_ = false; }
  void clear_uncompressed_size() { uncompressed_size_.clear(); }
  void add_uncompressed_size(uint64 v) { uncompressed_size_.push_back(v); }
  int uncompressed_size_size() const { return (int)uncompressed_size_.size(); }
  uint64 uncompressed_size(int i) const { return uncompressed_size_.at(i); }

  Type type_ = KEY_CACHING;
  bool clear_cache_if_done_ = false;
  int32 num_bytes_ = 3;            // filter.proto:21 default
  std::deque<FixedFloatConfig> fixed_point_;
  float mean_ = 0.f, std_ = 0.f;
  bool has_signature_ = false;
  uint32 signature_ = 0;
  std::vector<uint64> uncompressed_size_;
};

struct ParamCall {
  bool push() const { return push_; }
  bool push_ = false;
};

struct Task {
  bool request() const { return request_; }
  int32 key_channel() const { return key_channel_; }
  const PbRange& key_range() const { return key_range_; }
  bool has_key_range() const { return has_key_range_; }
  PbRange* mutable_key_range() { has_key_range_ = true; return &key_range_; }
  void clear_has_key() { has_key_ = false; }
  void set_has_key(bool v) { has_key_ = v; }
  void set_key_type(DataType t) { key_type_ = t; }
  int value_type_size() const { return (int)value_type_.size(); }
  DataType value_type(int i) const { return value_type_.at(i); }
  int filter_size() const { return (int)filter_.size(); }
  const FilterConfig& filter(int i) const { return filter_.at(i); }
  FilterConfig* mutable_filter(int i) { return &filter_.at(i); }
  FilterConfig* add_filter() { filter_.emplace_back(); return &filter_.back(); }
  bool has_param() const { return has_param_; }
  const ParamCall& param() const { return param_; }

  bool request_ = false;
  int32 key_channel_ = 0;
  PbRange key_range_;
  bool has_key_range_ = false;
  bool has_key_ = false;
  DataType key_type_ = OTHER;
  std::vector<DataType> value_type_;
  std::deque<FilterConfig> filter_;
  bool has_param_ = false;
  ParamCall param_;
};

// ---------------------------------------------------------------- Message --
struct Message {
  Task task;
  SArray<char> key;
  std::vector<SArray<char>> value;
  bool has_key() const { return !key.empty(); }
  void clear_key() { task.clear_has_key(); key.clear(); }
  template <typename T> void set_key(const SArray<T>& k) {
    task.set_key_type(CHAR);   // only set_key<char> is reached from the filters
    if (has_key()) clear_key();
    task.set_has_key(true);
    key = SArray<char>(k);
    if (!task.has_key_range()) Range<Key>::All().To(task.mutable_key_range());
  }
  std::string DebugString() const { return "[stub message]"; }
};

// ------------------------------------------------------------ Filter ----
// Declared exactly as filter.h:9-24 so that the reference's filter.cc
// provides Filter::create / Filter::find.
class Filter {
 public:
  Filter() {}
  virtual ~Filter() {}
  static Filter* create(const FilterConfig& conf);
  virtual void encode(Message* msg) {}
  virtual void decode(Message* msg) {}
  static FilterConfig* find(FilterConfig::Type type, Message* msg) {
    return find(type, &(msg->task));
  }
  static FilterConfig* find(FilterConfig::Type type, Task* task);
};

}  // namespace PS

namespace std {
template <> struct hash<std::pair<int, PS::Range<PS::Key>>> {
  size_t operator()(const std::pair<int, PS::Range<PS::Key>>& s) const {
    return std::hash<uint64_t>()((uint64_t)s.first * 0x9E3779B97F4A7C15ull ^
                                 s.second.begin() ^ (s.second.end() << 1));
  }
};
}  // namespace std
