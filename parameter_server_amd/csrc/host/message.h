// Host-side message model of libpsf: the fields of the reference's Message /
// Task / FilterConfig that the codec chain reads and writes, with buffers that
// live in HBM (or host memory at the host edge).
//
//   Message     <- reference src/system/message.h:10-76 (key, value, has_key,
//                  clear_key, set_key<char> semantics incl. key_type=CHAR and the
//                  default key_range = Range::All())
//   Task        <- src/system/proto/task.proto:10-57 (request, key_range,
//                  key_channel, has_key, key_type, value_type, filter, param.push)
//   FilterConfig<- src/filter/proto/filter.proto:3-35 (field defaults and has-bits)
//   Buffer      <- SArray<char> (util/shared_array.h:29): a shared, zero-copy byte
//                  view; the owner keeps the storage alive (custom deleter, as the
//                  van's zero-copy frames do, van.cc:244-249).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace psf {

// An append-only sequence whose elements never move while it grows (pointers
// to them stay valid across emplace_back, as std::deque's do), with the first
// N elements stored inline: copying a Task of a few filters allocates nothing,
// where a std::deque allocates a map and a node even when empty (the batched
// drivers copy a Task per message per step).
template <typename T, size_t N>
class StableList {
 public:
  template <typename L, typename R>
  class Iter {
   public:
    Iter(L* l, size_t i) : l_(l), i_(i) {}
    R& operator*() const { return (*l_)[i_]; }
    R* operator->() const { return &(*l_)[i_]; }
    Iter& operator++() { ++i_; return *this; }
    bool operator==(const Iter& o) const { return i_ == o.i_; }
    bool operator!=(const Iter& o) const { return i_ != o.i_; }
   private:
    L* l_;
    size_t i_;
  };
  typedef Iter<StableList, T> iterator;
  typedef Iter<const StableList, const T> const_iterator;

  StableList() = default;
  StableList(const StableList& o) { append(o); }
  StableList& operator=(const StableList& o) {
    if (this != &o) { clear(); append(o); }
    return *this;
  }
  // moving the list moves its elements (the inline ones to new addresses:
  // stability holds while a list grows, not across a move of the list)
  StableList(StableList&& o) noexcept { take(o); }
  StableList& operator=(StableList&& o) noexcept {
    if (this != &o) { clear(); take(o); }
    return *this;
  }
  ~StableList() { clear(); }

  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T& operator[](size_t i) { return i < N ? inl()[i] : (*extra_)[i - N]; }
  const T& operator[](size_t i) const { return i < N ? inl()[i] : (*extra_)[i - N]; }
  T& back() { return (*this)[n_ - 1]; }
  const T& back() const { return (*this)[n_ - 1]; }
  iterator begin() { return iterator(this, 0); }
  iterator end() { return iterator(this, n_); }
  const_iterator begin() const { return const_iterator(this, 0); }
  const_iterator end() const { return const_iterator(this, n_); }

  template <typename... A>
  T& emplace_back(A&&... a) {
    if (n_ < N) {
      T* p = new (inl() + n_) T(std::forward<A>(a)...);
      ++n_;
      return *p;
    }
    if (!extra_) extra_.reset(new std::deque<T>());
    extra_->emplace_back(std::forward<A>(a)...);
    ++n_;
    return extra_->back();
  }
  void clear() {
    for (size_t i = 0; i < n_ && i < N; ++i) inl()[i].~T();
    extra_.reset();
    n_ = 0;
  }

 private:
  void append(const StableList& o) {
    for (size_t i = 0; i < o.n_; ++i) emplace_back(o[i]);
  }
  void take(StableList& o) noexcept {
    const size_t k = o.n_ < N ? o.n_ : N;
    for (size_t i = 0; i < k; ++i) new (inl() + i) T(std::move(o.inl()[i]));
    extra_ = std::move(o.extra_);
    n_ = o.n_;
    o.clear();
  }
  T* inl() { return std::launder(reinterpret_cast<T*>(buf_)); }
  const T* inl() const { return std::launder(reinterpret_cast<const T*>(buf_)); }
  alignas(T) unsigned char buf_[N * sizeof(T)];
  size_t n_ = 0;
  std::unique_ptr<std::deque<T>> extra_;
};

enum class Loc : int { kHost = 0, kDevice = 1 };

// Buffer::layout: kLayoutStored1 / 2 -- `bytes` payload bytes written into the
// stored snappy stream layout at ptr (psf_internal.h StoredLayout), by FIXING_FLOAT with num_bytes 1 / 2: output
// that only COMPRESSING (next in the chain) reads
enum BufferLayout : uint8_t { kLayoutPlain = 0, kLayoutStored1 = 1, kLayoutStored2 = 2 };
struct Buffer {
  std::shared_ptr<void> owner;  // null => caller-owned memory (caller keeps it alive)
  uint8_t* ptr = nullptr;
  size_t bytes = 0;
  Loc loc = Loc::kDevice;
  BufferLayout layout = kLayoutPlain;
  bool empty() const { return bytes == 0; }
  void clear() { owner.reset(); ptr = nullptr; bytes = 0; }
};

// glog CHECK failures of the reference map to this exception; the C ABI turns
// it into a status code (include/psf.h).
struct CheckError : std::runtime_error {
  int code;
  CheckError(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

struct KeyRange {
  uint64_t begin = 0, end = 0;
  bool operator==(const KeyRange& o) const { return begin == o.begin && end == o.end; }
  static KeyRange All() { return KeyRange{0, ~0ull}; }  // range.h:92-95
};

struct RangeBatch;  // context.h

struct FixedFloatConfig {  // filter.proto:22-25
  bool has_min = false, has_max = false;
  float min_value = -1.f, max_value = 1.f;
  void set_min(float v) { min_value = v; has_min = true; }
  void set_max(float v) { max_value = v; has_max = true; }
  // A batched encode leaves computed min/max on the device: entry `pending_idx`
  // of `pending` holds {min, max, status}.  A decode on the same context reads
  // them there; every host reader calls settle() first, which brings them over
  // (and reports CHECK_GT(bin, 0) then).
  std::shared_ptr<RangeBatch> pending;
  int pending_idx = -1;
  bool pending_min = false, pending_max = false;
  void settle();                      // filters.cc
  const float* device_range() const;  // filters.cc
};

struct FilterConfig {  // filter.proto:3-35
  enum Type { KEY_CACHING = 1, COMPRESSING = 2, FIXING_FLOAT = 3, NOISE = 4 };
  Type type = KEY_CACHING;
  bool clear_cache_if_done = false;            // field 20
  int32_t num_bytes = 3;                       // field 5, default 3
  StableList<FixedFloatConfig, 2> fixed_point;  // field 4 (stable addresses)
  float mean = 0.f, std = 0.f;                 // fields 6, 7
  bool has_signature = false;                  // field 2
  uint32_t signature = 0;
  std::vector<uint64_t> uncompressed_size;     // field 3
  // proto2 has-bits of the optional fields above (what the wire carries)
  bool has_clear_cache_if_done = false, has_num_bytes = false, has_mean = false, has_std = false;
};

struct Task {
  bool request = false;
  int32_t key_channel = 0;
  bool has_key_range = false;
  KeyRange key_range;
  bool has_key = false;
  bool has_key_type = false;
  int key_type = 0;
  std::vector<int> value_type;
  StableList<FilterConfig, 4> filter;  // stable addresses
  bool has_param = false;
  bool push = false;  // param.push
};

// A value array left FIXING_FLOAT-encoded by a decode that deferred the
// dequantise to its consumer (RemoteNode::set_defer_dequant): the codes stay in
// `value[i]`, and this records what ff_decode would have used
// (fixing_float.h:89-101).  nb == 0: the array holds decoded data.
struct PendingDequant {
  int nb = 0;
  float min_value = 0.f, max_value = 0.f;
};

struct Message {
  Task task;
  Buffer key;
  std::vector<Buffer> value;
  std::vector<PendingDequant> pending;  // empty, or one entry per value array
  // value arrays whose FIXING_FLOAT decode already ran, fused into the
  // COMPRESSING decode before it (decode_batch); empty, or one per value array
  std::vector<uint8_t> predecoded;
  // where a FIXING_FLOAT decode writes value array i (empty, or one entry per
  // value array; an entry of the decoded size names device memory the caller
  // owns -- e.g. the array's place in a pull's key-ordered result -- and any
  // other entry is ignored).  Only a hint: the decode that cannot use it
  // allocates, and the caller checks where value[i] landed.
  std::vector<Buffer> value_dest;
  bool key_frame_seen = false;          // Van::Recv bookkeeping (psf_msg_recv_frame)

  bool is_pending(size_t i) const { return i < pending.size() && pending[i].nb != 0; }

  bool has_key() const { return !key.empty(); }
  void clear_key() { task.has_key = false; key.clear(); }
  // message.h:70-76 (set_key<char>)
  void set_key(const Buffer& k) {
    task.key_type = 11;  // CHAR
    task.has_key_type = true;
    if (has_key()) clear_key();
    task.has_key = true;
    key = k;
    if (!task.has_key_range) { task.has_key_range = true; task.key_range = KeyRange::All(); }
  }
};
// the batched drivers keep messages in vectors: growing one must move them,
// not copy every Task (and its side-info references) again
static_assert(std::is_nothrow_move_constructible<Message>::value, "Message moves cheaply");

}  // namespace psf
