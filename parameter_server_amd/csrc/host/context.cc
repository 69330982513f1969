#include "context.h"

#include <sched.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <iterator>
#include <list>
#include <unordered_map>
#include <vector>

namespace psf {

// The stream plus a stream-ordered caching allocator for codec outputs.  A
// buffer whose last reference drops goes back on a free list of its size class
// and is handed to a later allocation on the same stream, so stream order
// alone protects it (no per-message hipMallocAsync/hipFreeAsync packets in the
// queue).  Shared by every Buffer the context allocates, so it outlives the
// Context if buffers do.
//
// The free lists are bounded: the bytes they hold (HBM and pinned host memory
// alike) stay under a per-context cap (Context::kDefaultCache*, or
// psf_context_set_cache_limit).  A release that would pass the cap first
// frees the least recently released blocks, after the stream has drained (a
// block on a free list may still be in use by queued kernels).  A server that
// sees many distinct message sizes therefore keeps at most the cap cached,
// on top of what its live messages hold.
struct Context::StreamHolder {
  int device;
  hipStream_t stream;
  bool own;
  std::mutex mu;
  struct Pool {
    struct Entry {
      size_t cls;
      void* p;
    };
    std::list<Entry> lru;  // released blocks, oldest first
    std::unordered_map<size_t, std::vector<std::list<Entry>::iterator>> by_class;  // per class, oldest first
    size_t cached = 0, allocated = 0, cap = 0;
    uint64_t evictions = 0;
    void* take(size_t cls) {
      auto it = by_class.find(cls);
      if (it == by_class.end() || it->second.empty()) return nullptr;
      auto e = it->second.back();  // the most recently released
      it->second.pop_back();
      void* p = e->p;
      lru.erase(e);
      cached -= cls;
      return p;
    }
    // the blocks to free so that `extra` more cached bytes fit the cap
    void make_room(size_t extra, std::vector<Entry>* out) {
      while (!lru.empty() && cached + extra > cap) {
        Entry e = lru.front();
        auto& v = by_class[e.cls];
        v.erase(v.begin());  // the class's oldest is the overall oldest of its class
        lru.pop_front();
        cached -= e.cls;
        allocated -= e.cls;
        ++evictions;
        out->push_back(e);
      }
    }
    void give(size_t cls, void* p) {
      lru.push_back(Entry{cls, p});
      by_class[cls].push_back(std::prev(lru.end()));
      cached += cls;
    }
  };
  Pool dev, host;

  StreamHolder(int d, hipStream_t s, bool o) : device(d), stream(s), own(o) {
    dev.cap = kDefaultCacheBytes;
    host.cap = kDefaultPinnedCacheBytes;
  }
  ~StreamHolder() {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    for (auto& e : dev.lru) (void)hipFree(e.p);
    for (auto& e : host.lru) (void)hipHostFree(e.p);
    if (own) (void)hipStreamDestroy(stream);
  }
  static size_t size_class(size_t bytes) {
    if (bytes <= 4096) return 4096;
    if (bytes <= (1u << 20)) {  // next power of two
      size_t c = 8192;
      while (c < bytes) c <<= 1;
      return c;
    }
    return (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);  // 1 MiB granules
  }
  // release `evict` (taken out of a pool under the lock) once the stream has drained
  void free_blocks(const std::vector<Pool::Entry>& evict, bool pinned) {
    if (evict.empty()) return;
    (void)hipStreamSynchronize(stream);
    for (const auto& e : evict) (void)(pinned ? hipHostFree(e.p) : hipFree(e.p));
  }
  void* get(size_t cls) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (void* p = dev.take(cls)) return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess) {  // out of HBM: drop every cached block, then once more
      (void)hipGetLastError();
      std::vector<Pool::Entry> evict;
      {
        std::lock_guard<std::mutex> l(mu);
        const size_t c = dev.cap;
        dev.cap = 0;
        dev.make_room(0, &evict);
        dev.cap = c;
      }
      free_blocks(evict, false);
      PSF_HIP_CHECK(hipMalloc(&p, cls));
    }
    std::lock_guard<std::mutex> l(mu);
    dev.allocated += cls;
    return p;
  }
  void put(size_t cls, void* p) {
    std::vector<Pool::Entry> evict;
    bool drop = false;
    {
      std::lock_guard<std::mutex> l(mu);
      if (cls > dev.cap) {  // larger than the whole cache: not kept
        drop = true;
        dev.allocated -= cls;
        ++dev.evictions;
      } else {
        dev.make_room(cls, &evict);
        dev.give(cls, p);
      }
    }
    if (drop) evict.push_back(Pool::Entry{cls, p});
    free_blocks(evict, false);
  }
  void* get_pinned(size_t cls) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (void* p = host.take(cls)) return p;
    }
    void* p = nullptr;
    PSF_HIP_CHECK(hipHostMalloc(&p, cls, hipHostMallocMapped | hipHostMallocCoherent));
    std::lock_guard<std::mutex> l(mu);
    host.allocated += cls;
    return p;
  }
  void put_pinned(size_t cls, void* p) {
    std::vector<Pool::Entry> evict;
    bool drop = false;
    {
      std::lock_guard<std::mutex> l(mu);
      if (cls > host.cap) {
        drop = true;
        host.allocated -= cls;
        ++host.evictions;
      } else {
        host.make_room(cls, &evict);
        host.give(cls, p);
      }
    }
    if (drop) evict.push_back(Pool::Entry{cls, p});
    free_blocks(evict, true);
  }
  void set_caps(size_t dev_cap, size_t host_cap) {
    std::vector<Pool::Entry> ed, eh;
    {
      std::lock_guard<std::mutex> l(mu);
      dev.cap = dev_cap;
      host.cap = host_cap;
      dev.make_room(0, &ed);
      host.make_room(0, &eh);
    }
    free_blocks(ed, false);
    free_blocks(eh, true);
  }
  void stats(MemoryStats* s) {
    std::lock_guard<std::mutex> l(mu);
    s->dev_cached = dev.cached;
    s->dev_cap = dev.cap;
    s->dev_allocated = dev.allocated;
    s->dev_evictions = dev.evictions;
    s->host_cached = host.cached;
    s->host_cap = host.cap;
    s->host_allocated = host.allocated;
    s->host_evictions = host.evictions;
  }
};

void Context::set_cache_limit(size_t dev_bytes, size_t pinned_bytes) {
  if (holder_) holder_->set_caps(dev_bytes, pinned_bytes);
}
Context::MemoryStats Context::memory_stats() const {
  MemoryStats s;
  if (holder_) holder_->stats(&s);
  return s;
}

// compress: the look-back words of up to 8191 fragments (512 MiB per launch);
// uncompress: the control words of kSnappyBatchMax streams
static constexpr size_t kZeroBytes[Context::kZeroKinds] = {65536, 2048};

Context::Context(int device, hipStream_t stream, bool own) : device_(device), stream_(nullptr) {
  if (device < 0) return;  // host-only context: host-resident buffers, no HIP calls
  PSF_HIP_CHECK(hipSetDevice(device));
  if (own) stream = nullptr;
  if (own) PSF_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  stream_ = stream;
  // constructed in place: a temporary StreamHolder would destroy the stream
  holder_ = std::shared_ptr<StreamHolder>(new StreamHolder(device, stream, own));
  PSF_HIP_CHECK(hipMalloc(&d_partials_, 2 * sizeof(uint64_t) * kMaxGrid));
  PSF_HIP_CHECK(hipMalloc(&zero_base_, 2 * (kZeroBytes[0] + kZeroBytes[1])));
  PSF_HIP_CHECK(hipMemset(zero_base_, 0, 2 * (kZeroBytes[0] + kZeroBytes[1])));
  PSF_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d_slots_), sizeof(Slot) * kSlots));
  PSF_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_slots_), sizeof(Slot) * kSlots,
                              hipHostMallocMapped | hipHostMallocCoherent));
  memset(h_slots_, 0, sizeof(Slot) * kSlots);
  PSF_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&m_slots_), h_slots_, 0));
  PSF_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&lazy_h_), 16 * kLazyRing,
                              hipHostMallocMapped | hipHostMallocCoherent));
  memset(lazy_h_, 0, 16 * kLazyRing);
  PSF_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&lazy_m_), lazy_h_, 0));
}

Context::~Context() {
  if (device_ < 0) return;
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  for (auto& u : ring_uses_) {  // messages may outlive the context: leave their ranges on the host
    auto rb = u.rb.lock();
    if (rb && !rb->done) {
      memcpy(rb->host.data(), rb->ring, rb->host.size() * 4);
      rb->done = true;
    }
  }
  ring_uses_.clear();
  tracked_.clear();
  for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  (void)hipHostFree(lazy_h_);
  (void)hipFree(d_partials_);
  (void)hipFree(zero_base_);
  (void)hipFree(d_slots_);
  (void)hipHostFree(h_slots_);
}

Buffer Context::alloc(size_t bytes) {
  Buffer b;
  b.bytes = bytes;
  b.loc = Loc::kDevice;
  if (bytes == 0) return b;
  if (device_ < 0) throw CheckError(kErrArg, "host-only context cannot hold HBM buffers");
  const size_t cls = StreamHolder::size_class(bytes);
  void* p = holder_->get(cls);
  auto holder = holder_;
  b.owner = std::shared_ptr<void>(p, [holder, cls](void* q) { holder->put(cls, q); });
  b.ptr = static_cast<uint8_t*>(p);
  return b;
}

#ifdef PSF_HOST_PROF
int64_t g_hprof_ns[kHProfSlots], g_hprof_n[kHProfSlots];
extern "C" int psf_debug_host_prof(int64_t* ns, int64_t* n, int reset) {
  for (int i = 0; i < kHProfSlots; ++i) {
    ns[i] = g_hprof_ns[i];
    n[i] = g_hprof_n[i];
    if (reset) g_hprof_ns[i] = g_hprof_n[i] = 0;
  }
  return 0;
}
#endif

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

ZeroPair Context::zero_pair(int kind, size_t need) {
  if (device_ < 0 || kind < 0 || kind >= kZeroKinds || need > kZeroBytes[kind]) return ZeroPair{};
  uint8_t* base = static_cast<uint8_t*>(zero_base_);
  for (int k = 0; k < kind; ++k) base += 2 * kZeroBytes[k];
  const int p = zero_parity_[kind];
  zero_parity_[kind] ^= 1;
  return ZeroPair{base + p * kZeroBytes[kind], base + (p ^ 1) * kZeroBytes[kind], kZeroBytes[kind]};
}

Context::Pinned Context::pinned(size_t bytes) {
  Pinned p;
  if (bytes == 0) return p;
  if (device_ < 0) throw CheckError(kErrArg, "host-only context has no mapped memory");
  const size_t cls = StreamHolder::size_class(bytes);
  void* h = holder_->get_pinned(cls);
  auto holder = holder_;
  p.owner = std::shared_ptr<void>(h, [holder, cls](void* q) { holder->put_pinned(cls, q); });
  p.host = static_cast<uint8_t*>(h);
  void* d = nullptr;
  PSF_HIP_CHECK(hipHostGetDevicePointer(&d, h, 0));
  p.dev = static_cast<uint8_t*>(d);
  p.bytes = bytes;
  return p;
}

hipEvent_t Context::take_event() {
  if (!events_.empty()) {
    hipEvent_t e = events_.back();
    events_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  PSF_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

void Context::give_event(hipEvent_t e) {
  if (e) events_.push_back(e);
}

void Context::wait_event(hipEvent_t e, int w) {
  hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return;
  WaitTimer wt(this, static_cast<HostWait>(w));
  for (uint64_t spin = 0; q == hipErrorNotReady; ++spin) {
    if (spin > 4096) sched_yield();
    q = hipEventQuery(e);
  }
  if (q != hipSuccess) throw CheckError(kErrHip, std::string("event wait failed: ") + hipGetErrorString(q));
}

void Context::wait_ticket(int i, uint32_t ticket) {
  if (device_ < 0) throw CheckError(kErrArg, "host-only context has no device workspace");
  const Slot* s = h_slots_ + i;
  if (__atomic_load_n(&s->ticket, __ATOMIC_ACQUIRE) == ticket) return;
  WaitTimer wt(this, kWaitPublish);
  for (uint64_t spin = 0;; ++spin) {
    if (__atomic_load_n(&s->ticket, __ATOMIC_ACQUIRE) == ticket) return;
    if ((spin & 255) == 255) {
      hipError_t q = hipStreamQuery(stream_);
      if (q == hipSuccess) {  // stream drained: the publish must be visible now
        if (__atomic_load_n(&s->ticket, __ATOMIC_ACQUIRE) == ticket) return;
        throw CheckError(kErrHip, "kernel finished without publishing its side-info");
      }
      if (q != hipErrorNotReady)
        throw CheckError(kErrHip, std::string("stream failed: ") + hipGetErrorString(q));
      if (spin > (1u << 16)) sched_yield();
    }
  }
}

uint32_t Context::wait_crc(int i, uint32_t ticket) {
  if (device_ < 0) throw CheckError(kErrArg, "host-only context has no device workspace");
  const Slot* s = h_slots_ + i;
  {
    const uint64_t w = __atomic_load_n(&s->crc_ticket, __ATOMIC_ACQUIRE);
    if ((uint32_t)(w >> 32) == ticket) return (uint32_t)w;
  }
  WaitTimer wt(this, kWaitPublish);
  for (uint64_t spin = 0;; ++spin) {
    uint64_t w = __atomic_load_n(&s->crc_ticket, __ATOMIC_ACQUIRE);
    if ((uint32_t)(w >> 32) == ticket) return (uint32_t)w;
    if ((spin & 255) == 255) {
      hipError_t q = hipStreamQuery(stream_);
      if (q == hipSuccess) {  // stream drained: the publish must be visible now
        w = __atomic_load_n(&s->crc_ticket, __ATOMIC_ACQUIRE);
        if ((uint32_t)(w >> 32) == ticket) return (uint32_t)w;
        throw CheckError(kErrHip, "kernel finished without publishing its CRC");
      }
      if (q != hipErrorNotReady)
        throw CheckError(kErrHip, std::string("stream failed: ") + hipGetErrorString(q));
      if (spin > (1u << 16)) sched_yield();
    }
  }
}

void Context::sync() {
  if (device_ < 0) return;
  WaitTimer wt(this, kWaitSync);
  PSF_HIP_CHECK(hipStreamSynchronize(stream_));
}

void RangeBatch::resolve(bool synced) {
  if (done) return;
  if (!synced) ctx->sync();  // the kernels' host-mapped stores are visible after it
  memcpy(host.data(), ring, host.size() * 4);
  done = true;
}

float* Context::claim_lazy(const std::shared_ptr<RangeBatch>& rb, int n) {
  if (n <= 0 || (uint64_t)n > kLazyRing) throw CheckError(kErrArg, "lazy side-info batch too large");
  uint64_t start = lazy_next_;
  const uint64_t pos = start % kLazyRing;
  if (pos + (uint64_t)n > kLazyRing) start += kLazyRing - pos;  // records stay contiguous
  // this claim overwrites the records of absolute indices [start - R, start + n - R)
  bool synced = false;
  while (!ring_uses_.empty() && ring_uses_.front().start + kLazyRing < start + (uint64_t)n) {
    auto old = ring_uses_.front().rb.lock();
    ring_uses_.pop_front();
    if (old && !old->done) {
      if (!synced) sync();
      synced = true;
      old->resolve(true);
    }
  }
  lazy_next_ = start + (uint64_t)n;
  ring_uses_.push_back(RingUse{rb, start, (uint64_t)n});
  const uint64_t at = start % kLazyRing;
  rb->ring = lazy_h_ + 4 * at;
  return reinterpret_cast<float*>(lazy_m_ + 4 * at);
}

void Context::track(std::shared_ptr<RangeBatch> rb) {
  tracked_.push_back(std::move(rb));
  if (tracked_.size() >= kMaxTracked) check_ranges();
}

void Context::check_ranges() {
  std::vector<std::shared_ptr<RangeBatch>> t;
  t.swap(tracked_);
  bool bad = false;
  if (!t.empty()) sync();
  for (auto& rb : t) {
    rb->resolve(true);
    for (size_t i = 2; i < rb->host.size(); i += 4) bad |= (int32_t)rb->host[i] != kOk;
  }
  if (bad) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
}

Buffer Context::to_device(const Buffer& b) {
  if (b.loc == Loc::kDevice || b.empty()) return b;
  Buffer d = alloc(b.bytes);
  PSF_HIP_CHECK(hipMemcpyAsync(d.ptr, b.ptr, b.bytes, hipMemcpyHostToDevice, stream_));
  return d;
}

const void* Context::noise_table(int value_type, size_t n) {
  if (device_ < 0) throw CheckError(kErrArg, "host-only context has no device workspace");
  Buffer& t = value_type == kFloat ? noise_f32_ : noise_f64_;
  const size_t vsz = value_type == kFloat ? 4 : 8;
  if (t.bytes / vsz >= n) return t.ptr;
  size_t len = t.bytes / vsz * 2;
  if (len < n) len = n;
  if (len < (1u << 16)) len = 1u << 16;
  Buffer nt = alloc(len * vsz);
  Buffer scratch = alloc(noise_scratch_bytes(len));
  int s = noise_build_table(value_type, nt.ptr, len, scratch.ptr, scratch.bytes, stream_, &prof_);
  if (s != kOk) throw CheckError(s, "NOISE table build failed");
  t = nt;
  return t.ptr;
}

// ------------------------------------------------------------ clock ------
static std::atomic<bool> g_clock_override{false};
static std::atomic<int64_t> g_clock_value{0};

void set_clock_override(bool enable, int64_t t) {
  g_clock_value.store(t);
  g_clock_override.store(enable);
}

int32_t ff_clock_seed() {
  if (g_clock_override.load()) return (int32_t)g_clock_value.load();
  return (int32_t)time(nullptr);  // `int seed = time(NULL);`
}

// ------------------------------------------------------------ crc32c -----
uint32_t crc32c_host(const void* p, size_t n) {
  static uint32_t table[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      table[i] = c;
    }
  });
  const uint8_t* b = static_cast<const uint8_t*>(p);
  uint32_t l = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) l = table[(l ^ b[i]) & 0xFF] ^ (l >> 8);
  return l ^ 0xFFFFFFFFu;
}

}  // namespace psf
