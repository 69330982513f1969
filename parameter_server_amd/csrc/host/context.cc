#include "context.h"

#include <sched.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <algorithm>
#include <iterator>
#include <list>
#include <map>
#include <vector>

namespace psf {

// The stream a context launches on, plus its share of the device's caching
// allocator for codec outputs.  A buffer whose last reference drops goes back
// on a free list and is handed to a later allocation on the SAME stream, so
// stream order alone protects it (no per-message hipMallocAsync/hipFreeAsync
// packets in the queue).  Shared by every Buffer the context allocates, so it
// outlives the Context if buffers do.
//
// The free lists are bounded per DEVICE, not per context (DevicePool): the
// bytes cached by every holder on a device (HBM and pinned host memory alike)
// stay under one cap (Context::kDefaultCache*, psf_set_device_cache_limit).  A
// release that would pass the cap first frees the least recently released
// blocks of the whole device, whichever holder released them, each after its
// own stream has drained (a block on a free list may still be in use by
// kernels queued before its release); an hipMalloc that fails drops every
// cached block of the device and tries again.  So a server with many peers
// (one context per peer, or per filter instance) keeps at most the cap cached
// on top of what its live messages hold.
struct Context::StreamHolder : std::enable_shared_from_this<Context::StreamHolder> {
  int device;
  hipStream_t stream;
  bool own;
  bool retired = false;  // its context is gone: releases are freed, not cached
  // this holder's share (under the pool's lock)
  uint64_t dev_cached = 0, dev_allocated = 0, dev_evictions = 0;
  uint64_t host_cached = 0, host_allocated = 0, host_evictions = 0;
  StreamHolder(int d, hipStream_t s, bool o) : device(d), stream(s), own(o) {}
  ~StreamHolder() {
    int cur = -1;  // (no DeviceScope: a destructor must not throw)
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    if (own) (void)hipStreamDestroy(stream);
    if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
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
  void* get(size_t cls);
  void put(size_t cls, void* p);
  void* get_pinned(size_t cls);
  void put_pinned(size_t cls, void* p);
  void retire();  // the context is gone: free this holder's cached blocks
};

namespace {
typedef Context::StreamHolder Holder;

struct PoolEntry {
  size_t cls;
  void* p;
  std::shared_ptr<Holder> h;  // keeps the stream alive until the block is freed
};

// released blocks of one kind (HBM or pinned) on one device
struct PoolSide {
  bool pinned;
  std::list<PoolEntry> lru;  // oldest first
  // per (holder, class): the entries, oldest first
  std::map<std::pair<const Holder*, size_t>, std::vector<std::list<PoolEntry>::iterator>> by_key;
  uint64_t cached = 0, allocated = 0, cap = 0, evictions = 0;
  uint64_t& h_cached(Holder* h) { return pinned ? h->host_cached : h->dev_cached; }
  uint64_t& h_allocated(Holder* h) { return pinned ? h->host_allocated : h->dev_allocated; }
  uint64_t& h_evictions(Holder* h) { return pinned ? h->host_evictions : h->dev_evictions; }

  void* take(Holder* h, size_t cls) {
    auto it = by_key.find({h, cls});
    if (it == by_key.end() || it->second.empty()) return nullptr;
    auto e = it->second.back();  // the most recently released
    it->second.pop_back();
    if (it->second.empty()) by_key.erase(it);
    void* p = e->p;
    lru.erase(e);
    cached -= cls;
    h_cached(h) -= cls;
    return p;
  }
  void unlink(std::list<PoolEntry>::iterator e, std::vector<PoolEntry>* out) {
    auto k = by_key.find({e->h.get(), e->cls});
    auto& v = k->second;
    v.erase(std::find(v.begin(), v.end(), e));
    if (v.empty()) by_key.erase(k);
    cached -= e->cls;
    allocated -= e->cls;
    ++evictions;
    h_cached(e->h.get()) -= e->cls;
    h_allocated(e->h.get()) -= e->cls;
    ++h_evictions(e->h.get());
    out->push_back(std::move(*e));
    lru.erase(e);
  }
  // the blocks to free so that `extra` more cached bytes fit the cap
  void make_room(uint64_t extra, std::vector<PoolEntry>* out) {
    while (!lru.empty() && cached + extra > cap) unlink(lru.begin(), out);
  }
  void drop_holder(const Holder* h, std::vector<PoolEntry>* out) {
    for (auto e = lru.begin(); e != lru.end();) {
      auto n = std::next(e);
      if (e->h.get() == h) unlink(e, out);
      e = n;
    }
  }
  void give(std::shared_ptr<Holder> h, size_t cls, void* p) {
    Holder* raw = h.get();
    lru.push_back(PoolEntry{cls, p, std::move(h)});
    by_key[{raw, cls}].push_back(std::prev(lru.end()));
    cached += cls;
    h_cached(raw) += cls;
  }
};

struct DevicePool {
  std::mutex mu;
  PoolSide dev{false}, host{true};
  uint64_t holders = 0;  // live stream holders on the device
  std::vector<std::shared_ptr<Holder>> shared;  // the device's shared streams (psf_context_create own_stream=2)
  size_t next_shared = 0;
  DevicePool() {
    dev.cap = Context::kDefaultCacheBytes;
    host.cap = Context::kDefaultPinnedCacheBytes;
  }
};

constexpr int kMaxDevices = 64;
DevicePool* device_pool(int device) {
  static DevicePool* pools[kMaxDevices];
  static std::mutex mu;
  if (device < 0 || device >= kMaxDevices) throw CheckError(kErrArg, "device index out of range");
  std::lock_guard<std::mutex> l(mu);
  if (!pools[device]) pools[device] = new DevicePool();  // process lifetime
  return pools[device];
}

// free evicted blocks, each after its holder's stream has drained
void free_entries(std::vector<PoolEntry>& ev, bool pinned) {
  if (ev.empty()) return;
  DeviceScope ds(ev.front().h->device, true);
  const Holder* synced = nullptr;
  for (auto& e : ev) {
    if (e.h.get() != synced) {
      (void)hipStreamSynchronize(e.h->stream);
      synced = e.h.get();
    }
    (void)(pinned ? hipHostFree(e.p) : hipFree(e.p));
  }
  ev.clear();  // (drops the holder references after the frees)
}
}  // namespace

void* Holder::get(size_t cls) {
  DevicePool* pool = device_pool(device);
  {
    std::lock_guard<std::mutex> l(pool->mu);
    if (void* p = pool->dev.take(this, cls)) return p;
  }
  void* p = nullptr;
  DeviceScope ds(device);
  hipError_t e = hipMalloc(&p, cls);
  if (e != hipSuccess) {  // out of HBM: drop every cached block of the device, then once more
    (void)hipGetLastError();
    std::vector<PoolEntry> ev;
    {
      std::lock_guard<std::mutex> l(pool->mu);
      const uint64_t c = pool->dev.cap;
      pool->dev.cap = 0;
      pool->dev.make_room(0, &ev);
      pool->dev.cap = c;
    }
    free_entries(ev, false);
    PSF_HIP_CHECK(hipMalloc(&p, cls));
  }
  std::lock_guard<std::mutex> l(pool->mu);
  pool->dev.allocated += cls;
  dev_allocated += cls;
  return p;
}

void* Holder::get_pinned(size_t cls) {
  DevicePool* pool = device_pool(device);
  {
    std::lock_guard<std::mutex> l(pool->mu);
    if (void* p = pool->host.take(this, cls)) return p;
  }
  void* p = nullptr;
  DeviceScope ds(device);
  PSF_HIP_CHECK(hipHostMalloc(&p, cls, hipHostMallocMapped | hipHostMallocCoherent));
  std::lock_guard<std::mutex> l(pool->mu);
  pool->host.allocated += cls;
  host_allocated += cls;
  return p;
}

// (called from Buffer deleters: never throws)
static void release(Holder* h, PoolSide DevicePool::*side, size_t cls, void* p) {
  DevicePool* pool = device_pool(h->device);
  std::vector<PoolEntry> ev;
  PoolSide& s = pool->*side;
  {
    std::lock_guard<std::mutex> l(pool->mu);
    if (h->retired || cls > s.cap) {  // not kept: freed once the stream drains
      s.allocated -= cls;
      ++s.evictions;
      s.h_allocated(h) -= cls;
      ++s.h_evictions(h);
      ev.push_back(PoolEntry{cls, p, h->shared_from_this()});
    } else {
      s.make_room(cls, &ev);
      s.give(h->shared_from_this(), cls, p);
    }
  }
  free_entries(ev, s.pinned);
}
void Holder::put(size_t cls, void* p) { release(this, &DevicePool::dev, cls, p); }
void Holder::put_pinned(size_t cls, void* p) { release(this, &DevicePool::host, cls, p); }

void Holder::retire() {
  DevicePool* pool = device_pool(device);
  std::vector<PoolEntry> ed, eh;
  {
    std::lock_guard<std::mutex> l(pool->mu);
    retired = true;
    pool->dev.drop_holder(this, &ed);
    pool->host.drop_holder(this, &eh);
    --pool->holders;
  }
  free_entries(ed, false);
  free_entries(eh, true);
}

static void set_device_caps(int device, uint64_t dev_cap, uint64_t host_cap) {
  DevicePool* pool = device_pool(device);
  std::vector<PoolEntry> ed, eh;
  {
    std::lock_guard<std::mutex> l(pool->mu);
    pool->dev.cap = dev_cap;
    pool->host.cap = host_cap;
    pool->dev.make_room(0, &ed);
    pool->host.make_room(0, &eh);
  }
  free_entries(ed, false);
  free_entries(eh, true);
}

void Context::set_cache_limit(size_t dev_bytes, size_t pinned_bytes) {
  if (device_ >= 0) set_device_caps(device_, dev_bytes, pinned_bytes);
}
void set_device_cache_limit(int device, uint64_t dev_bytes, uint64_t pinned_bytes) {
  set_device_caps(device, dev_bytes, pinned_bytes);
}

Context::MemoryStats Context::memory_stats() const {
  MemoryStats s;
  if (!holder_) return s;
  DevicePool* pool = device_pool(device_);
  std::lock_guard<std::mutex> l(pool->mu);
  const Holder& h = *holder_;
  s.dev_cached = h.dev_cached;
  s.dev_cap = pool->dev.cap;
  s.dev_allocated = h.dev_allocated;
  s.dev_evictions = h.dev_evictions;
  s.host_cached = h.host_cached;
  s.host_cap = pool->host.cap;
  s.host_allocated = h.host_allocated;
  s.host_evictions = h.host_evictions;
  return s;
}

DeviceMemoryStats device_memory_stats(int device) {
  DeviceMemoryStats s;
  DevicePool* pool = device_pool(device);
  std::lock_guard<std::mutex> l(pool->mu);
  s.m.dev_cached = pool->dev.cached;
  s.m.dev_cap = pool->dev.cap;
  s.m.dev_allocated = pool->dev.allocated;
  s.m.dev_evictions = pool->dev.evictions;
  s.m.host_cached = pool->host.cached;
  s.m.host_cap = pool->host.cap;
  s.m.host_allocated = pool->host.allocated;
  s.m.host_evictions = pool->host.evictions;
  s.holders = pool->holders;
  s.shared_streams = pool->shared.size();
  return s;
}

// uncompress: the control words of kSnappyBatchMax streams (the compressor
// keeps no zeroed state: kZeroCompress is unused)
static constexpr size_t kZeroBytes[Context::kZeroKinds] = {0, 2048};

Context::Context(int device, hipStream_t stream, int mode) : device_(device), stream_(nullptr) {
  if (device < 0) return;  // host-only context: host-resident buffers, no HIP calls
  DeviceScope ds(device);
  DevicePool* pool = device_pool(device);
  if (mode == kStreamShared) {
    // one of the device's kSharedStreams streams, round robin: contexts keep
    // their own order on it, and a process with hundreds of contexts does not
    // alias hundreds of streams onto GPU_MAX_HW_QUEUES hardware queues
    std::lock_guard<std::mutex> l(pool->mu);
    if (pool->shared.size() < (size_t)kSharedStreams) {
      hipStream_t s = nullptr;
      PSF_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      pool->shared.push_back(std::shared_ptr<StreamHolder>(new StreamHolder(device, s, true)));
      ++pool->holders;
    }
    holder_ = pool->shared[pool->next_shared++ % pool->shared.size()];
    stream_ = holder_->stream;
  } else {
    const bool own = mode == kStreamOwn;
    if (own) stream = nullptr;
    if (own) PSF_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    stream_ = stream;
    // constructed in place: a temporary StreamHolder would destroy the stream
    holder_ = std::shared_ptr<StreamHolder>(new StreamHolder(device, stream, own));
    std::lock_guard<std::mutex> l(pool->mu);
    ++pool->holders;
  }
  shared_stream_ = mode == kStreamShared;
  PSF_HIP_CHECK(hipMalloc(&d_partials_, 2 * sizeof(uint64_t) * kMaxGrid));
  PSF_HIP_CHECK(hipMalloc(&zero_base_, 2 * (kZeroBytes[0] + kZeroBytes[1])));
  PSF_HIP_CHECK(hipMemset(zero_base_, 0, 2 * (kZeroBytes[0] + kZeroBytes[1])));
  PSF_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&fused_.ctl), kFusedCtlBytes));
  PSF_HIP_CHECK(hipMemset(fused_.ctl, 0, kFusedCtlBytes));
  PSF_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sticky_h_), 64, hipHostMallocMapped | hipHostMallocCoherent));
  memset(sticky_h_, 0, 64);
  {
    void* d = nullptr;
    PSF_HIP_CHECK(hipHostGetDevicePointer(&d, sticky_h_, 0));
    fused_.sticky = static_cast<int32_t*>(d);
  }
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
  int cur = -1;  // (no DeviceScope: a destructor must not throw)
  (void)hipGetDevice(&cur);
  if (cur != device_) (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  if (side_) {
    (void)hipStreamSynchronize(side_);
    (void)hipStreamDestroy(side_);
  }
  if (side_order_) (void)hipEventDestroy(side_order_);
  for (auto& u : ring_uses_) {  // messages may outlive the context: leave their ranges on the host
    auto rb = u.rb.lock();
    if (rb && !rb->done) {
      memcpy(rb->host.data(), rb->ring, rb->host.size() * 4);
      rb->done = true;
    }
  }
  ring_uses_.clear();
  for (auto& w : dev_records_) {
    auto rb = w.lock();
    if (rb && !rb->done) {
      if (hipMemcpy(rb->host.data(), rb->dev.ptr, rb->host.size() * 4, hipMemcpyDeviceToHost) == hipSuccess)
        rb->done = true;
      rb->ctx = nullptr;
    }
  }
  dev_records_.clear();
  tracked_.clear();
  for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  for (hipEvent_t e : markers_) (void)hipEventDestroy(e);
  (void)hipHostFree(lazy_h_);
  (void)hipFree(d_partials_);
  (void)hipFree(zero_base_);
  (void)hipFree(fused_.ctl);
  if (sticky_h_) (void)hipHostFree(sticky_h_);
  (void)hipFree(d_slots_);
  (void)hipHostFree(h_slots_);
  // a private stream's cached blocks go now (buffers still held by messages
  // are freed when they drop); a shared stream keeps its cache for the
  // device's other contexts
  if (!shared_stream_) holder_->retire();
  holder_.reset();
  if (cur >= 0 && cur != device_) (void)hipSetDevice(cur);
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
  DeviceScope ds(device_);
  PSF_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

void Context::give_event(hipEvent_t e) {
  if (e) events_.push_back(e);
}

hipEvent_t Context::take_marker() {
  if (!markers_.empty()) {
    hipEvent_t e = markers_.back();
    markers_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  DeviceScope ds(device_);
  PSF_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  return e;
}

void Context::give_marker(hipEvent_t e) {
  if (e) markers_.push_back(e);
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

hipStream_t Context::side_stream() {
  if (device_ < 0) throw CheckError(kErrArg, "host-only context has no device stream");
  if (!side_) {
    DeviceScope ds(device_);
    PSF_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  }
  return side_;
}

hipStream_t Context::side_stream_after_main() {
  hipStream_t s = side_stream();
  if (!side_order_) {
    DeviceScope ds(device_);
    PSF_HIP_CHECK(hipEventCreateWithFlags(&side_order_, hipEventDisableTiming));
  }
  PSF_HIP_CHECK(hipEventRecord(side_order_, stream_));
  PSF_HIP_CHECK(hipStreamWaitEvent(s, side_order_, 0));
  return s;
}

void Context::reset_fused() {
  if (fused_.ctl) PSF_HIP_CHECK(hipMemsetAsync(fused_.ctl, 0, kFusedCtlBytes, stream_));
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
      if (q == hipSuccess && side_) q = hipStreamQuery(side_);  // (presign CRCs run there)
      if (q == hipSuccess) {  // streams drained: the publish must be visible now
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
  {
    WaitTimer wt(this, kWaitSync);
    PSF_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  check_sticky();
}

void Context::check_sticky() {
  if (sticky_h_ && __atomic_load_n(sticky_h_, __ATOMIC_ACQUIRE) != 0) handoff_failed();
}

void Context::handoff_failed() {
  // the launch may still be running: let it finish so that every workgroup
  // that gave up has set the sticky word, then take the word and clean the
  // counter lines for the next launch
  (void)hipStreamSynchronize(stream_);
  if (sticky_h_) __atomic_store_n(sticky_h_, 0, __ATOMIC_RELEASE);
  reset_fused();
  throw CheckError(kErrHip, "FIXING_FLOAT: in-launch min/max hand-off timed out");
}

void RangeBatch::resolve(bool synced) {
  if (done) return;
  if (!ctx) {  // its context went first and the records could not be read
    done = true;
    return;
  }
  if (!synced) ctx->sync();  // the kernels' host-mapped stores are visible after it
  if (ring) {
    memcpy(host.data(), ring, host.size() * 4);
  } else {  // records in HBM (received with a spilled slice, spill.cc)
    DeviceScope ds(ctx->device());
    PSF_HIP_CHECK(hipMemcpy(host.data(), dev.ptr, host.size() * 4, hipMemcpyDeviceToHost));
  }
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

void Context::adopt_device_records(const std::shared_ptr<RangeBatch>& rb) {
  if (dev_records_.size() >= 1024) {
    dev_records_.erase(std::remove_if(dev_records_.begin(), dev_records_.end(),
                                      [](const std::weak_ptr<RangeBatch>& w) { return w.expired(); }),
                       dev_records_.end());
  }
  dev_records_.push_back(rb);
}

void Context::track(std::shared_ptr<RangeBatch> rb) {
  tracked_.push_back(std::move(rb));
  if (tracked_.size() >= kMaxTracked) check_ranges();
}

void Context::check_ranges() {
  std::vector<std::shared_ptr<RangeBatch>> t;
  t.swap(tracked_);
  bool bad = false, late = false;
  if (!t.empty()) sync();
  for (auto& rb : t) {
    rb->resolve(true);
    for (size_t i = 2; i < rb->host.size(); i += 4) {
      bad |= (int32_t)rb->host[i] != kOk;
      late |= (int32_t)rb->host[i] == kErrHip;
    }
  }
  if (late) handoff_failed();
  if (bad) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
}

void Context::flush_deferred() {
  if (deferred.arrs.empty()) return;
  const int st = ff_decode_batch_launch(deferred.value_type, deferred.nb, deferred.arrs.data(),
                                        (int)deferred.arrs.size(), stream_, &prof_);
  deferred.clear();
  if (st != kOk) throw CheckError(st, "ff_decode batch launch failed");
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
