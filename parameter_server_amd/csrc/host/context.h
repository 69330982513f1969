// Per-(device, stream) execution context of libpsf: the HIP stream the codec
// kernels are ordered on, stream-ordered HBM allocation for codec outputs, a
// small device workspace (min/max partials, per-array side-info slots) and a
// pinned host mirror of the slots so side-info reaches the FilterConfig with one
// D2H copy + one stream sync per message.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <deque>
#include <memory>
#include <vector>
#include <mutex>
#include <string>
#include <thread>

#include "../psf_internal.h"
#include "message.h"

namespace psf {

#define PSF_HIP_CHECK(expr)                                                         \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      throw ::psf::CheckError(::psf::kErrHip, std::string(#expr) + ": " +            \
                                                  hipGetErrorString(_e));           \
  } while (0)

typedef PubSlot Slot;

// Makes `device` the calling thread's current device for the scope and
// restores the previous one after (no HIP call when it already is current;
// device < 0 = host-only, nothing to do).  hipMalloc, hipEventCreate and the
// per-device kernel tables follow the thread's current device, so every
// libpsf entry that allocates or launches runs inside one.
struct DeviceScope {
  int prev = -1;
  // nothrow: for destructors and deleters (a failure leaves the device as is)
  explicit DeviceScope(int device, bool nothrow = false) {
    if (device < 0) return;
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e == hipSuccess && cur == device) return;
    if (e == hipSuccess) e = hipSetDevice(device);
    if (e == hipSuccess) {
      prev = cur;
    } else if (!nothrow) {
      throw CheckError(kErrHip, std::string("hipSetDevice: ") + hipGetErrorString(e));
    }
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

class Context;
// FIXING_FLOAT side-info of one lazy encode batch: the kernels write
// {min, max, status, 0} (16 bytes) per array into `dev`; resolve() brings
// them to the host with one stream sync when a host reader needs them.
struct RangeBatch {
  Context* ctx = nullptr;
  Buffer dev;                      // read by decodes on ctx's stream
  const uint32_t* ring = nullptr;  // the same records in ctx's host-mapped ring (null: read dev)
  std::vector<uint32_t> host;      // 4 words per array, valid once done
  bool done = false;
  void resolve(bool synced = false);
};

class Context {
 public:
  static constexpr int kSlots = 1280;
  // slots [0, kSyncSlots) serve launches whose results the host waits for
  // before returning; [kSyncSlots, kPresignSlot0) the KEY_CACHING signatures
  // that a batched encode leaves in flight while later filters launch;
  // [kPresignSlot0, kPresignEnd) the round-trip drivers' signatures of the
  // next iteration (presign_launch); [kCompressSlot0, kDecodeSlot0) the
  // COMPRESSING encodes a batched encode leaves in flight for its caller
  // (PendingEncode), [kDecodeSlot0, kSlots) the uncompress launches a batched
  // decode leaves in flight (PendingDecode) -- the router's multi-step driver
  // holds one of each at once.  Every region holds kSyncSlots.
  static constexpr int kSyncSlots = 256;
  static constexpr int kDeferSlot0 = kSyncSlots;
  static constexpr int kPresignSlot0 = 512;
  static constexpr int kPresignEnd = 768;
  static constexpr int kCompressSlot0 = 768;
  static constexpr int kDecodeSlot0 = 1024;

  // mode kStreamOwn -> a private non-blocking stream owned by the context;
  // kStreamGiven -> `stream` as given (nullptr = the legacy default stream);
  // kStreamShared -> one of the device's kSharedStreams process-wide streams.
  // device < 0 -> host-only context (host-resident buffers; no HIP calls).
  enum StreamMode { kStreamGiven = 0, kStreamOwn = 1, kStreamShared = 2 };
  static constexpr int kSharedStreams = 4;  // = GPU_MAX_HW_QUEUES' default
  Context(int device, hipStream_t stream, int mode);
  ~Context();

  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }

  // Lifetime: the C ABI's handle holds one reference, every node, router,
  // exchange and KV map made on the context one more; the context is deleted
  // when the last goes (a binding may destroy them in any order, e.g. a
  // garbage collector finalising a cycle).
  std::atomic<int> refs{1};
  static void ref(Context* c) {
    if (c) c->refs.fetch_add(1, std::memory_order_relaxed);
  }
  static void unref(Context* c) {
    if (c && c->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete c;
  }
  // side-info records a received message's decodes read in HBM (spill.cc):
  // settled to the host if the context goes first
  void adopt_device_records(const std::shared_ptr<RangeBatch>& rb);
  // a second stream of this context for work no kernel of stream() depends
  // on (the round-trip drivers' KEY_CACHING presign CRCs of the next
  // iteration's keys, read back through publish slots), created on first use
  hipStream_t side_stream();
  // side_stream(), ordered after everything queued on stream() so far (one
  // event record + wait): for side work that reads what earlier main-stream
  // work may have written (presign CRCs of keys a decode produced)
  hipStream_t side_stream_after_main();
  // ff_fused_batch's counter lines zeroed on the stream: after an in-launch
  // hand-off gave up, the aborted launch left them dirty (only the last
  // workgroup of an array re-zeroes its line)
  void reset_fused();

  // HBM buffer freed (stream-ordered) when its last reference drops.
  Buffer alloc(size_t bytes);
  // Host-mapped coherent memory (kernel inputs the host fills, results the
  // host reads once an event after the kernel has completed), pooled by size
  // class; returned to the pool when the last reference drops.
  struct Pinned {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    std::shared_ptr<void> owner;
  };
  Pinned pinned(size_t bytes);
  // ZeroPair regions (psf_internal.h) by kind, zeroed at creation; a call
  // whose `need` fits returns {this launch's, the next launch's} and flips the
  // kind's parity, else {} (the launch then memsets its own scratch)
  enum ZeroKind { kZeroCompress = 0, kZeroUncompress, kZeroKinds };
  ZeroPair zero_pair(int kind, size_t need);
  // the launch that took `z` failed before its kernel ran: nothing dirtied
  // z.cur or cleared z.next, so the next launch of the kind takes z.cur again
  void zero_pair_unused(int kind, const ZeroPair& z) {
    if (z.cur) zero_parity_[kind] ^= 1;
  }
  // The caching allocator's bounds (bytes kept on the free lists of the
  // context's DEVICE, shared by every context on it): HBM and pinned host
  // memory.  Defaults below; see context.cc.
  static constexpr size_t kDefaultCacheBytes = size_t(8) << 30;
  static constexpr size_t kDefaultPinnedCacheBytes = size_t(1) << 30;
  void set_cache_limit(size_t dev_bytes, size_t pinned_bytes);
  struct MemoryStats {
    uint64_t dev_cached = 0, dev_cap = 0, dev_allocated = 0, dev_evictions = 0;
    uint64_t host_cached = 0, host_cap = 0, host_allocated = 0, host_evictions = 0;
  };
  MemoryStats memory_stats() const;  // this context's stream's share; caps per device
  // pooled timing-free events
  hipEvent_t take_event();
  void give_event(hipEvent_t e);
  // events the host only polls for completion (no data read through them):
  // recorded without the system-scope fence, which costs the stream about
  // 2 us more per record (tools/event_gap_probe.hip)
  hipEvent_t take_marker();
  void give_marker(hipEvent_t e);

  void* partials() const { return d_partials_; }
  FfFusedCtl* fused() { return fused_.ctl ? &fused_ : nullptr; }  // ff_fused_batch's counters
  Slot* d_slots() const { return d_slots_; }
  // host-mapped, coherent publish slots: kernels write through pub_dev(i),
  // the host reads pub_host(i)
  Slot* pub_dev(int i) const { return m_slots_ + i; }
  Slot* pub_host(int i) const { return h_slots_ + i; }
  uint32_t next_ticket() { return ++ticket_; }
  // Wait until slot i carries `ticket` (spins on host memory; falls back to
  // the stream state so a kernel that never publishes cannot hang the host).
  void wait_ticket(int i, uint32_t ticket);
  // the same for a CRC published with its ticket in one word; returns the CRC
  uint32_t wait_crc(int i, uint32_t ticket);
  void sync();
  // throws kErrHip (once) if a kernel of this context gave up an in-launch
  // hand-off since the last check; sync() calls it after the stream drains
  void check_sticky();
  // an in-launch hand-off gave up: drain the stream, take the sticky word,
  // clean the counters, throw kErrHip
  [[noreturn]] void handoff_failed();
  // spin until `e` has completed; the time is counted as wait `w`
  void wait_event(hipEvent_t e, int w);
  // stage a host buffer into HBM (used at the host edge)
  Buffer to_device(const Buffer& b);
  // NOISE: device table of the reference engine's standard normals, >= n long
  const void* noise_table(int value_type, size_t n);

  // lazy side-info batches not yet checked: check_ranges() resolves them all
  // and reports a CHECK_GT(bin, 0) failure among them (called by sync_checked
  // and by the batched round trip; also once the list reaches kMaxTracked)
  void track(std::shared_ptr<RangeBatch> rb);
  // n consecutive 16-byte records of the host-mapped ring for rb (sets
  // rb->ring; returns their device address).  Records are reused after the
  // ring wraps; a batch still unresolved then is resolved first.
  static constexpr uint64_t kLazyRing = 1u << 15;
  float* claim_lazy(const std::shared_ptr<RangeBatch>& rb, int n);
  void check_ranges();
  // (the ranges first: a sticky hand-off error thrown by sync() must not leave
  // the tracked ranges behind for the next check)
  void sync_checked() { check_ranges(); sync(); }

  std::mutex& mu() { return mu_; }
  Profiler* prof() { return &prof_; }

  // A FIXING_FLOAT decode batch held back (psf_nodes_roundtrip_opts turns
  // this on for its own duration): the next batched encode on the context
  // launches it together with its min/max pass, or flush_deferred() on its
  // own.  `keep` holds the batch's buffers until it is launched (the caching
  // allocator's stream order covers only launched work).
  // `ranges` keeps the RangeBatches the arrays' device {min, max} point into.
  // Deferral is the driver's own: only decodes on the thread that turned it
  // on are held back (defers_here), so another caller of the context never
  // gets a buffer whose decode has not been launched.
  struct DeferredDecode {
    int value_type = 0, nb = 0;
    std::vector<FfDecArray> arrs;
    std::vector<Buffer> keep;
    std::vector<std::shared_ptr<RangeBatch>> ranges;
    void clear() {
      arrs.clear();
      keep.clear();
      ranges.clear();
    }
  };
  void set_defer_decodes(bool on) {
    defer_decodes_ = on && device_ >= 0;
    defer_owner_ = std::this_thread::get_id();
  }
  bool defers_here() const { return defer_decodes_ && defer_owner_ == std::this_thread::get_id(); }
  DeferredDecode deferred;
  void flush_deferred();

  // Host time spent blocked on the device, by cause (psf_context_host_stats):
  // stream synchronisations, waits on a kernel's published side-info, and
  // slice-position read-backs.
  enum HostWait { kWaitSync = 0, kWaitPublish, kWaitSlice, kWaitNum };
  void add_wait(HostWait w, int64_t ns) {
    wait_ns_[w] += ns;
    ++wait_n_[w];
  }
  int64_t wait_ns(int w) const { return wait_ns_[w]; }
  int64_t wait_count(int w) const { return wait_n_[w]; }
  void reset_waits() {
    for (int w = 0; w < kWaitNum; ++w) wait_ns_[w] = wait_n_[w] = 0;
  }

  struct StreamHolder;  // a stream + its share of the device's caching allocator (context.cc)

 private:
  Profiler prof_;
  int64_t wait_ns_[kWaitNum] = {0, 0, 0}, wait_n_[kWaitNum] = {0, 0, 0};
  static constexpr size_t kMaxTracked = 1024;
  std::vector<std::shared_ptr<RangeBatch>> tracked_;
  uint32_t* lazy_h_ = nullptr;  // host view of the ring
  uint32_t* lazy_m_ = nullptr;  // device view
  uint64_t lazy_next_ = 0;      // absolute index of the next record
  struct RingUse {
    std::weak_ptr<RangeBatch> rb;
    uint64_t start, n;
  };
  std::deque<RingUse> ring_uses_;
  std::vector<std::weak_ptr<RangeBatch>> dev_records_;
  int device_;
  bool shared_stream_ = false;
  hipStream_t stream_;
  hipStream_t side_ = nullptr;
  hipEvent_t side_order_ = nullptr;  // side_stream_after_main's event
  bool defer_decodes_ = false;
  std::thread::id defer_owner_;
  std::shared_ptr<StreamHolder> holder_;
  void* d_partials_ = nullptr;
  Slot* d_slots_ = nullptr;
  Slot* h_slots_ = nullptr;
  Slot* m_slots_ = nullptr;
  uint32_t ticket_ = 0;
  std::vector<hipEvent_t> events_;
  std::vector<hipEvent_t> markers_;
  void* zero_base_ = nullptr;
  FfFusedCtl fused_;
  int32_t* sticky_h_ = nullptr;  // fused_.sticky's host side
  int zero_parity_[kZeroKinds] = {0, 0};
  Buffer noise_f32_, noise_f64_;
  std::mutex mu_;
};

// the device-wide view of the caching allocator (psf_device_memory_stats)
struct DeviceMemoryStats {
  Context::MemoryStats m;
  uint64_t holders = 0, shared_streams = 0;
};
DeviceMemoryStats device_memory_stats(int device);
void set_device_cache_limit(int device, uint64_t dev_bytes, uint64_t pinned_bytes);

// monotonic nanoseconds (host waits, router phase timers)
int64_t now_ns();
// adds the time from construction to destruction to ctx's wait counter w
struct WaitTimer {
  Context* ctx;
  Context::HostWait w;
  int64_t t0;
  WaitTimer(Context* c, Context::HostWait which) : ctx(c), w(which), t0(now_ns()) {}
  ~WaitTimer() { ctx->add_wait(w, now_ns() - t0); }
};

// Diagnostic builds (-DPSF_HOST_PROF): host time per code section, read with
// psf_debug_host_prof.  Compiles to nothing otherwise.
#ifdef PSF_HOST_PROF
constexpr int kHProfSlots = 16;
extern int64_t g_hprof_ns[kHProfSlots], g_hprof_n[kHProfSlots];
struct HProf {
  int id;
  int64_t t0;
  explicit HProf(int i) : id(i), t0(now_ns()) {}
  ~HProf() {
    g_hprof_ns[id] += now_ns() - t0;
    ++g_hprof_n[id];
  }
};
#define PSF_HPROF(id) ::psf::HProf _hprof_##id(id)
#else
#define PSF_HPROF(id) \
  do {                \
  } while (0)
#endif

// time(NULL) as the reference's FIXING_FLOAT seed source (fixing_float.h:78),
// with an override hook so parity tests can pin it (psf_set_clock).
int32_t ff_clock_seed();
void set_clock_override(bool enable, int64_t t);

// CRC32C on the host (for KEY_CACHING on host-resident keys).
uint32_t crc32c_host(const void* p, size_t n);

}  // namespace psf
