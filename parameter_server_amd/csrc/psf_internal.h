// Internal declarations shared by the HIP kernels and the C++ host layer of
// libpsf.  The public C ABI is include/psf.h.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stddef.h>
#include <stdint.h>

#include <memory>

namespace psf {

constexpr int kBlock = 256;     // 4 waves of 64
constexpr int kMaxGrid = 2048;  // 256 CUs x 8 workgroups; streaming kernels grid-stride

// status codes (mirrored by PSF_* in include/psf.h)
constexpr int kOk = 0;
constexpr int kErrArg = -1;
constexpr int kErrNbytes = -2;
constexpr int kErrBin = -3;
constexpr int kErrHip = -4;
constexpr int kErrCheck = -5;
constexpr int kErrUnsupported = -6;
constexpr int kErrTimeout = -7;  // reserved (PSF_ERR_TIMEOUT): no kernel waits on another, none returns it
constexpr int kErrHeaderHint = -100;  // internal: a snappy stream's header differs from the size hint

// task.proto DataType values used by the codecs
constexpr int kFloat = 9;
constexpr int kDouble = 10;
constexpr int kChar = 11;

// boolrand LCG, fixing_float.h:18-21
constexpr uint32_t kLcgA = 214013u;
constexpr uint32_t kLcgC = 2531011u;

// status of the most recent launch(es) on this thread
inline int launch_status() { return hipGetLastError() == hipSuccess ? kOk : kErrHip; }

struct FixedPoint {
  int has_min, has_max;
  float min_value, max_value;
};

// Side-info a kernel publishes to host-mapped coherent memory as soon as it is
// known (FIXING_FLOAT min/max + CHECK_GT(bin,0) outcome, KEY_CACHING CRC);
// `ticket` is written last, after the other fields' write-through stores
// have drained, so the host can act on it while the rest of the kernel is
// still streaming.
struct PubSlot {
  float range[2];
  int32_t status;
  uint32_t crc;
  uint32_t ticket;
  uint32_t pad;
  uint64_t size;         // COMPRESSING: stream / output length
  uint64_t crc_ticket;   // KEY_CACHING: ticket << 32 | crc, one store
};

// A slot field written through to host memory (a system-scope store: the
// write bypasses the XCD's L2 whatever the page's caching).
template <typename T>
__device__ __forceinline__ void pub_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The ticket, after the fields this thread wrote with pub_store: draining them
// (vmcnt: their write-through acknowledged) orders them before the ticket's
// store.  No system-scope release: on MI355X that writes back and invalidates
// the XCD's whole L2 (two buffer_wbl2 and a buffer_inv) in the middle of the
// publishing workgroup, whose tiles then finish last.
__device__ __forceinline__ void publish_ticket(PubSlot* s, uint32_t ticket) {
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&s->ticket, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a CRC and its ticket in one 8-byte system-scope store: nothing else needs
// ordering before it, so no fence (a system-scope release writes the whole L2
// back, which 64 signature workgroups would each pay for)
__device__ __forceinline__ void publish_crc(PubSlot* s, uint32_t crc, uint32_t ticket) {
  __hip_atomic_store(&s->crc_ticket, ((uint64_t)ticket << 32) | crc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Kernel launch profiler: HIP events recorded on the launch stream around
// each kernel, plus the kernel's algorithmic HBM bytes.
enum KernelId { kKMinmax = 0, kKEncode, kKDecode, kKCrc, kKNoise, kKSnappyCompress,
                kKSnappyDecompress, kKMatch, kKKvPush, kKKvGet, kKDecodeMinmax, kKFused, kKNum };
class Profiler {
 public:
  ~Profiler();
  bool on(KernelId id) const { return (mask_ >> id) & 1u; }
  // on(id), and this launch is one of every `stride` launches of kernel id
  bool sample(KernelId id) { return on(id) && seen_[id]++ % stride_ == 0; }
  void enable(uint32_t kernel_mask) { mask_ = kernel_mask; }
  void set_stride(uint32_t stride) {
    stride_ = stride ? stride : 1;
    for (auto& s : seen_) s = 0;
  }
  void begin(hipStream_t st);
  // arms g_ext_events for the scope's one launch (psf_launch): the kernel's
  // own dispatch timestamps, no marker packets in the stream
  void begin_ext();
  void end(KernelId id, hipStream_t st, double alg_bytes);
  void collect();  // waits for pending events, accumulates
  void reset();
  long launches[kKNum] = {0};
  double total_ms[kKNum] = {0};
  double bytes[kKNum] = {0};

 private:
  struct Pending { KernelId id; hipEvent_t a, b; double bytes; };
  hipEvent_t take();
  void pool_push(hipEvent_t e);
  uint32_t mask_ = 0;
  uint32_t stride_ = 1;
  uint64_t seen_[kKNum] = {0};
  hipEvent_t cur_ = nullptr, cur_b_ = nullptr;
  Pending* pend_ = nullptr;
  int npend_ = 0, cap_ = 0;
  hipEvent_t* pool_ = nullptr;
  int npool_ = 0, cappool_ = 0;
};

// RAII bracket around one kernel launch
struct ProfScope {
  Profiler* p; KernelId id; hipStream_t st; double bytes;
  // ext: the scope holds exactly one kernel launch, made through psf_launch,
  // which takes its start / stop from the dispatch itself (hipExtLaunchKernel):
  // a marker event pair costs the stream about 4 us per record on MI355X
  // (two barrier packets around the kernel), which a 15 us kernel's step
  // cannot hide (C3: 4.3 us gaps on both sides of the encode, kernel trace)
  ProfScope(Profiler* p_, KernelId id_, hipStream_t st_, double bytes_, bool ext = false)
      : p(p_ && p_->sample(id_) ? p_ : nullptr), id(id_), st(st_), bytes(bytes_) {
    if (p) {
      if (ext) p->begin_ext();
      else p->begin(st);
    }
  }
  ~ProfScope() { if (p) p->end(id, st, bytes); }
};

// hipExtLaunchKernel's start / stop events armed by a ProfScope(ext) for the
// next psf_launch on this thread
struct ExtEvents { hipEvent_t a = nullptr, b = nullptr; };
extern thread_local ExtEvents g_ext_events;

template <typename F, typename... Args>
inline void psf_launch(F kernel, dim3 grid, dim3 block, uint32_t shm, hipStream_t st, Args... args) {
  ExtEvents& e = g_ext_events;
  if (e.a) {
    hipEvent_t a = e.a, b = e.b;
    e.a = e.b = nullptr;
    hipExtLaunchKernelGGL(kernel, grid, block, shm, st, a, b, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shm, st, args...);
  }
}

// ff_codec.hip
double ff_ratio(int nb);
int ff_grid(size_t work_items);
// range_out/status_out: optional device pointers (async API); pub: optional
// host-mapped slot published with `ticket` once min/max/status are known.
int ff_encode_launch(const void* x, size_t n, int value_type, int nb, const FixedPoint& preset,
                     uint32_t seed, void* out, void* partials, float* range_out, int* status_out,
                     hipStream_t st, Profiler* prof = nullptr, PubSlot* pub = nullptr,
                     uint32_t ticket = 0, float* range_host = nullptr);
int ff_decode_launch(const void* code, size_t n, int value_type, int nb, const float* range,
                     float mn, float mx, void* out, hipStream_t st, Profiler* prof = nullptr);
// Batched launches over up to kFfBatchMax arrays of one value type and
// num_bytes (aligned, nb 1..3: ff_batchable); encode publishes each array's
// side-info to pub_base[slot] with its ticket.
constexpr int kFfBatchMax = 512;
struct FfArray {
  const void* x;
  void* out;
  size_t n;
  FixedPoint preset;
  uint32_t seed;
  int slot;
  uint32_t ticket;
  float* range;       // device {min, max, status} for a lazy reader, or null
  float* range_host;  // the same into host-mapped memory, or null
  bool stored = false;  // out is a stored snappy stream (StoredLayout; nb 1 or 2)
};
struct FfDecArray {
  const void* code;
  void* out;
  size_t n;
  float mn, mx;
  const float* range;  // device {min, max} written by the encode, or null (use mn, mx)
};
// A context's state for ff_fused_batch (a small batch's min/max, encode and a
// pending decode in one launch): a 128-byte line of device counters per array
// slot, zero between launches (the kernel zeroes what it used)
constexpr int kFusedArrays = 64;  // = kBatchSmall (ff_codec.hip)
struct FfFusedCtl {
  uint32_t* ctl = nullptr;
  // host-mapped word a workgroup whose hand-off gave up sets to kErrHip
  // (the array's status can only carry workgroup 0's verdict)
  int32_t* sticky = nullptr;
};
constexpr size_t kFusedCtlBytes = 128 * kFusedArrays;
bool ff_batchable(const void* x, const void* out, size_t n, int nb, int value_type, bool encode);
size_t ff_batch_partials_bytes(const FfArray* arrs, int count);
// dec / ndec / dec_nb: a FIXING_FLOAT decode batch of the same value type,
// independent of these arrays, launched together with their min/max pass
// when both fit one small batch (ff_dec_mm_batch), else just before it
// fused: the context's FfFusedCtl (null: min/max and encode in two launches)
int ff_encode_batch_launch(int value_type, int nb, const FfArray* arrs, int count, void* partials,
                           PubSlot* pub_base, hipStream_t st, Profiler* prof, const FfDecArray* dec = nullptr,
                           int ndec = 0, int dec_nb = 0, FfFusedCtl* fused = nullptr);
int ff_decode_batch_launch(int value_type, int nb, const FfDecArray* arrs, int count, hipStream_t st,
                           Profiler* prof);

// crc32c.hip: CRC32C of d[0:n) written to *out (device).  n may be any size.
// When the message fits one workgroup (n <= kCrcSingleBlock) the result is also
// published to `pub` with `ticket`.
constexpr size_t kCrcSingleBlock = 8 * kBlock;
int crc32c_launch(const void* d, size_t n, uint32_t* out, hipStream_t st,
                  Profiler* prof = nullptr, PubSlot* pub = nullptr, uint32_t ticket = 0);
// up to kCrcBatchMax buffers of 1..kCrcSingleBlock bytes, one workgroup each,
// each CRC published to pub[slot[i]] with ticket[i]
constexpr int kCrcBatchMax = 256;  // 5 KiB of kernel arguments
int crc32c_batch_launch(const void* const* d, const uint32_t* n, const int* slot, const uint32_t* ticket,
                        int count, PubSlot* pub, hipStream_t st, Profiler* prof);

// crc32c.hip: the split positions of many sorted key arrays at the same
// number of boundaries, with the CRC32C signature of each slice's first
// min(2048, bytes) key bytes (slice i of message m: keys [pos[i], pos[i+1]))
struct SliceSigParams {
  const uint64_t* desc;    // per message {key pointer, key count}
  const uint64_t* bounds;  // per message nslices + 1 lower_bound targets
  int nslices;
  int nmsg;
  uint64_t* pos;  // per message nslices + 1 positions
  uint32_t* sig;  // per message nslices signatures (0 for an empty slice)
};
int slice_sig_launch(const SliceSigParams& p, int key_bytes, hipStream_t st);

// noise.hip: the standard-normal sequence of add_noise.h's default-seeded
// engine (built once, on the device) and the per-message in-place apply.
size_t noise_scratch_bytes(uint64_t nz);
int noise_build_table(int value_type, void* z, uint64_t nz, void* scratch, size_t scratch_bytes,
                      hipStream_t st, Profiler* prof = nullptr);
int noise_apply_launch(void* v, const void* z, size_t n, int value_type, float mean, float sd,
                       hipStream_t st, Profiler* prof = nullptr);

// snappy.hip: COMPRESSING (snappy 1.1.8 raw format).  `out` holds at least
// snappy_max_compressed(n) bytes; the stream length is published to pub->size.
constexpr uint32_t kSnappyFragOut = 76544;  // >= MaxCompressedLength(64 KiB), 256-aligned

// The snappy 1.1.8 stream of data without matches -- what RawCompress writes
// for incompressible input such as FIXING_FLOAT codes: varint32(n), then per
// 64 KiB fragment one literal (tag + bytes).  A full fragment's tag is the 3
// bytes 0xF4 0xFF 0xFF (EmitLiteral of 65536 bytes), so fragment k's bytes
// start at hdr + 65539 k + 3; the last fragment has its own tag.  FIXING_FLOAT
// writes its codes straight into this layout when COMPRESSING follows
// (Buffer::kLayoutStored), and COMPRESSING leaves a stream whose fragments all
// come out stored where it is (snappy.hip K-place).
constexpr uint32_t kStoredFragBytes = 65536 + 3;
__host__ __device__ __forceinline__ uint32_t snappy_varint_len(uint64_t v) {
  uint32_t n = 1;
  for (; v >= 128; v >>= 7) ++n;
  return n;
}
// EmitLiteral's tag bytes for a literal of len >= 1 bytes
__host__ __device__ __forceinline__ uint32_t snappy_literal_tag_len(uint32_t len) {
  const uint32_t m = len - 1;
  return m < 60 ? 1u : m < 256 ? 2u : m < 65536 ? 3u : m < (1u << 24) ? 4u : 5u;
}
struct StoredLayout {
  uint32_t hdr;     // varint bytes
  uint32_t tl;      // the last fragment's tag bytes
  uint32_t last;    // index of the last fragment
  uint32_t nbytes;  // payload bytes (n < 2^32)
};
__host__ __device__ __forceinline__ StoredLayout stored_layout(uint32_t nbytes) {
  StoredLayout s;
  s.hdr = snappy_varint_len(nbytes);
  s.last = (nbytes - 1) >> 16;
  s.tl = snappy_literal_tag_len(nbytes - (s.last << 16));
  s.nbytes = nbytes;
  return s;
}
// stream bytes of the whole stored stream
__host__ __device__ __forceinline__ uint64_t stored_stream_bytes(const StoredLayout& s) {
  return (uint64_t)s.hdr + (uint64_t)s.last * kStoredFragBytes + s.tl + (s.nbytes - (s.last << 16));
}
// where fragment k's tag starts, and its bytes
__host__ __device__ __forceinline__ uint64_t stored_frag_tag(const StoredLayout& s, uint32_t k) {
  return (uint64_t)s.hdr + (uint64_t)k * kStoredFragBytes;
}
__host__ __device__ __forceinline__ uint64_t stored_frag_data(const StoredLayout& s, uint32_t k) {
  return stored_frag_tag(s, k) + (k == s.last ? s.tl : 3u);
}
// stream position of payload byte b
__host__ __device__ __forceinline__ uint64_t stored_pos(const StoredLayout& s, uint32_t b) {
  return stored_frag_data(s, b >> 16) + (b & 65535u);
}
constexpr int kSkipN = 6 * 64 + 1;  // a skip loop from ip = 1 ends before probe 270
// cum[k]: offset of probe k from the start of a skip loop (skip starts at 32,
// each probe advances by skip>>5 and then skip += skip>>5)
struct SkipCum {
  uint32_t v[kSkipN];
};
constexpr SkipCum make_skip() {
  SkipCum s{};
  uint32_t skip = 32, cum = 0;
  for (int k = 0; k < kSkipN; ++k) {
    s.v[k] = cum;
    const uint32_t step = skip >> 5;
    skip += step;
    cum += step;
  }
  return s;
}
// bytes allocated after a stored stream: the compressor's aligned reads past a
// fragment's end (64), and the room an in-place compressed stream may grow
// into (snappy.hip kShiftMax)
constexpr uint32_t kStoredSlack = 192;
__host__ __device__ __forceinline__ uint64_t stored_alloc_bytes(const StoredLayout& s) {
  return stored_stream_bytes(s) + kStoredSlack;
}

// the stream byte at P, a header / tag byte before fragment k's data
__host__ __device__ __forceinline__ uint8_t stored_prefix_byte(const StoredLayout& s, uint32_t k, uint64_t P) {
  if (P < s.hdr) return (uint8_t)(((s.nbytes >> (7 * P)) & 127u) | (P + 1 < s.hdr ? 128u : 0u));
  const uint32_t i = (uint32_t)(P - stored_frag_tag(s, k));
  const uint32_t m = (k == s.last ? s.nbytes - (k << 16) : 65536u) - 1;
  const uint32_t tl = k == s.last ? s.tl : 3u;
  if (i == 0) return tl == 1 ? (uint8_t)(m << 2) : (uint8_t)((59 + tl - 1) << 2);
  return (uint8_t)(m >> (8 * (i - 1)));
}
size_t snappy_max_compressed(size_t n);
size_t snappy_compress_scratch(size_t n);
int snappy_compress_launch(const void* in, size_t n, void* out, void* scratch, hipStream_t st,
                           Profiler* prof, PubSlot* pub, uint32_t ticket);
// `hdr` = bytes of the varint32 header (parsed on the host), dsize = its value;
// the verdict of RawUncompress (kOk / kErrCheck) is published to pub->status.
size_t snappy_uncompress_scratch(size_t c, size_t dsize);
int snappy_uncompress_launch(const void* in, size_t c, uint32_t hdr, size_t dsize, void* out,
                             void* scratch, hipStream_t st, Profiler* prof, PubSlot* pub,
                             uint32_t ticket);
// Up to kSnappyBatchMax streams in one launch chain (the COMPRESSING arrays of
// a batch of messages); stream i publishes to pub_base[slot_i] with ticket_i.
constexpr int kSnappyBatchMax = 32;
struct SnappyCJob {
  const void* in;
  size_t n;
  void* out;  // snappy_max_compressed(n) bytes
  int slot;
  uint32_t ticket;
  // nonzero: `in` is a StoredLayout stream of n payload bytes (FIXING_FLOAT
  // wrote it): when every fragment comes out stored the stream is left where
  // it is and published with pub->pad = kStoredInPlace (out untouched); else
  // out as usual
  uint32_t stored = 0;
};
constexpr uint32_t kStoredInPlace = 1;
// A pair of device regions of `bytes` each that replaces a launch's memset of
// its small control state: `cur` is zero when the launch starts (the previous
// launch of the same kind cleared it), and the launch clears `next` for the
// one after it.  {} (or a region too small): the launch memsets its scratch.
struct ZeroPair {
  void* cur = nullptr;
  void* next = nullptr;
  size_t bytes = 0;
};
size_t snappy_compress_batch_scratch(const SnappyCJob* jobs, int njobs);
int snappy_compress_batch_launch(const SnappyCJob* jobs, int njobs, void* scratch, hipStream_t st,
                                 Profiler* prof, PubSlot* pub_base);
// FIXING_FLOAT's decode fused into the uncompress (decode_batch, when a
// COMPRESSING array's next decode is FIXING_FLOAT): the stream holds codes of
// nb bytes (1 or 2), and `values` receives dsize / nb dequantised values
// (fixing_float.h:89-101) with the bits ff_decode would give.  `out` still
// receives the codes of any fragment the fast path does not place, so the
// fallback kernels dequantise from there.
struct SnappyDequant {
  void* values = nullptr;        // null: no fused decode
  int nb = 0;
  int value_type = 0;            // kFloat / kDouble
  const float* range = nullptr;  // device {min, max} left by the encode, or null: (mn, mx)
  float mn = 0.f, mx = 0.f;
};
struct SnappyDJob {
  const void* in;
  size_t c;
  uint32_t hdr;
  size_t dsize;
  void* out;
  int slot;
  uint32_t ticket;
  SnappyDequant dq = {};
};
// whether an uncompress of dsize code bytes into `values` can take the fused decode
bool snappy_dequant_ok(const SnappyDequant& dq, size_t dsize);
size_t snappy_uncompress_batch_scratch(const SnappyDJob* jobs, int njobs);
// The kernels after the fast path (window scan / link / index, fragment
// decode, verdict) of one launched batch; they find nothing to do on streams
// the fast path decoded whole, which then published their verdict already.
struct SnappyTail {
  std::shared_ptr<void> jobs;  // the batch's job table (kernel arguments)
  bool pending = false;        // launched fast path, tail not launched yet
};
// tail != null: launch the fast path only and leave the rest in *tail for
// snappy_uncompress_tail_launch -- to be called (before any other uncompress
// launch with a ZeroPair on this stream) unless every stream of the batch has
// published its ticket once the fast path has completed
int snappy_uncompress_batch_launch(const SnappyDJob* jobs, int njobs, void* scratch, hipStream_t st,
                                   Profiler* prof, PubSlot* pub_base, const ZeroPair& z = ZeroPair{},
                                   SnappyTail* tail = nullptr);
int snappy_uncompress_tail_launch(SnappyTail* tail, hipStream_t st);

// spill.hip: gather `n` copies (sorted by chunk0) into one send buffer; copy i
// moves len bytes from src to dst + dst_off and owns chunks
// [chunk0, chunk0 + ceil(len / kSpillChunk)) of the grid
constexpr uint64_t kSpillChunk = 32768;
struct SpillCopy {
  const uint8_t* src;
  uint64_t dst_off;
  uint64_t len;
  uint64_t chunk0;
};
int spill_gather_launch(const SpillCopy* d_copies, int n, uint64_t nchunks, void* dst, hipStream_t st);

// kv_store.hip: server-side consumers.  `code` != null
// makes the source a FIXING_FLOAT code array (nb bytes, range [mn, mx]) that
// is dequantised in-register exactly as ff_decode would.
int ordered_match_launch(const uint64_t* src_key, size_t nsrc, const void* src_val, const void* code,
                         int nb, float mn, float mx, const uint64_t* dst_key, size_t ndst, void* dst_val,
                         int k, int value_type, int op, int64_t* match_scratch,
                         unsigned long long* d_matched, hipStream_t st, Profiler* prof);
size_t kvmap_slot_bytes();
size_t kvmap_stats_bytes();
int kvmap_init_launch(void* table, size_t cap, hipStream_t st);
int kvmap_rehash_launch(const void* from, size_t nfrom, void* to, size_t cap_to, hipStream_t st);
int kvmap_push_launch(void* table, size_t cap, const uint64_t* keys, size_t n, const float* grad,
                      const void* code, int nb, float mn, float mx, float alpha, float beta,
                      int lr_decay, float lambda1, float lambda2, void* stats, hipStream_t st,
                      Profiler* prof);
int kvmap_get_launch(const void* table, size_t cap, const uint64_t* keys, size_t n, float* out,
                     hipStream_t st, Profiler* prof);
// GetValue of many key arrays in one launch: job j looks up keys[0, n) into
// out; `first` = the sum of the earlier jobs' n (jobs in device memory, in
// that order); total = the sum of all n
struct KvGetJob {
  const uint64_t* keys;
  float* out;
  uint64_t first, n;
};
int kvmap_get_batch_launch(const void* table, size_t cap, const KvGetJob* d_jobs, int njobs, uint64_t total,
                           hipStream_t st, Profiler* prof);

}  // namespace psf
