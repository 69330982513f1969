// COMPRESSING on the device: snappy raw compress / uncompress, byte-identical to
// snappy 1.1.8 (the version the reference links; compressing.h:8-37 ->
// SArray::CompressTo / UncompressFrom, shared_array_inl.h:232-255).
//
// Compress.  A snappy stream is varint32(n) followed by the greedy LZ77 parse
// of each 64 KiB input fragment, and every fragment is parsed on its own (fresh
// hash table, no references across fragments).  A wave runs the exact 1.1.8
// parse of a fragment with lane-parallel helpers -- 64 speculative probes of
// the skip heuristic per step (the probe positions do not depend on the data,
// only on where the skip loop started), match extension 64 bytes per step,
// literal bytes copied 64 per step.  Fragments with no match at all (one
// literal: incompressible data) are found first by a probe-only pass that
// reads the input where the skip loop probes; the others are parsed in LDS.
// Fragment offsets come from a per-stream scan of the fragment lengths, and a
// last launch places tags and literals (snappy_parse / _scan / _place;
// no workgroup waits for another).
//
// Uncompress accepts any valid snappy stream (a reference sender's included)
// and reproduces RawUncompress's verdict.  First every output fragment is
// assumed stored as one literal where a 1.1.8 encoder of incompressible data
// puts it, checked and copied (K-spec; such a stream is done there).
// Otherwise tag boundaries are found in parallel: a one-wave linker hops over
// stored fragments (K0); if it meets too many small tags, every 4 KiB window
// of the compressed bytes is parsed speculatively from each of its first 64
// offsets (K1) and one lane links the windows (K2) -- the true chain enters a
// window on one of those chains almost always, and their bookkeeping gives the
// exit and the output count.  K3 re-walks each window from its true entry,
// validates every copy (1 <= offset <= produced) and indexes the tag that
// starts each 64 KiB output fragment.  K4 decodes the output fragments in
// parallel in LDS.  A stream whose tags straddle output fragments or whose
// copies reach into an earlier fragment (never produced by a 1.1.8 encoder,
// but valid) is decoded by one lane instead (K5).
#include "psf_internal.h"

#include <algorithm>
#include <atomic>
#include "ff_dequant.h"

namespace psf {
namespace {

constexpr uint32_t kFrag = 65536;     // snappy kBlockSize
constexpr uint32_t kMaxTable = 16384;  // kMaxHashTableSize
constexpr uint32_t kMul = 0x1e35a7bdu;
__constant__ SkipCum kSkip = make_skip();  // (psf_internal.h)

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t ld32(const uint32_t* s, uint32_t p) {
  return __builtin_amdgcn_alignbyte(s[(p >> 2) + 1], s[p >> 2], p & 3);
}

__device__ __forceinline__ uint32_t hash(uint32_t v, int shift) { return (v * kMul) >> shift; }

// a pointer the caller knows is device memory, as a global-address-space one
// (plain vector loads, not flat ones, which also count against the LDS
// counter and make every LDS wait wait for them)
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gbl(const void* p) {
  return (const __attribute__((address_space(1))) T*)reinterpret_cast<uintptr_t>(p);
}

// K-parse: kParseWaves waves per workgroup parse one fragment each, reading
// the fragment from memory (L1/L2) and keeping only the hash table and the
// skip loop's per-step slot words in LDS: 36 KiB per wave.
constexpr uint32_t kParseWaves = 4;
constexpr uint32_t kMinSlots = 1024;
static_assert((kParseWaves - 1) * kMaxTable * 2 >= kFrag + 16, "a staged fragment fits the other tables");
struct ParseLds {
  uint16_t table[kParseWaves][kMaxTable];  // (one fragment alone is staged in tables 1..3)
  uint32_t minlane[kParseWaves][kMinSlots + 1];  // per hash slot: lowest lane of the step that probed it (+ a spare)
};

// diagnostic builds (-DPSF_DIAG_NOSTORE): the parse emits nothing (timing only)
#ifdef PSF_DIAG_NOSTORE
#define PSF_SINK(lane) ((lane) + 64u)
#else
#define PSF_SINK(lane) (lane)
#endif

template <uint32_t kLanes = 64>
__device__ uint32_t emit_literal(uint8_t* out, uint32_t op, const uint8_t* srcb, uint32_t lit,
                                 uint32_t len, uint32_t lane) {
  lane = PSF_SINK(lane);
  const uint32_t n = len - 1;
  uint32_t hl = 1;
  if (n < 60) {
    if (lane == 0) out[op] = (uint8_t)(n << 2);
  } else {
    const uint32_t count = ((31 - __builtin_clz(n)) >> 3) + 1;
    if (lane == 0) out[op] = (uint8_t)((59 + count) << 2);
    if (lane >= 1 && lane <= count) out[op + lane] = (uint8_t)(n >> (8 * (lane - 1)));
    hl += count;
  }
  // the literal bytes: byte stores up to the first aligned output position,
  // then whole dwords (16-byte chunks for long literals) composed from LDS
  // (ld32 reads unaligned), then the tail.  `out` is 16-byte aligned.
  const uint32_t d0 = op + hl, d1 = d0 + len;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(srcb);
  if (len >= 256) {
    const uint32_t a0 = (d0 + 15) & ~15u, a1 = d1 & ~15u;
    if (lane < a0 - d0) out[d0 + lane] = srcb[lit + lane];
    uint4* o16 = reinterpret_cast<uint4*>(out);
    for (uint32_t j = (a0 >> 4) + lane; j < (a1 >> 4); j += kLanes) {
      const uint32_t q = lit + (16 * j - d0);
      o16[j] = make_uint4(ld32(s32, q), ld32(s32, q + 4), ld32(s32, q + 8), ld32(s32, q + 12));
    }
    if (lane < d1 - a1) out[a1 + lane] = srcb[lit + (a1 - d0) + lane];
    return d1;
  }
  const uint32_t a0 = (d0 + 3) & ~3u, a1 = d1 & ~3u;
  if (a0 >= a1) {
    for (uint32_t i = lane; i < len; i += kLanes) out[d0 + i] = srcb[lit + i];
    return d1;
  }
  if (lane < a0 - d0) out[d0 + lane] = srcb[lit + lane];
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out);
  for (uint32_t j = (a0 >> 2) + lane; j < (a1 >> 2); j += kLanes) o32[j] = ld32(s32, lit + (4 * j - d0));
  if (lane < d1 - a1) out[a1 + lane] = srcb[lit + (a1 - d0) + lane];
  return d1;
}

__device__ __forceinline__ void put_copy2(uint8_t* out, uint32_t op, uint32_t offset, uint32_t len) {
  out[op] = (uint8_t)(2 + ((len - 1) << 2));
  out[op + 1] = (uint8_t)(offset & 0xff);
  out[op + 2] = (uint8_t)(offset >> 8);
}

__device__ uint32_t emit_copy(uint8_t* out, uint32_t op, uint32_t offset, uint32_t len, uint32_t lane) {
  lane = PSF_SINK(lane);
  if (len >= 68) {  // while (len >= 68) { EmitCopyAtMost64(64); len -= 64; }
    const uint32_t q = (len - 68) / 64 + 1;
    for (uint32_t i = lane; i < q; i += 64) put_copy2(out, op + 3 * i, offset, 64);
    op += 3 * q;
    len -= 64 * q;
  }
  if (len > 64) {
    if (lane == 0) put_copy2(out, op, offset, 60);
    op += 3;
    len -= 60;
  }
  if (len < 12 && offset < 2048) {
    if (lane == 0) {
      out[op] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
      out[op + 1] = (uint8_t)(offset & 0xff);
    }
    return op + 2;
  }
  if (lane == 0) put_copy2(out, op, offset, len);
  return op + 3;
}

// number of equal bytes b[s1+i] == b[s2+i] for s2+i < limit
__device__ __forceinline__ uint32_t match_len(const uint8_t* b, uint32_t s1, uint32_t s2, uint32_t limit,
                                              uint32_t lane) {
  uint32_t m = 0;
  for (;;) {
    const uint32_t i = s2 + m + lane;
    const bool ok = i < limit && b[s1 + m + lane] == b[i];
    const uint64_t bad = __ballot(!ok);
    if (bad) return m + (uint32_t)__builtin_ctzll(bad);
    m += 64;
  }
}

// the 16 bytes that start sh bytes into lo:hi (sh is the same in every lane)
__device__ __forceinline__ uint4 funnel16(const uint4& lo, const uint4& hi, uint32_t sh) {
  const uint32_t b = sh & 3;
#define AB(x, y) __builtin_amdgcn_alignbyte(x, y, b)
  switch (sh >> 2) {
    case 0: return make_uint4(AB(lo.y, lo.x), AB(lo.z, lo.y), AB(lo.w, lo.z), AB(hi.x, lo.w));
    case 1: return make_uint4(AB(lo.z, lo.y), AB(lo.w, lo.z), AB(hi.x, lo.w), AB(hi.y, hi.x));
    case 2: return make_uint4(AB(lo.w, lo.z), AB(hi.x, lo.w), AB(hi.y, hi.x), AB(hi.z, hi.y));
    default: return make_uint4(AB(hi.x, lo.w), AB(hi.y, hi.x), AB(hi.z, hi.y), AB(hi.w, hi.z));
  }
#undef AB
}

__device__ __forceinline__ uint4 shfl_down1(const uint4& v) {
  return make_uint4(__shfl_down(v.x, 1, 64), __shfl_down(v.y, 1, 64), __shfl_down(v.z, 1, 64),
                    __shfl_down(v.w, 1, 64));
}

// snappy's literal tag for a literal of len bytes at p (lanes pt 0..4)
__device__ __forceinline__ uint32_t literal_tag(uint8_t* p, uint32_t len, uint32_t pt) {
  const uint32_t m = len - 1;
  if (m < 60) {
    if (pt == 0) p[0] = (uint8_t)(m << 2);
    return 1;
  }
  const uint32_t count = ((31 - __builtin_clz(m)) >> 3) + 1;
  if (pt == 0) p[0] = (uint8_t)((59 + count) << 2);
  if (pt >= 1 && pt <= count) p[pt] = (uint8_t)(m >> (8 * (pt - 1)));
  return 1 + count;
}

// Phase timestamps of the compress kernel (diagnostic builds only,
// -DPSF_SNAPPY_TRACE, tools/snappy_trace.py): per fragment the 100 MHz clock at
// the start of staging (0), after staging (4), after the parse (1), after the
// look-back (2) and after the placement (3), plus the workgroup (5).
#ifdef PSF_SNAPPY_TRACE
constexpr uint32_t kTraceFrags = 1u << 14;
__device__ uint64_t g_snappy_trace[kTraceFrags * 6];
#define PSF_TRACE_T(f, k, t)                                                                \
  do {                                                                                      \
    if (threadIdx.x == (t) && (f) < kTraceFrags) {                                          \
      g_snappy_trace[(f) * 6 + (k)] = __builtin_amdgcn_s_memrealtime();                     \
      if ((k) == 0) g_snappy_trace[(f) * 6 + 5] = blockIdx.x;                               \
    }                                                                                       \
  } while (0)
#else
#define PSF_TRACE_T(f, k, t) \
  do {                       \
  } while (0)
#endif
#define PSF_TRACE(f, k) PSF_TRACE_T(f, k, 0)
#ifdef PSF_SNAPPY_TRACE
__device__ uint64_t g_dfrag_trace[kTraceFrags * 4];
#define PSF_DTRACE(f, k)                                                          \
  do {                                                                            \
    if (threadIdx.x == 0 && (f) < kTraceFrags)                                    \
      g_dfrag_trace[(f) * 4 + (k)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
#else
#define PSF_DTRACE(f, k) \
  do {                   \
  } while (0)
#endif

// K-parse: 12 waves -- a round probes 12 fragments, so 2048 < n <= 3072
// fragments (C5 + COMPRESSING on a key cache miss: 2048 value + 128 key
// fragments) still take one round on 256 CUs; 12 waves of its 162 registers
// fit 3 per SIMD.  Staging a fragment uses the first kStageThreads.
constexpr uint32_t kCThreads = 768;
constexpr uint32_t kStageThreads = 512;
constexpr uint32_t kStageT = 256;    // lanes of the staging waves
constexpr int kPre = (int)(kFrag / 16 / kStageT);  // uint4 per staging lane that cover one fragment
// one fragment's share of a lane as one vector value (an array of uint4 would
// be placed in scratch memory)
typedef uint32_t FragRegs __attribute__((ext_vector_type(4 * kPre)));

// issue the loads of fragment f (16-byte aligned input) into registers
__device__ __forceinline__ void prefetch_frag(const uint8_t* __restrict__ in, size_t n, uint32_t f, FragRegs& pre,
                                              uint32_t st) {
  const size_t start = (size_t)f * kFrag;
  const uint32_t nv = (uint32_t)(min((size_t)kFrag, n - start) >> 4);
  const uint4* g4 = reinterpret_cast<const uint4*>(in + start);
#pragma unroll
  for (int u = 0; u < kPre; ++u) {
    const uint32_t i = u * kStageT + st;
    if (i < nv) {
      const uint4 v = g4[i];
      pre[4 * u] = v.x;
      pre[4 * u + 1] = v.y;
      pre[4 * u + 2] = v.z;
      pre[4 * u + 3] = v.w;
    }
  }
}

// ---- compress: four launches per batch of streams, no device-side waits.
//
// The parse of a 64 KiB fragment reads the table only at the positions it
// probes, and on data without 4-byte matches at those positions (FIXING_FLOAT
// codes, anything incompressible) 1.1.8's skip heuristic probes some 270
// positions and emits the whole fragment as one literal.  So:
//   K-probe  one wave per fragment runs 1.1.8's skip loop exactly, 64 probes
//            per step, reading the input where it probes (no staging) and
//            keeping the inserted positions in a small map in LDS; a
//            fragment whose loop ends without a match is stored (one
//            literal); any other goes on the list for K-parse.
//   K-parse  the full 1.1.8 parse of the listed fragments, in LDS (fragment
//            + 32 KiB hash table, one persistent workgroup per CU, the next
//            fragment prefetched into registers while wave 0 parses); tags to
//            the fragment's scratch slot.
//   K-scan   one workgroup per stream: the stream offset of every fragment
//            (exclusive sum of the fragment lengths), the varint header and
//            the stream length (published to the host).
//   K-place  one workgroup per fragment: its tags from scratch and its final
//            literal (all of a stored fragment) from the input to their place.
// No workgroup ever waits for another: every dependency is a kernel boundary.
// Several streams compress in one launch chain (the COMPRESSING arrays of a
// batch of messages): fragments are numbered across the streams.
struct CJob {
  const uint8_t* in;  // the input; a stored job: the StoredLayout stream FIXING_FLOAT wrote
  uint8_t* dst;
  uint64_t n;
  uint32_t frag0, nfrag, hdr, slot, ticket, stored;  // stored: `in` is a StoredLayout stream
};
struct SnappyCJobs {
  CJob j[kSnappyBatchMax];
  PubSlot* pub;
  uint32_t njobs, nfrag;
  uint64_t* finfo;     // per fragment: op (tag bytes) << 32 | next_emit (start of the final literal)
  uint64_t* offset;    // per fragment: its offset in the stream (K-scan)
  uint32_t* in_place;  // per job (K-scan streams): a PlaceMode
  uint8_t* stash;      // per fragment of a stored job: its first and last kEdge bytes (K-probe)
};
// How K-place treats a stream.  A stored job (FIXING_FLOAT wrote the stored
// layout) whose fragments all come out stored is the result as it stands.  If
// some carry tags and every fragment's new start lies within kShiftMax bytes
// of its stored one (the usual case on codes: a fragment with one 4-byte match
// comes out 2 bytes longer than a literal), the stream is rewritten in place:
// fragments before the first one with tags stay, each later one is moved by
// its own workgroup (tags from scratch, the final literal from where it lies).
// A workgroup's writes reach at most kShiftMax bytes into a neighbour's
// bytes -- the first ones of the next fragment (moved right) or the last ones
// of the previous (moved left) -- so K-probe keeps every stored fragment's
// first and last kEdge bytes, and a moved fragment takes those from there.
// Otherwise the stream is placed into the job's dst.
enum PlaceMode : uint32_t { kPlaceCopy = 0, kPlaceStored = 1, kPlaceShift = 2 };
constexpr uint32_t kEdge = 64;
constexpr uint32_t kStash = 2 * kEdge;  // per fragment: its first kEdge bytes, then its last
#ifdef PSF_NO_PLACE_SHIFT  // A/B builds: every stream with tags placed by the copy
constexpr int64_t kShiftMax = -1;
#else
constexpr int64_t kShiftMax = 64;
#endif
static_assert(kStoredSlack >= 64 + 64 + 8, "the stored stream's room for growth and the stash reads");
// fragment k's input bytes: consecutive 64 KiB blocks, or in a stored job the
// fragment's literal in the StoredLayout stream
__device__ __forceinline__ const uint8_t* frag_src(const CJob& c, uint32_t k) {
  if (!c.stored) return c.in + (size_t)k * kFrag;
  const StoredLayout L = stored_layout((uint32_t)c.n);
  return c.in + stored_frag_data(L, k);
}
__device__ __forceinline__ uint32_t cjob_index(const SnappyCJobs& J, uint32_t g) {
  uint32_t i = 0;
  while (i + 1 < J.njobs && g >= J.j[i + 1].frag0) ++i;
  return i;
}
__device__ __forceinline__ const CJob& cjob_of(const SnappyCJobs& J, uint32_t g) { return J.j[cjob_index(J, g)]; }
__device__ __forceinline__ bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// bytes of the literal tag of a literal of m + 1 bytes, and of the fragment
__device__ __forceinline__ uint32_t lit_tag_len(uint32_t m) { return 1 + (m < 60 ? 0 : ((31 - __builtin_clz(m)) >> 3) + 1); }
__device__ __forceinline__ uint32_t frag_len(uint64_t info, uint32_t len) {
  const uint32_t op = (uint32_t)(info >> 32), ne = (uint32_t)info;
  return op + (ne < len ? lit_tag_len(len - ne - 1) + (len - ne) : 0);
}
__device__ __forceinline__ uint32_t hash_shift(uint32_t len) {
  uint32_t tsize = 256;
  while (tsize < kMaxTable && tsize < len) tsize <<= 1;
  return __builtin_clz(tsize) + 1;  // 32 - log2(tsize)
}

// ---- K-probe
constexpr uint32_t kMapSlots = 1024;  // per wave: every inserted probe (<= 270) as {hash + 1, position, 4 bytes}
constexpr uint32_t kProbeMax = 6 * 64;  // probes a skip loop from ip = 1 can make in 64 KiB (< kSkipN)
// the 4 input bytes at p of a fragment starting at g (any alignment): one
// global_load_dword at the unaligned address -- gfx950 runs in unaligned mode,
// as the stored-layout code stores rely on (round 4 read two aligned dwords
// and shifted; the probe's ~270 scattered loads per fragment are bound by the
// texture unit's cache-line rate, so half the load instructions)
typedef uint32_t __attribute__((aligned(1))) u32u;
__device__ __forceinline__ uint32_t gld32(const uint8_t* g, uint32_t p) {
  return *gbl<u32u>(g + p);
}
// the table entry of hash h: 0 when never inserted (the table's initial 0)
__device__ __forceinline__ uint64_t map_get(const uint64_t* m, uint32_t h) {
  uint32_t s = h & (kMapSlots - 1);
  for (;;) {
    const uint64_t e = m[s];
    if (e == 0 || (uint32_t)(e >> 48) == h + 1) return e;
    s = (s + 1) & (kMapSlots - 1);
  }
}
// (no two lanes of a step insert the same hash)
__device__ __forceinline__ void map_put(uint64_t* m, uint32_t h, uint32_t pos, uint32_t v) {
  const uint64_t e = ((uint64_t)(h + 1) << 48) | ((uint64_t)pos << 32) | v;
  uint32_t s = h & (kMapSlots - 1);
  for (;;) {
    uint64_t cur = m[s];
    if (cur == 0) {
      cur = atomicCAS(reinterpret_cast<unsigned long long*>(&m[s]), 0ull, (unsigned long long)e);
      if (cur == 0) return;
    }
    if ((uint32_t)(cur >> 48) == h + 1) {
      m[s] = e;
      return;
    }
    s = (s + 1) & (kMapSlots - 1);
  }
}

// the probe's fast path: inserts the 4-byte value v into the set m (entries
// 1 << 32 | v); returns whether v was there already
__device__ __forceinline__ bool set_insert(uint64_t* m, uint32_t v) {
  const uint64_t e = (1ull << 32) | v;
  uint32_t s = (v * 0x9E3779B1u) >> 22;
  for (;;) {
    const uint64_t cur = atomicCAS(reinterpret_cast<unsigned long long*>(&m[s]), 0ull, (unsigned long long)e);
    if (cur == 0) return false;
    if (cur == e) return true;
    s = (s + 1) & (kMapSlots - 1);
  }
}

struct ProbeLds {  // the probe phase: per wave, the table as a map and every probe's bytes
  uint64_t map[kCThreads / 64][kMapSlots];
  uint32_t val[kCThreads / 64][kProbeMax];
};
union CompressPhaseLds {
  ParseLds p;
  ProbeLds q;
};

// dst[0, len) = s[0, len) (global to global, any alignment of either) by T
// lanes (tid 0..T-1): lane l of a wave loads the aligned source block under
// destination chunk l of its row of 63 and takes the chunk's second block
// from the next lane; a row's loads are all issued before its stores.
template <uint32_t T>
__device__ void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ s, uint32_t len, uint32_t tid) {
  constexpr int U = 8, W = T / 64;
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const uint32_t head = (uint32_t)(-reinterpret_cast<uintptr_t>(dst) & 15);
  if (head >= len) {
    for (uint32_t i = tid; i < len; i += T) dst[i] = s[i];
    return;
  }
  if (tid < head) dst[tid] = s[tid];
  const uint32_t nc = (len - head) >> 4;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(s + head);
  typedef uint32_t V4 __attribute__((ext_vector_type(4)));
  const auto s16 = gbl<V4>(reinterpret_cast<const void*>(sp & ~(uintptr_t)15));  // global, not flat, loads
  const uint32_t sh = (uint32_t)(sp & 15);
  const uint32_t lim = nc + (sh ? 1u : 0u);  // blocks that hold source bytes
  uint4* d16 = reinterpret_cast<uint4*>(dst + head);
  for (uint32_t c0 = 0; c0 < nc; c0 += U * W * 63) {
    uint4 lo[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + (u * W + wv) * 63 + lane;
      V4 x = {0, 0, 0, 0};
      if (c < lim) x = s16[c];
      lo[u] = make_uint4(x[0], x[1], x[2], x[3]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + (u * W + wv) * 63 + lane;
      const uint4 hi = shfl_down1(lo[u]);
      if (lane < 63 && c < nc) d16[c] = funnel16(lo[u], hi, sh);
    }
  }
  const uint32_t t0 = head + 16 * nc;
  for (uint32_t i = tid; i < len - t0; i += T) dst[t0 + i] = s[t0 + i];
}

// One wave probes one fragment.  From ip = 1 the skip loop's probe positions
// are fixed (1 + kSkip[k]) until it matches, so all of their 4-byte values are
// loaded at once; the candidate a probe compares with is a position an
// earlier probe inserted (its bytes are already here) or the table's initial
// 0 (the fragment's first 4 bytes).  The loop then runs in LDS and registers,
// 64 probes per step, with exactly the full parse's rules: lanes up to the
// first one whose hash an earlier lane of the step also has see the table as
// it was, that lane sees the earlier lane's insert; later lanes wait for the
// next step.  Returns whether the loop ends without a match (one literal).
__device__ __forceinline__ bool probe_stored(const uint8_t* g, uint32_t len, const uint32_t* skip, uint64_t* m, uint32_t* pv,
                             uint32_t lane) {
  if (len < 15) return true;
  const uint32_t shift = hash_shift(len), ip_limit = len - 15, ip = 1;
  // every probe's bytes (probe k is made iff ip + skip[k + 1] <= ip_limit)
  uint32_t pre[kProbeMax / 64], vbits = 0;
#pragma unroll
  for (uint32_t r = 0; r < kProbeMax / 64; ++r) {
    const uint32_t k = r * 64 + lane;
    const bool valid = ip + skip[k + 1] <= ip_limit;
    pre[r] = valid ? gld32(g, ip + skip[k]) : 0;
    vbits |= (valid ? 1u : 0u) << r;
  }
  const uint32_t v_at0 = uni(gld32(g, 0));
  for (uint32_t i = lane; i < kMapSlots; i += 64) m[i] = 0;
#pragma unroll
  for (uint32_t r = 0; r < kProbeMax / 64; ++r) pv[r * 64 + lane] = pre[r];
  // Fast path: a probe matches only a candidate with its own 4 bytes, and
  // every candidate is position 0 or an earlier probe; when the first 4 bytes
  // and all probes' 4 bytes are distinct the loop ends without a match.
  {
    bool dup = false;
    if (lane == 0) set_insert(m, v_at0);
#pragma unroll
    for (uint32_t r = 0; r < kProbeMax / 64; ++r)
      if ((vbits >> r) & 1) dup |= set_insert(m, pre[r]);
    if (!__ballot(dup)) return true;
    for (uint32_t i = lane; i < kMapSlots; i += 64) m[i] = 0;  // the exact loop below
  }
  for (uint32_t kbase = 0;;) {
    const uint32_t k = kbase + lane;
    const uint32_t pos = ip + skip[k];
    const bool valid = ip + skip[k + 1] <= ip_limit;  // else "goto emit_remainder"
    const uint32_t v = valid ? pv[k] : 0;
    const uint32_t h = valid ? hash(v, shift) : 0;
    const uint64_t vm = __ballot(valid);
    uint64_t eq = vm;  // the valid lanes whose hash equals this lane's (14 bits)
#pragma unroll
    for (int b = 0; b < 14; ++b) {
      const bool bit = (h >> b) & 1;
      const uint64_t bm = __ballot(bit);
      eq &= bit ? bm : ~bm;
    }
    const uint32_t first = valid ? (uint32_t)__builtin_ctzll(eq) : lane;
    const uint64_t em = __ballot(valid && first < lane);
    int limit = 63, jc = 64, jm = 0;
    if (em) {
      jc = __builtin_ctzll(em);
      jm = (int)__builtin_amdgcn_readlane(first, jc);
      limit = jc;
    }
    uint32_t cv = v_at0;  // the candidate's 4 bytes
    if (valid && (int)lane <= limit) {
      const uint64_t e = map_get(m, h);
      if (e) cv = (uint32_t)e;
    }
    const uint32_t vjm = __builtin_amdgcn_readlane(v, jm & 63);
    if (em && (int)lane == jc) cv = vjm;  // lane jm's insert
    if (__ballot(valid && (int)lane <= limit && v == cv)) return false;  // a match
    // no match up to `limit`: every probe up to it inserts its position
    // (jm's insert is overwritten by jc's, same hash)
    if (valid && (int)lane <= limit && !(em && (int)lane == jm)) map_put(m, h, pos, v);
    const uint64_t lim_mask = limit >= 63 ? ~0ull : ((1ull << (limit + 1)) - 1);
    if ((vm & lim_mask) != lim_mask) return true;  // emit_remainder: one literal
    kbase += (uint32_t)limit + 1;
  }
}

// The 4 bytes at p of the fragment g[0, len) (len >= 15), without reading a
// dword that holds no byte of g[0, len): past len - 4 the word is the last
// one shifted right (its low byte is still the byte at p); p >= len reads as
// len - 1.
__device__ __forceinline__ uint32_t gw32(const uint8_t* g, uint32_t p, uint32_t len) {
  p = p < len ? p : len - 1;
  const uint32_t q = p < len - 4 ? p : len - 4;
  return gld32(g, q) >> (8 * (p - q));
}
__device__ __forceinline__ uint32_t lane_of(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
// the same from a fragment staged in LDS (16 zero bytes after it)
__device__ __forceinline__ uint32_t ldc(const uint32_t* s, uint32_t p, uint32_t len) {
  return ld32(s, p < len ? p : len);
}
// the parse's source: the fragment in memory (g) or staged in LDS (s)
template <bool kLds>
__device__ __forceinline__ uint32_t srcw(const uint8_t* g, const uint32_t* s, uint32_t p, uint32_t len) {
  return kLds ? ldc(s, p, len) : gw32(g, p, len);
}

// The literal g[lit, lit + len) at op: for len <= 60 one tag byte (lane 0)
// and the bytes (lanes 1..len), one store instruction; else the tag and a
// wave copy.
// kDefer: the staged single-fragment parse hands literals longer than
// kDeferMin to the whole workgroup (defer[0] entries of {out offset of the
// bytes, lit, len} after it), copied from the fragment in memory after the
// parse, instead of one wave's 16-byte stores; a full list falls back to them.
constexpr uint32_t kDeferMax = 8, kDeferMin = 1024;
template <bool kLds>
__device__ __forceinline__ uint32_t emit_lit(uint8_t* out, uint32_t op, const uint8_t* g, const uint32_t* s,
                                             uint32_t glen, uint32_t lit, uint32_t len, uint32_t lane,
                                             uint32_t* defer = nullptr) {
  if (len <= 60) {
    uint32_t i = lit + (lane ? lane - 1 : 0);
    i = i < glen ? i : glen - 1;
    const uint8_t b = kLds ? reinterpret_cast<const uint8_t*>(s)[i] : gbl<uint8_t>(g)[i];
    lane = PSF_SINK(lane);
    if (lane <= len) out[op + lane] = lane ? b : (uint8_t)((len - 1) << 2);
    return op + 1 + len;
  }
  // a staged fragment: 16-byte stores composed from LDS (a wave issues them
  // back to back); from memory: the wave copy (loads before stores)
  if (kLds && defer && len >= kDeferMin && defer[0] < kDeferMax) {
    const uint32_t hl = literal_tag(out + op, len, PSF_SINK(lane));
    const uint32_t n = defer[0];
    if (lane == 0) {
      defer[1 + 3 * n] = op + hl;
      defer[2 + 3 * n] = lit;
      defer[3 + 3 * n] = len;
      defer[0] = n + 1;
    }
    return op + hl + len;
  }
  if (kLds) return emit_literal(out, op, reinterpret_cast<const uint8_t*>(s), lit, len, lane);
  const uint32_t hl = literal_tag(out + op, len, PSF_SINK(lane));
#ifndef PSF_DIAG_NOSTORE
  copy_bytes<64>(out + op + hl, g + lit, len, lane);
#endif
  return op + hl + len;
}
// The literal of len <= 4 bytes that starts where a copy ended, whose bytes
// are the low ones of cur (the 4 bytes there, already in a register): no
// load on the parse's chain before the store (emit_lit would read them back
// from the fragment first, and the store waits for that read)
__device__ __forceinline__ uint32_t emit_short_lit(uint8_t* out, uint32_t op, uint32_t cur, uint32_t len,
                                                   uint32_t lane) {
  const uint8_t b = lane ? (uint8_t)(cur >> (8 * ((lane - 1) & 3))) : (uint8_t)((len - 1) << 2);
  lane = PSF_SINK(lane);
  if (lane <= len) out[op + lane] = b;
  return op + 1 + len;
}
// EmitCopy (1.1.8) of a copy that fits one tag, one store instruction; the
// rest go to emit_copy
__device__ __forceinline__ uint32_t emit_copy_fast(uint8_t* out, uint32_t op, uint32_t offset, uint32_t len,
                                                   uint32_t lane) {
  if (len < 12 && offset < 2048) {  // COPY_1_BYTE_OFFSET
    const uint8_t b = lane ? (uint8_t)offset : (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
    lane = PSF_SINK(lane);
    if (lane < 2) out[op + lane] = b;
    return op + 2;
  }
  if (len <= 64) {  // COPY_2_BYTE_OFFSET
    const uint8_t b = lane ? (uint8_t)(offset >> (8 * (lane - 1))) : (uint8_t)(2 + ((len - 1) << 2));
    lane = PSF_SINK(lane);
    if (lane < 3) out[op + lane] = b;
    return op + 3;
  }
  return emit_copy(out, op, offset, len, lane);
}

#ifdef PSF_DIAG_COUNT
#define PSF_CNT(i) (cnt[i] += 1)
#else
#define PSF_CNT(i) ((void)0)
#endif

// The exact 1.1.8 parse of one fragment g[0, len) by one wave (CompressFragment,
// snappy.cc): tags to out, returns {tag bytes, start of the final literal}.
// The fragment is read from memory (what the probe touched is in L1 / L2); the
// hash table and the skip loop's slot words are the wave's own LDS.  One wave
// issues about one vector instruction per 4 cycles, so the parse is bound by
// its instruction count and its dependent reads per tag; the common paths are
// short:
//  * copies: each lane holds the 4 bytes at ip + off + lane and at
//    cand + off + lane, so one round of reads gives 64 bytes of the match
//    length, and the bytes at the new ip - 1, ip and ip + 1 come from the
//    lanes where the match ended;
//  * after a copy, the table updates, the check whether ip matches at once
//    and the skip loop's first probe (at ip + 1, which sees those updates)
//    are issued together, with the first round of the next copy's match
//    length for both outcomes;
//  * otherwise the skip loop runs 64 probes per step (positions ip + kSkip[k];
//    the first two steps' offsets sit in registers), every probe's hash slot,
//    candidate and the slot's lowest probing lane read together; a lane whose
//    earlier same-hash lane inserted this step compares with that lane's
//    bytes; lanes past the first lane with an earlier lane in its slot wait
//    for the next step (as in probe_stored).
template <bool kLds>
__device__ __forceinline__ uint2 parse_fragment(uint16_t* __restrict__ table, uint32_t* __restrict__ minlane,
                                                const uint32_t* skip, uint32_t skA, uint32_t skB, uint32_t skC,
                                                const uint8_t* __restrict__ g, const uint32_t* s, uint32_t len,
                                                uint8_t* __restrict__ out, uint32_t lane, uint32_t* defer
#ifdef PSF_DIAG_COUNT
                                                , uint32_t* cnt
#endif
) {
  uint32_t op = 0, next_emit = 0;
  if (len < 15) return make_uint2(0, 0);
  const uint32_t shift = hash_shift(len), ip_limit = len - 15;
  uint32_t ip = 1, kbase = 0;  // the skip loop from ip, at its probe kbase
  for (;;) {
    // ---- skip loop steps (loading the next step's probe bytes ahead
    // measured slower: 16.6 against 15.9 ms for 128 MiB of sorted keys)
    uint32_t cand;
    for (;;) {
      PSF_CNT(0);
      const uint32_t k = kbase + lane;
      const uint32_t o0 = kbase == 0 ? skA : kbase == 1 ? skB : kbase == 2 ? skC : skip[k];
      const uint32_t o1 = kbase == 0 ? skB : kbase == 1 ? skC : skip[k + 1];
      const bool valid = ip + o1 <= ip_limit;  // else "goto emit_remainder"
      const uint32_t pos = ip + o0;
      const uint32_t v = srcw<kLds>(g, s, pos, len);
      const uint32_t h = hash(v, shift);
      const uint32_t slot = valid ? (h & (kMinSlots - 1)) : kMinSlots;  // invalid lanes: the spare slot
      const uint32_t c = table[h];
      atomicMin(&minlane[slot], lane);
      asm volatile("" ::: "memory");
      const uint32_t fl = minlane[slot];
      asm volatile("" ::: "memory");
      minlane[slot] = 0xffffffffu;  // clean for the next step
      const uint32_t wc = srcw<kLds>(g, s, c, len);
      const uint32_t first = valid ? fl : lane;
      const uint64_t vm = __ballot(valid);
      const uint64_t em = __ballot(valid && first < lane);
      int limit = 63, jc = 64, jm = 0;
      bool exact_pair = false;
      if (em) {
        jc = __builtin_ctzll(em);
        jm = (int)lane_of(first, jc);
        exact_pair = lane_of(h, jm) == lane_of(h, jc);
        limit = jc;
      }
      const uint32_t vjm = lane_of(v, jm);
      const bool pair = exact_pair && (int)lane == jc;  // sees lane jm's insert: compares with its bytes
      const bool m = valid && (int)lane <= limit && v == (pair ? vjm : wc);
      const uint64_t mm = __ballot(m);
      const int last = mm ? __builtin_ctzll(mm) : limit;
      const bool overwritten = exact_pair && (int)lane == jm && jc <= last;
      if (valid && (int)lane <= last && !overwritten) table[h] = (uint16_t)pos;
      if (mm) {
        const int ks = __builtin_ctzll(mm);
        cand = (exact_pair && ks == jc) ? lane_of(pos, jm) : lane_of(c, ks);
        ip = lane_of(pos, ks);
        break;
      }
      const uint64_t lim_mask = limit >= 63 ? ~0ull : ((1ull << (limit + 1)) - 1);
      if ((vm & lim_mask) != lim_mask) goto remainder;
      kbase += (uint32_t)limit + 1;
    }
    op = emit_lit<kLds>(out, op, g, s, len, next_emit, ip - next_emit, lane, defer);
    // ---- copies
    {
      uint32_t off = 3, wa = 0, wb = 0;  // lane 0 of the first round: byte ip + 3 (known equal)
      bool have = false;
      for (;;) {
        uint32_t k;
        for (;;) {
          const uint32_t pb = ip + off + lane;
          if (!have) {
            wb = srcw<kLds>(g, s, pb, len);
            wa = srcw<kLds>(g, s, cand + off + lane, len);
          }
          have = false;
          const uint64_t bad = __ballot(pb >= len || ((wa ^ wb) & 0xffu) != 0);
          if (bad) {
            k = (uint32_t)__builtin_ctzll(bad);  // >= 1: lane 0 is a byte known equal
            break;
          }
          off += 63;  // the next round's lane 0 is this round's lane 63
          PSF_CNT(1);
        }
        const uint32_t prev = lane_of(wb, k - 1), cur = lane_of(wb, k);
        uint32_t nxt = lane_of(wb, k < 63 ? k + 1 : 63);
        uint32_t nxt2 = lane_of(wb, k < 62 ? k + 2 : 63);
        op = emit_copy_fast(out, op, ip - cand, off + k, lane);
        ip += off + k;
        next_emit = ip;
        if (ip >= ip_limit) goto remainder;
        PSF_CNT(2);
        if (k == 63) nxt = uni(srcw<kLds>(g, s, ip + 1, len));
        if (k >= 62) nxt2 = uni(srcw<kLds>(g, s, ip + 2, len));
        const uint32_t hp = hash(prev, shift), hc = hash(cur, shift), hn = hash(nxt, shift), h2 = hash(nxt2, shift);
        if (lane == 0) table[hp] = (uint16_t)(ip - 1);
        const uint32_t c = table[hc];
        if (lane == 0) table[hc] = (uint16_t)ip;
        const uint32_t c1 = table[hn];  // the skip loop's probe 0 at ip + 1, if ip does not match
        const uint32_t c2 = table[h2];  // its probe 1 at ip + 2 (probe 0's insert aside)
        wb = srcw<kLds>(g, s, ip + lane, len);
        const uint32_t wb1 = srcw<kLds>(g, s, ip + 1 + lane, len);
        const uint32_t wb2 = srcw<kLds>(g, s, ip + 2 + lane, len);
        wa = srcw<kLds>(g, s, c + lane, len);
        const uint32_t wa1 = srcw<kLds>(g, s, c1 + lane, len);
        const uint32_t wa2 = srcw<kLds>(g, s, c2 + lane, len);
        if (lane_of(wa, 0) == cur) {  // a copy from ip at once; its first round is loaded
          PSF_CNT(3);
          cand = uni(c);
          off = 0;
          have = true;
          continue;
        }
        ip += 1;  // the skip loop from ip + 1: probe 0 is made iff ip + 1 <= ip_limit
        if (ip + 1 > ip_limit) goto remainder;
        if (lane == 0) table[hn] = (uint16_t)ip;
        if (lane_of(wa1, 0) == nxt) {  // probe 0 matches: a one-byte literal, then a copy
          PSF_CNT(4);
          cand = uni(c1);
          op = emit_short_lit(out, op, cur, 1, lane);
          wa = wa1;
          wb = wb1;
          off = 0;
          have = true;
          continue;
        }
        // probe 1 at ip + 1, made iff ip + 2 <= ip_limit; it sees probe 0's
        // insert when the hashes agree (its candidate then ip, whose bytes
        // are nxt).  On sorted keys nearly every skip loop after a copy ends
        // here (tools/bench_snappy.py --only sorted_keys_1e9 with
        // -DPSF_DIAG_COUNT: 6346 of 6395 skip steps per fragment matched at
        // probe 1), so the 64-probe step is skipped.
        if (ip + 2 > ip_limit) goto remainder;
        {
          const bool same = h2 == hn;
          const uint32_t c2v = same ? ip : c2;
          if (lane == 0) table[h2] = (uint16_t)(ip + 1);
          if ((same ? nxt : lane_of(wa2, 0)) == nxt2) {  // a two-byte literal, then a copy
            PSF_CNT(5);
            cand = uni(c2v);
            op = emit_short_lit(out, op, cur, 2, lane);
            ip += 1;
            wa = same ? wb1 : wa2;
            wb = wb2;
            off = 0;
            have = true;
            continue;
          }
        }
        kbase = 2;
        break;
      }
    }
  }
remainder:
  return make_uint2(op, next_emit);
}

// LDS src[0, len) = g[0, len) (g 16-byte aligned) by T lanes: a full
// fragment's loads are all issued before its LDS stores (one memory latency
// per fragment instead of one per T x 16 bytes: 12 -> 2 us for 512 lanes);
// the lane's share is one vector value (an array of uint4 would live in
// scratch memory)
template <uint32_t T>
__device__ __forceinline__ void stage_frag(const uint8_t* __restrict__ g, uint32_t len, uint32_t* src, uint32_t tid) {
  constexpr uint32_t U = kFrag / 16 / T;
  typedef uint32_t Share __attribute__((ext_vector_type(4 * U)));
  const uint4* g4 = reinterpret_cast<const uint4*>(g);
  uint4* s4 = reinterpret_cast<uint4*>(src);
  if (len == kFrag) {
    Share v;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint4 x = g4[u * T + tid];
      v[4 * u] = x.x;
      v[4 * u + 1] = x.y;
      v[4 * u + 2] = x.z;
      v[4 * u + 3] = x.w;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) s4[u * T + tid] = make_uint4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
    return;
  }
  const uint32_t nv = len >> 4;
  for (uint32_t i = tid; i < nv; i += T) s4[i] = g4[i];
  uint8_t* srcb = reinterpret_cast<uint8_t*>(src);
  if (tid < len - (nv << 4)) srcb[(nv << 4) + tid] = g[(nv << 4) + tid];
}

// the same for a fragment at any alignment (a stored job's literal sits at
// hdr + 65539 k + 3): each lane composes its 16-byte LDS blocks from two
// aligned source blocks (the stored stream is allocated with 64 bytes to
// spare); bytes past len are zero
template <uint32_t T>
__device__ __forceinline__ void stage_frag_shifted(const uint8_t* __restrict__ g, uint32_t len, uint32_t* src,
                                                   uint32_t tid) {
  typedef uint32_t V4 __attribute__((ext_vector_type(4)));
  const uintptr_t a = reinterpret_cast<uintptr_t>(g);
  const uint32_t sh = (uint32_t)(a & 15);
  const auto s16 = gbl<V4>(reinterpret_cast<const void*>(a & ~(uintptr_t)15));
  uint4* d4 = reinterpret_cast<uint4*>(src);
  const uint32_t nb = (len + 15) >> 4;
  constexpr uint32_t U = kFrag / 16 / T;
  for (uint32_t i0 = 0; i0 < nb; i0 += U * T) {
    V4 lo[U], hi[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * T + tid;
      if (i < nb) {
        lo[u] = s16[i];
        hi[u] = s16[i + 1];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * T + tid;
      if (i >= nb) continue;
      uint4 w = funnel16(make_uint4(lo[u][0], lo[u][1], lo[u][2], lo[u][3]),
                         make_uint4(hi[u][0], hi[u][1], hi[u][2], hi[u][3]), sh);
      if (16 * i + 16 > len) {  // the block holding the end: zero past len
        const uint32_t keep = len - 16 * i;  // 1..15
        uint32_t* wp = reinterpret_cast<uint32_t*>(&w);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          const uint32_t kb = keep > 4 * q ? (keep - 4 * q < 4 ? keep - 4 * q : 4) : 0;
          wp[q] &= kb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * kb)) - 1u);
        }
      }
      d4[i] = w;
    }
  }
}

// K-parse: persistent workgroups of 12 waves, each over its stripe of the
// fragments (b, b + G, b + 2G, ...) in rounds of 12: every wave probes one
// fragment; then the fragments that matched are parsed by waves
// 0..kParseWaves-1, one fragment per wave at a time (tags to the fragment's
// scratch slot).  No workgroup depends on another.
__global__ __launch_bounds__(kCThreads) void snappy_parse(const SnappyCJobs J, uint8_t* __restrict__ scratch) {
  __shared__ uint32_t skip[kSkipN + 3];
  __shared__ CompressPhaseLds U;
  __shared__ uint32_t s_need[kCThreads / 64];
  __shared__ uint32_t s_defer[1 + 3 * kDeferMax];
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = tid >> 6, lane = tid & 63;
  constexpr uint32_t W = kCThreads / 64;
  for (uint32_t i = tid; i < (uint32_t)kSkipN; i += kCThreads) skip[i] = kSkip.v[i];
  const uint32_t sk0 = kSkip.v[lane], sk1 = kSkip.v[lane + 1], sk2 = kSkip.v[lane + 2];  // the first skip steps' offsets
#ifdef PSF_DIAG_COUNT
  uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  __syncthreads();
  const uint32_t G = gridDim.x;
  for (uint32_t r0 = 0; (size_t)r0 * G + blockIdx.x < J.nfrag; r0 += W) {
    // ---- probe: wave w takes fragment (r0 + w) G + b
    {
      const uint32_t f = (r0 + wave) * G + blockIdx.x;
      bool need = false;
      if (f < J.nfrag) {
        PSF_TRACE_T(f, 0, wave * 64);
        const CJob& c = cjob_of(J, f);
        const size_t start = (size_t)(f - c.frag0) * kFrag;
        const uint32_t len = (uint32_t)min((size_t)kFrag, c.n - start);
        const uint8_t* g = frag_src(c, f - c.frag0);
        // a stored job's fragment may be moved in place by K-place, whose
        // neighbours can overwrite its first or last bytes before it reads
        // them: keep them (reads past a short last fragment stay inside the
        // stream's kStoredSlack)
        if (c.stored && (lane < kEdge / 4 || (lane < kStash / 4 && len >= kEdge))) {
          const uint32_t p = lane < kEdge / 4 ? 4 * lane : len - kStash + 4 * lane;
          reinterpret_cast<uint32_t*>(J.stash + (size_t)f * kStash)[lane] = gld32(g, p);
        }
        need = !probe_stored(g, len, skip, U.q.map[wave], U.q.val[wave], lane);
        if (!need && lane == 0) J.finfo[f] = 0;  // no tags, the final literal from byte 0
        PSF_TRACE_T(f, 4, wave * 64);
      }
      if (lane == 0) s_need[wave] = need;
    }
    __syncthreads();
    uint32_t need = 0;
    for (uint32_t w = 0; w < W; ++w) need |= s_need[w] << w;
    __syncthreads();  // (the probe maps are overwritten by the parses)
    if (!need) continue;
    // ---- parse.  One fragment (data with few matches: a fragment of
    // FIXING_FLOAT codes now and then): staged in LDS where the other
    // tables would be and parsed there by wave 0.  More: wave p < kParseWaves
    // takes the matched fragments p, p + kParseWaves, ... from memory.
    if (wave < kParseWaves)
      for (uint32_t i = lane; i <= kMinSlots; i += 64) U.p.minlane[wave][i] = 0xffffffffu;  // each step cleans up after itself
    if (__builtin_popcount(need) == 1) {
      const uint32_t f = (r0 + __builtin_ctz(need)) * G + blockIdx.x;
      if (tid == 0) s_defer[0] = 0;
      const CJob& c = cjob_of(J, f);
      const size_t start = (size_t)(f - c.frag0) * kFrag;
      const uint32_t len = (uint32_t)min((size_t)kFrag, c.n - start);
      const uint8_t* g = frag_src(c, f - c.frag0);
      uint32_t* src = reinterpret_cast<uint32_t*>(U.p.table[1]);  // tables 1..3: 96 KiB
      uint8_t* srcb = reinterpret_cast<uint8_t*>(src);
      if (aligned16(g)) {
        if (tid < kStageThreads) stage_frag<kStageThreads>(g, len, src, tid);
      } else if (c.stored) {
        if (tid < kStageThreads) stage_frag_shifted<kStageThreads>(g, len, src, tid);
      } else {
        for (uint32_t i = tid; i < len; i += kCThreads) srcb[i] = g[i];
      }
      if (tid < 16) srcb[len + tid] = 0;
      uint4* t16 = reinterpret_cast<uint4*>(U.p.table[0]);
      for (uint32_t j = tid; j < (1u << (32 - hash_shift(len))) / 8; j += kCThreads) t16[j] = make_uint4(0, 0, 0, 0);
      __syncthreads();
      if (wave == 0) {
        const uint2 r = parse_fragment<true>(U.p.table[0], U.p.minlane[0], skip, sk0, sk1, sk2, g, src, len,
                                             scratch + (size_t)f * kSnappyFragOut, lane, s_defer
#ifdef PSF_DIAG_COUNT
                                             , cnt
#endif
        );
        if (lane == 0) J.finfo[f] = ((uint64_t)r.x << 32) | r.y;
        PSF_TRACE(f, 1);
      }
    } else if (wave < kParseWaves) {
      uint16_t* table = U.p.table[wave];
      uint32_t* minlane = U.p.minlane[wave];
      uint32_t m = need;
      for (uint32_t i = 0; m; ++i) {
        const uint32_t w = __builtin_ctz(m);
        m &= m - 1;
        if (i % kParseWaves != wave) continue;
        const uint32_t f = (r0 + w) * G + blockIdx.x;
        const CJob& c = cjob_of(J, f);
        const size_t start = (size_t)(f - c.frag0) * kFrag;
        const uint32_t len = (uint32_t)min((size_t)kFrag, c.n - start);
        uint4* t16 = reinterpret_cast<uint4*>(table);
        for (uint32_t j = lane; j < (1u << (32 - hash_shift(len))) / 8; j += 64) t16[j] = make_uint4(0, 0, 0, 0);
        asm volatile("" ::: "memory");
        const uint2 r = parse_fragment<false>(table, minlane, skip, sk0, sk1, sk2, frag_src(c, f - c.frag0), nullptr, len,
                                              scratch + (size_t)f * kSnappyFragOut, lane, nullptr
#ifdef PSF_DIAG_COUNT
                                              , cnt
#endif
        );
        if (lane == 0) J.finfo[f] = ((uint64_t)r.x << 32) | r.y;
        PSF_TRACE_T(f, 1, wave * 64);
      }
    }
    __syncthreads();  // (the next round's probe maps overwrite the tables)
    if (__builtin_popcount(need) == 1 && s_defer[0]) {  // the long literals it handed over
      const uint32_t f = (r0 + __builtin_ctz(need)) * G + blockIdx.x;
      const CJob& c = cjob_of(J, f);
      const uint8_t* g = frag_src(c, f - c.frag0);
      uint8_t* out = scratch + (size_t)f * kSnappyFragOut;
      for (uint32_t d = 0; d < s_defer[0]; ++d)
        copy_bytes<kCThreads>(out + s_defer[1 + 3 * d], g + s_defer[2 + 3 * d], s_defer[3 + 3 * d], tid);
      __syncthreads();  // (s_defer is reset by the next single parse)
    }
  }
#ifdef PSF_DIAG_COUNT
  if (blockIdx.x == 0 && lane == 0 && wave < kParseWaves)
    printf("parse counts wg0 wave %u: steps %u ext_rounds %u copies %u immediate %u probe0 %u probe1 %u\n", wave,
           cnt[0], cnt[1], cnt[2], cnt[3], cnt[4], cnt[5]);
#endif
}

// ---- K-scan: one workgroup per stream.  Fragment offsets = the varint
// header + the exclusive sum of the fragment lengths; the stream length is
// published to the host (the bytes are in place once K-place has run).
constexpr uint32_t kScanT = 1024;
// how far fragment k's new start lies after its stored one (a stored job)
__device__ __forceinline__ int64_t stored_shift(const CJob& c, uint32_t k, uint64_t off) {
  return (int64_t)off - (int64_t)stored_frag_tag(stored_layout((uint32_t)c.n), k);
}
__global__ __launch_bounds__(kScanT) void snappy_scan(const SnappyCJobs J) {
  __shared__ uint64_t wsum[kScanT / 64];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_any;
  __shared__ int64_t s_lo[kScanT / 64], s_hi[kScanT / 64];
  const CJob& c = J.j[blockIdx.x];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid == 0) {
    s_base = c.hdr;
    s_any = 0;
  }
  __syncthreads();
  uint32_t any = 0;  // a fragment with tags (not stored from byte 0)
  for (uint32_t k = tid; k < c.nfrag; k += kScanT) any |= J.finfo[c.frag0 + k] != 0 ? 1u : 0u;
  if (any) s_any = 1;
  __syncthreads();
  int64_t lo = 0, hi = 0;  // the fragments' shifts (kPlaceShift's bounds)
  for (uint32_t k0 = 0; k0 < c.nfrag; k0 += kScanT) {
    const uint32_t k = k0 + tid;
    uint64_t v = 0;
    if (k < c.nfrag) {
      const size_t start = (size_t)k * kFrag;
      const uint64_t info = J.finfo[c.frag0 + k];
      v = frag_len(info, (uint32_t)min((size_t)kFrag, c.n - start));
    }
    uint64_t x = v;  // inclusive scan in the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if ((int)lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t before = s_base;
    for (uint32_t q = 0; q < wave; ++q) before += wsum[q];
    if (k < c.nfrag) {
      J.offset[c.frag0 + k] = before + x - v;
      if (c.stored) {
        const int64_t d = stored_shift(c, k, before + x - v);
        lo = min(lo, d);
        hi = max(hi, d);
      }
    }
    __syncthreads();
    if (tid == kScanT - 1) s_base = before + x;
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (int64_t)__shfl_xor(lo, o, 64));
    hi = max(hi, (int64_t)__shfl_xor(hi, o, 64));
  }
  if (lane == 0) {
    s_lo[wave] = lo;
    s_hi[wave] = hi;
  }
  __syncthreads();
  for (uint32_t w = 0; w < kScanT / 64; ++w) {
    lo = min(lo, s_lo[w]);
    hi = max(hi, s_hi[w]);
  }
  // (the stream's end: its growth must fit the stored stream's slack)
  const int64_t grow = c.stored ? (int64_t)s_base - (int64_t)stored_stream_bytes(stored_layout((uint32_t)c.n)) : 0;
  const uint32_t mode = !c.stored ? kPlaceCopy
                        : !s_any  ? kPlaceStored
                        : (lo >= -kShiftMax && hi <= kShiftMax && grow <= kShiftMax) ? kPlaceShift
                                                                                        : kPlaceCopy;
  if (tid == 0) J.in_place[blockIdx.x] = mode;
  if (mode == kPlaceCopy && tid < c.hdr) c.dst[tid] = (uint8_t)(((uint32_t)c.n >> (7 * tid)) | (tid + 1 < c.hdr ? 128u : 0u));
  if (tid == 0 && J.pub) {
    PubSlot* pub = J.pub + c.slot;
    pub_store(&pub->size, (uint64_t)s_base);
    pub_store(&pub->status, (int32_t)kOk);
    pub_store(&pub->pad, mode != kPlaceCopy ? (uint32_t)kStoredInPlace : 0u);
    publish_ticket(pub, c.ticket);
  }
}

// ---- K-place: one workgroup of 256 per fragment
constexpr uint32_t kPlaceT = 256;  // (512: C5 + COMPRESSING 1377 -> 1364, 1024: 1281 GiB/s)
constexpr int kMoveRows = 6;  // rows of 63 16-byte chunks per wave and pass (58 VGPRs: 8 waves per SIMD)
constexpr uint32_t kMovePass = kMoveRows * (kPlaceT / 64) * 63;  // chunks per pass (23.6 KiB)

// A fragment rewritten in place (kPlaceShift): at d its op tag bytes from tg,
// then the literal tag and the literal s[0, lit), which moves by D = (its new
// place - s), |D| small.  The literal goes in passes of kMovePass 16-byte
// destination chunks (lane l of a wave loads the aligned block under chunk l
// of its row of 63, as copy_bytes), each pass loaded whole before the
// workgroup's barrier and stored after it; the passes run from the end when
// D > 0 (a pass's stores then land only on bytes already read) and from the
// start when D < 0.  The tags, which may cover the literal's first D bytes,
// are stored last.
__device__ void place_moved(uint8_t* d, const uint8_t* tg, uint32_t op, const uint8_t* s, uint32_t lit, uint32_t tid) {
  constexpr uint32_t W = kPlaceT / 64;
  const uint32_t lane = tid & 63, wv = tid >> 6;
  uint8_t* dl = d + op + (lit ? lit_tag_len(lit - 1) : 0);
  const bool right = dl >= s;
  const uint32_t head = min(lit, (uint32_t)(-reinterpret_cast<uintptr_t>(dl) & 15));
  const uint32_t nc = (lit - head) >> 4;
  const uint32_t t0 = head + 16 * nc;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(s + head);
  typedef uint32_t V4 __attribute__((ext_vector_type(4)));
  const auto s16 = gbl<V4>(reinterpret_cast<const void*>(sp & ~(uintptr_t)15));
  const uint32_t sh = (uint32_t)(sp & 15);
  const uint32_t lim = nc + (sh ? 1u : 0u);
  uint4* d16 = reinterpret_cast<uint4*>(dl + head);
  const uint32_t np = nc ? (nc + kMovePass - 1) / kMovePass : 1;
  uint8_t hb0 = 0;
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t j = right ? np - 1 - i : i;
    const uint32_t c0 = j * kMovePass;
    uint4 lo[kMoveRows];
#pragma unroll
    for (int u = 0; u < kMoveRows; ++u) {
      const uint32_t c = c0 + (u * W + wv) * 63 + lane;
      V4 x = {0, 0, 0, 0};
      if (c < lim) x = s16[c];
      lo[u] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    const uint8_t hb = j == 0 && tid < head ? s[tid] : 0;
    const uint8_t tb = j + 1 == np && tid < lit - t0 ? s[t0 + tid] : 0;
    __syncthreads();  // this pass's bytes are all in registers
#pragma unroll
    for (int u = 0; u < kMoveRows; ++u) {
      const uint32_t c = c0 + (u * W + wv) * 63 + lane;
      const uint4 hi = shfl_down1(lo[u]);
      if (lane < 63 && c < nc) d16[c] = funnel16(lo[u], hi, sh);
    }
    if (j + 1 == np && tid < lit - t0) dl[t0 + tid] = tb;
    if (j == 0) hb0 = hb;
  }
  // (pass 0 has been read: last when D > 0; when D < 0 nothing stored below
  // the literal's new start is read again)
  if (tid < head) dl[tid] = hb0;
  if (lit) literal_tag(d + op, lit, tid);
  if (op) copy_bytes<kPlaceT>(d, tg, op, tid);
}

// A K-place workgroup's view of stream c (no K-scan): the offset of its
// fragment k, the stream's length and its PlaceMode.  Thread t takes fragments
// [t q, t q + q): their lengths before fragment k, whether any has tags, and
// (a stored job) how much longer than stored they come out -- whose prefix
// sums are the fragments' shifts.
struct PlaceLds {
  uint64_t part[kPlaceT / 64], all[kPlaceT / 64];
  int64_t tot[kPlaceT / 64], lo[kPlaceT / 64], hi[kPlaceT / 64];
  uint32_t any[kPlaceT / 64];
};
__device__ __forceinline__ void place_summary(const SnappyCJobs& J, const CJob& c, uint32_t k, PlaceLds& S,
                                              uint64_t& off, uint64_t& size, uint32_t& mode) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t q = (c.nfrag + kPlaceT - 1) / kPlaceT;
  const uint32_t i0 = min(c.nfrag, tid * q), i1 = min(c.nfrag, i0 + q);
  uint64_t part = 0, all = 0;
  uint32_t any = 0;
  int64_t tot = 0;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint64_t fi = J.finfo[c.frag0 + i];
    const uint32_t li = (uint32_t)min((size_t)kFrag, c.n - (size_t)i * kFrag);
    const uint32_t fl = frag_len(fi, li);
    if (i < k) part += fl;
    all += fl;
    any |= fi != 0 ? 1u : 0u;
    tot += (int64_t)fl - (int64_t)frag_len(0, li);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    part += __shfl_xor(part, o, 64);
    all += __shfl_xor(all, o, 64);
    any |= __shfl_xor(any, o, 64);
  }
  if (lane == 0) {
    S.part[wave] = part;
    S.all[wave] = all;
    S.any[wave] = any;
  }
  __syncthreads();
  off = c.hdr;
  size = c.hdr;
  any = 0;
  for (uint32_t w = 0; w < kPlaceT / 64; ++w) {
    off += S.part[w];
    size += S.all[w];
    any |= S.any[w];
  }
  mode = !c.stored ? kPlaceCopy : !any ? kPlaceStored : kPlaceCopy;
  int64_t lo = 0, hi = 0;
  if (c.stored && any) {
    int64_t x = tot;  // the shift of fragment i0: the exclusive sum of the totals
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if ((int)lane >= o) x += y;
    }
    if (lane == 63) S.tot[wave] = x;
    __syncthreads();
    int64_t run = x - tot;
    for (uint32_t w = 0; w < wave; ++w) run += S.tot[w];
    for (uint32_t i = i0; i < i1; ++i) {
      const uint32_t li = (uint32_t)min((size_t)kFrag, c.n - (size_t)i * kFrag);
      run += (int64_t)frag_len(J.finfo[c.frag0 + i], li) - (int64_t)frag_len(0, li);
      lo = min(lo, run);  // (the shift of fragment i + 1, or the growth at the end)
      hi = max(hi, run);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, (int64_t)__shfl_xor(lo, o, 64));
      hi = max(hi, (int64_t)__shfl_xor(hi, o, 64));
    }
    if (lane == 0) {
      S.lo[wave] = lo;
      S.hi[wave] = hi;
    }
    __syncthreads();
    for (uint32_t w = 0; w < kPlaceT / 64; ++w) {
      lo = min(lo, S.lo[w]);
      hi = max(hi, S.hi[w]);
    }
    if (lo >= -kShiftMax && hi <= kShiftMax) mode = kPlaceShift;
  }
  __syncthreads();  // (S is used again by the caller)
}

// Streams of up to kInlineScan fragments need no K-scan: the workgroup of
// fragment k sums the lengths of the stream's fragments itself (all full but
// the last); the workgroup of fragment 0 writes the varint header and
// publishes the stream length and mode -- the first workgroup of the stream
// to run, so the host, which needs them to finish the compress and launch the
// decode behind it, has them while K-place still runs (published by the last
// fragment's workgroup they arrived at its end, and the decode started 12-15
// us after it: C5 + COMPRESSING's kernel trace).
constexpr uint32_t kInlineScan = 4096;
__global__ __launch_bounds__(kPlaceT) void snappy_place(const SnappyCJobs J, const uint8_t* __restrict__ scratch) {
  __shared__ PlaceLds S;
  const uint32_t f = blockIdx.x, tid = threadIdx.x;
  // no K-scan: block j (among the first to run) publishes stream j's length
  // and mode, which the host needs to finish the compress and launch the
  // decode behind it -- it has them while K-place runs (published by the
  // stream's last, then its first fragment's workgroup, they arrived late in
  // K-place, and the decode started 12 us after it: kernel trace)
  if (!J.offset && blockIdx.x < J.njobs && J.pub) {
    const CJob& cj = J.j[blockIdx.x];
    uint64_t o, size;
    uint32_t m;
    place_summary(J, cj, cj.nfrag, S, o, size, m);
    if (tid == 0) {
      PubSlot* pub = J.pub + cj.slot;
      pub_store(&pub->size, size);
      pub_store(&pub->status, (int32_t)kOk);
      pub_store(&pub->pad, m != kPlaceCopy ? (uint32_t)kStoredInPlace : 0u);
      publish_ticket(pub, cj.ticket);
    }
  }
  const uint32_t ji = cjob_index(J, f);
  const CJob& c = J.j[ji];
  const uint32_t k = f - c.frag0;
  const size_t start = (size_t)k * kFrag;
  const uint32_t len = (uint32_t)min((size_t)kFrag, c.n - start);
  const uint64_t info = J.finfo[f];
  const uint32_t op = (uint32_t)(info >> 32), ne = (uint32_t)info;
  PSF_TRACE(f, 2);
  uint64_t off, size;
  uint32_t mode;
  if (J.offset) {
    mode = J.in_place[ji];
    if (mode == kPlaceStored) return;  // K-scan found every fragment stored: the stream is in place
    off = J.offset[f];
  } else {
    place_summary(J, c, k, S, off, size, mode);
    if (k == 0 && tid < c.hdr && mode == kPlaceCopy)
      c.dst[tid] = (uint8_t)(((uint32_t)c.n >> (7 * tid)) | (tid + 1 < c.hdr ? 128u : 0u));
    if (mode == kPlaceStored) return;  // FIXING_FLOAT wrote the stream, header and tags included
  }
  if (mode == kPlaceShift) {
    const int64_t dk = stored_shift(c, k, off);                       // this fragment's start
    const int64_t dn = dk + (int64_t)frag_len(info, len) - (int64_t)frag_len(0, len);  // the next one's
    if (!info && !dk) return;  // stored where it was written
    uint8_t* base = const_cast<uint8_t*>(c.in);
    const uint8_t* src = frag_src(c, k);
    uint8_t* dl = base + off + op + (ne < len ? lit_tag_len(len - ne - 1) : 0);
    place_moved(base + off, scratch + (size_t)f * kSnappyFragOut, op, src + ne, len - ne, tid);
    // the previous fragment's bytes end dk - (stored tag bytes) into this
    // one's (dk > 0), the next one's start -dn bytes before this one's end
    // (dn < 0): what the loads above may have seen rewritten there comes
    // from the stash
    const uint8_t* st = J.stash + (size_t)f * kStash;
    const uint32_t e = min(len, kEdge);
    const bool fix_head = dk > 0 && ne < e;
    const bool fix_tail = dn < 0 && k + 1 < c.nfrag && len >= kEdge;
    if (fix_head || fix_tail) {
      __syncthreads();
      if (fix_head && tid >= ne && tid < e) dl[tid - ne] = st[tid];
      const uint32_t p = len - kEdge + (tid - kEdge);
      if (fix_tail && tid >= kEdge && tid < kStash && p >= ne) dl[p - ne] = st[tid];
    }
    PSF_TRACE(f, 3);
    return;
  }
  uint8_t* d = c.dst + off;
  if (op) copy_bytes<kPlaceT>(d, scratch + (size_t)f * kSnappyFragOut, op, tid);
  if (ne < len) {
    d += op;
    d += literal_tag(d, len - ne, tid);
    copy_bytes<kPlaceT>(d, frag_src(c, k) + ne, len - ne, tid);
  }
  PSF_TRACE(f, 3);
}

// ------------------------------------------------------------------ uncompress
// compressed bytes per parse window: K1 / K3 are one wave per window whose
// chain walks are the work, so shorter windows mean more waves at once and
// shorter walks; the linker's work grows with the window count.  Sorted keys,
// 128 MiB, with the one-workgroup linker: 16 KiB windows 18.2 GB/s, 8 KiB
// 22.4, 4 KiB 22.7 (tools/ab_win8.sh); with the three-launch linker (K2a-c)
// 8 KiB 27.5, 4 KiB 30.0 (tools/ab_dec.sh).  (A literal that carries the
// chain past a window's first 64 bytes sends the stream to K2's serial walk;
// smaller windows have more starts to straddle.)
constexpr uint32_t kWin = 4096;
constexpr uint32_t kInWin = 4096;  // staged compressed bytes in the fragment decoder
// The fragment decoder's output window: the last kRing bytes of the fragment
// decoded so far sit in an LDS ring; older ones have been flushed to the
// output.  One decode step (a batch, or one tag; a long literal in pieces of
// kRingStep) writes at most kRingStep bytes; a step starts with at most
// kRingFlushAt bytes unflushed, so it overwrites only flushed bytes, and a copy
// source it cannot find in the ring was flushed before the step.
constexpr uint32_t kRing = 8192;
constexpr uint32_t kRingStep = 64 * 64;
constexpr uint32_t kRingFlushAt = kRing - kRingStep - 64;
constexpr uint32_t kBatchLit = 16;     // literals the fragment decoder's batches take (longer ones: one by one)
constexpr uint32_t kBatchMargin = 96;  // staged bytes past p a batch reads: 64 tag starts + a tag + kBatchLit
constexpr uint64_t kNone = ~0ull;
constexpr uint32_t kFlagInvalid = 1, kFlagSerial = 2, kFlagScan = 4, kFlagHeader = 8;
constexpr uint64_t kFullLit = 65536 + 3;  // a 64 KiB fragment stored as one literal (tag 0xF4 + 2 length bytes)
constexpr uint32_t kStarts = 64;          // K1 parses from each of the first 64 offsets of a window
// K0's single steps before it hands the stream to K1/K2: one memory latency
// each, so a tag-dense stream costs K0 about 1 us per step until handed over
// (512: K-spec 0.59 ms on sorted keys, 64: 0.10; tools/ab_dec.sh); a stream of
// stored fragments with a few matches (C5's codes) stays well inside it
constexpr uint32_t kLitBudget = 64;

struct Tag {
  uint64_t next;  // position after the tag (literal data included)
  uint64_t len;   // output bytes
  uint32_t off;   // copy offset (0 for literals)
  uint32_t hl;    // header bytes (literal data follows)
  bool lit;
};

// Branch-free decode of the tag whose first 5 bytes are x (little endian).
__device__ __forceinline__ Tag decode_tag(uint64_t x, uint64_t p) {
  Tag t;
  const uint32_t c = (uint32_t)x & 0xff;
  const uint32_t ty = c & 3;
  const uint32_t k = (c >> 2) + 1 > 60 ? (c >> 2) + 1 - 60 : 0;  // literal length bytes
  const uint64_t litlen = k ? ((x >> 8) & ((1ull << (8 * k)) - 1)) + 1 : (c >> 2) + 1;
  const uint32_t off1 = ((c >> 5) << 8) | (uint32_t)((x >> 8) & 0xff);
  const uint32_t off2 = (uint32_t)((x >> 8) & 0xffff);
  const uint32_t off4 = (uint32_t)(x >> 8);
  t.lit = ty == 0;
  t.hl = ty == 0 ? 1 + k : ty == 1 ? 2 : ty == 2 ? 3 : 5;
  t.len = ty == 0 ? litlen : ty == 1 ? 4 + ((c >> 2) & 7) : (c >> 2) + 1;
  t.off = ty == 0 ? 0 : ty == 1 ? off1 : ty == 2 ? off2 : off4;
  t.next = p + t.hl + (ty == 0 ? litlen : 0);
  return t;
}

__device__ __forceinline__ uint32_t lane_of32(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t lane_of64(uint64_t v, uint32_t l) {
  return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | __builtin_amdgcn_readlane((uint32_t)v, l);
}
// The tag starts of a batch: lane l holds the (clamped) advance a of the tag
// that would start at p + l; from offset 0 the chain goes l -> l + a(l).
// Returns the bit mask of the chain's offsets below 64 that start before
// `lim` (relative to p) and lie in `ok`: a few scalar instructions per tag.
__device__ __forceinline__ uint64_t batch_mask(uint32_t a, uint64_t lim, uint64_t ok) {
  uint64_t M = 0;
  for (uint32_t q = 0; q < 64 && q < lim && ((ok >> q) & 1);) {
    M |= 1ull << q;
    q += __builtin_amdgcn_readlane(a, q);
  }
  return M;
}
// exclusive sum over the wave's lanes below this one, in DPP steps (no LDS
// round trips: a lane shuffle through ds_bpermute costs one each): the
// inclusive scan within each row of 16 lanes by row shifts 1, 2, 4, 8 (a lane
// with no source in its row adds 0), then row 15's total into the next row
// (row_bcast:15, rows 1 and 3) and lane 31's into rows 2 and 3 (row_bcast:31)
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t) {
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x - v;
}

// lane l's 64-bit v, in every lane (l per lane)
__device__ __forceinline__ uint64_t bperm64(uint32_t l, uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * l, (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * l, (int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// tag at LDS byte q of w (one two-dword read; q + 8 bytes must be staged)
__device__ __forceinline__ Tag lds_tag(const uint32_t* w, uint64_t q, uint64_t p) {
  const uint32_t i = (uint32_t)(q >> 2);
  const uint64_t x = (((uint64_t)w[i + 1] << 32) | w[i]) >> (8 * (q & 3));
  return decode_tag(x, p);
}

// Stage in[base, base+want) into LDS: aligned dword loads where the whole word
// lies inside the input, bytes at the edges (0 past the end).  Returns s with
// lds[s + i] == in[base + i].
__device__ __forceinline__ uint32_t stage(uint32_t* lds, const uint8_t* in, uint64_t C, uint64_t base, uint32_t want,
                                          uint32_t lane) {
  const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(in + base) & 3);
  const int64_t r0 = (int64_t)base - (int64_t)s;  // input offset of lds byte 0 (dword aligned)
  const uint32_t nw = (s + want + 3) >> 2;
  // 8 loads in flight per lane before their LDS stores (one memory latency
  // per 2 KiB instead of one per 256 B)
  for (uint32_t j0 = 0; j0 < nw; j0 += 8 * 64) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + u * 64 + lane;
      const int64_t r = r0 + 4 * (int64_t)j;
      v[u] = 0;
      if (j < nw) {
        if (r >= 0 && r + 4 <= (int64_t)C) {
          v[u] = *reinterpret_cast<const uint32_t*>(in + r);
        } else {
          for (int q = 0; q < 4; ++q)
            if (r + q >= 0 && r + q < (int64_t)C) v[u] |= (uint32_t)in[r + q] << (8 * q);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t j = j0 + u * 64 + lane;
      if (j < nw) lds[j] = v[u];
    }
  }
  return s;
}

// the 5 tag bytes at input offset p (zero past the end): three aligned dwords
__device__ __forceinline__ uint64_t tag_bytes(const uint8_t* in, uint64_t C, uint64_t p) {
  const uintptr_t ia = reinterpret_cast<uintptr_t>(in);
  const uint64_t a = (ia + p) & ~(uintptr_t)3;
  const uint64_t ai = a - ia;
  uint32_t d[3] = {0, 0, 0};
  if (ai + 12 <= C) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a);
    d[0] = q[0];
    d[1] = q[1];
    d[2] = q[2];
  } else {
    for (int i = 0; i < 12; ++i) {
      const uint64_t r = ai + i;
      if (r < C) d[i >> 2] |= (uint32_t)in[r] << (8 * (i & 3));
    }
  }
  const uint32_t sh = (uint32_t)(p - ai) * 8;
  const uint64_t lo = ((uint64_t)d[1] << 32) | d[0];
  return sh ? (lo >> sh) | ((uint64_t)d[2] << (64 - sh)) : lo;
}

// The host sized the launch from a hint (the FilterConfig's uncompressed
// size): the stream's own varint header must say the same, else the host
// redoes the call from the header (Varint::Parse32WithLimit).
__device__ __forceinline__ bool header_matches(const uint8_t* __restrict__ in, uint64_t C, uint32_t hdr,
                                               uint64_t dsize) {
  const uint64_t h = tag_bytes(in, C, 0);
  uint64_t v = 0;
  uint32_t len = 0;
  for (uint32_t i = 0; i < 5 && i < C; ++i) {
    const uint32_t b = (uint32_t)(h >> (8 * i)) & 0xff;
    if (i == 4 && b >= 16) break;
    v |= (uint64_t)(b & 127u) << (7 * i);
    if (b < 128) {
      len = i + 1;
      break;
    }
  }
  return len == hdr && v == dsize;
}

// d[0, len) = s[0, len) for any alignment of either, by 256 lanes: byte
// stores up to the first 4-aligned destination dword, then lane-contiguous
// dwords (each load and store instruction covers 256 contiguous bytes), each
// funnel-shifted from the two aligned source dwords that cover it, 16 per lane
// per step with all loads issued before the stores (a wave's memory counter
// retires in order: a load behind a store waits for it).  The loads are
// unconditional (clamped), the stores predicated, so the compiler keeps exact
// wait counts.  (Round 3: 16-byte chunks from five dword loads each ran the
// 128 MiB stored stream at 3.7 TB/s, tools/ab_dq.sh.)  U = dwords in flight
// per lane: 16 in K-spec, fewer in K4, whose occupancy its decoder sets.
template <int U = 16>
__device__ __forceinline__ void copy_g2g(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, uint32_t len,
                                         uint32_t tid) {
  uint32_t head = (uint32_t)(-reinterpret_cast<uintptr_t>(d) & 3);
  if (head > len) head = len;
  if (tid < head) d[tid] = s[tid];
  d += head;
  s += head;
  len -= head;
  const uintptr_t sa = reinterpret_cast<uintptr_t>(s);
  const uint32_t sh = (uint32_t)(sa & 3) * 8;
  const auto a = gbl<uint32_t>(reinterpret_cast<const void*>(sa & ~(uintptr_t)3));  // global, not flat, loads
  auto* o = reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(reinterpret_cast<uintptr_t>(d));
  const uint32_t ng = len >> 2;
  for (uint32_t g0 = 0; g0 < ng; g0 += U * 256) {
    uint32_t w0[U], w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t g = min(g0 + u * 256 + tid, ng - 1);
      w0[u] = a[g];
      w1[u] = a[sh ? g + 1 : g];  // the next dword lies inside the source only when it is needed
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t g = g0 + u * 256 + tid;
      if (g < ng) o[g] = sh ? __builtin_amdgcn_alignbit(w1[u], w0[u], sh) : w0[u];
    }
  }
  for (uint32_t i = (ng << 2) + tid; i < len; i += 256) d[i] = s[i];
}

// Last-workgroup election by one device-scope counter.  No fence: what the
// last workgroup goes on to do reads nothing the others wrote in this launch
// (an agent-scope fence on MI355X writes back the XCD's whole L2, which
// every workgroup of a streaming kernel would pay for).
__device__ __forceinline__ bool last_block(uint32_t* ctr, uint32_t total, uint32_t* s_last) {
  __syncthreads();
  if (threadIdx.x == 0) *s_last = atomicAdd(ctr, 1u) == total - 1;
  __syncthreads();
  return *s_last;
}

// Several streams decode in one launch chain (the COMPRESSING arrays of a
// batch of messages): every kernel's grid is the union of the streams' output
// fragments (or windows, or streams), and a workgroup first finds its stream
// in the job table, which rides in the kernel arguments.
struct DJob {
  const uint8_t* in;
  uint8_t* out;
  uint8_t* scratch;  // this stream's index arrays
  uint64_t C, dsize;
  uint32_t hdr, nfo, nwin;
  uint32_t fo0, win0;  // first output fragment / window of this stream in the grids
  uint32_t slot, ticket;
  // fused FIXING_FLOAT decode (SnappyDequant): values of the codes, or null
  void* fv;
  const float* frange;
  double fratio;
  float fmn, fmx;
  uint32_t fnb, fdbl;
  uint32_t blk0;  // first linker block of this stream in the linker grids
};
struct SnappyDJobs {
  DJob j[kSnappyBatchMax];
  uint32_t* ctrl;  // 8 words per stream: flags[0..3] (verdict, indexed, decoded by K-spec, linked by K2b), counters[4..7]
  PubSlot* pub;
  uint32_t njobs, nfo1, nwin;  // streams; output fragments (at least one per stream); windows
  uint32_t nblk;               // linker blocks (kLinkPer windows each)
  uint32_t* znext;  // the next launch's zeroed ctrl region (null: none), cleared by K-spec
  uint32_t zwords;
};
struct DScr {
  uint32_t *flags, *ctr;
  uint64_t *wexit, *wtotal, *wentry, *woff, *fragpos, *specpos, *specend;
  uint32_t *fdone;  // fused decode: fragment k's values written by K-spec (1) or still codes (0)
  uint32_t *bitmap, *cum;
};
__device__ __forceinline__ DScr dscr(const SnappyDJobs& J, const DJob& D, uint32_t i) {
  DScr S;
  S.flags = J.ctrl + 8 * i;
  S.ctr = S.flags + 4;
  S.wexit = reinterpret_cast<uint64_t*>(D.scratch);
  S.wtotal = S.wexit + (size_t)(D.nwin + 1) * kStarts;
  S.wentry = S.wtotal + (size_t)(D.nwin + 1) * kStarts;
  S.woff = S.wentry + (D.nwin + 1);
  S.fragpos = S.woff + (D.nwin + 1);
  S.specpos = S.fragpos + (D.nfo + 1);
  S.specend = S.specpos + (D.nfo + 1);
  S.fdone = reinterpret_cast<uint32_t*>(S.specend + (D.nfo + 1));
  S.bitmap = reinterpret_cast<uint32_t*>(S.specend + 2 * (D.nfo + 1));
  S.cum = S.bitmap + (size_t)(D.nwin + 1) * (kWin / 32);
  return S;
}
// the stream of output fragment b / window b of the union grids
__device__ __forceinline__ uint32_t djob_frag(const SnappyDJobs& J, uint32_t b) {
  uint32_t i = 0;
  while (i + 1 < J.njobs && b >= J.j[i + 1].fo0) ++i;
  return i;
}
__device__ __forceinline__ uint32_t djob_win(const SnappyDJobs& J, uint32_t b) {
  uint32_t i = 0;
  while (i + 1 < J.njobs && b >= J.j[i + 1].win0) ++i;
  return i;
}

// ---- FIXING_FLOAT decode fused into the uncompress (SnappyDequant) ----
// A stream of FIXING_FLOAT codes whose next decode is FIXING_FLOAT is decoded
// straight to values: where the fast path copies a stored fragment, it
// dequantises it instead (the codes never reach HBM), and fragments placed any
// other way are dequantised from their codes afterwards.  The arithmetic is
// ff_decode's (ff_dequant.h), so the values are bit-identical to the unfused
// chain.
typedef float dq_f32x4 __attribute__((ext_vector_type(4)));
typedef float dq_f32x2 __attribute__((ext_vector_type(2)));
typedef double dq_f64x2 __attribute__((ext_vector_type(2)));

struct DqParams {
  double ratio, inv, bin, min_v;
};
// ff_decode's parameters for stream D (the encode's device range when it left one)
__device__ __forceinline__ DqParams dq_params(const DJob& D) {
  float mn = D.fmn, mx = D.fmx;
  if (D.frange) {
    mn = D.frange[0];
    mx = D.frange[1];
  }
  DqParams P;
  P.min_v = (double)mn;
  P.bin = (double)mx - P.min_v;
  P.ratio = D.fratio;
  P.inv = 1.0 / P.ratio;
  return P;
}

// nb = 1: the 256-entry table ff_decode builds (same formula, same bits)
template <typename V>
__device__ __forceinline__ void dq_lut(V* lut, const DqParams& P, uint32_t tid) {
  lut[tid] = dequant<V>((uint64_t)tid, P.ratio, P.bin, P.min_v);
}

// the values of one dword of codes (4 / NB of them) to o, non-temporal
template <typename V, int NB>
__device__ __forceinline__ void dq_store(V* o, uint32_t w, const V* lut, const DqParams& P) {
  if (NB == 1) {
    const V x0 = lut[w & 255], x1 = lut[(w >> 8) & 255], x2 = lut[(w >> 16) & 255], x3 = lut[w >> 24];
    if constexpr (sizeof(V) == 4) {
      const dq_f32x4 t = {(float)x0, (float)x1, (float)x2, (float)x3};
      __builtin_nontemporal_store(t, reinterpret_cast<dq_f32x4*>(o));
    } else {
      const dq_f64x2 a = {(double)x0, (double)x1}, b = {(double)x2, (double)x3};
      __builtin_nontemporal_store(a, reinterpret_cast<dq_f64x2*>(o));
      __builtin_nontemporal_store(b, reinterpret_cast<dq_f64x2*>(o) + 1);
    }
  } else {
    const V x0 = dequant_q<V>(w & 0xFFFF, P.ratio, P.inv, P.bin, P.min_v);
    const V x1 = dequant_q<V>(w >> 16, P.ratio, P.inv, P.bin, P.min_v);
    if constexpr (sizeof(V) == 4) {
      const dq_f32x2 t = {(float)x0, (float)x1};
      __builtin_nontemporal_store(t, reinterpret_cast<dq_f32x2*>(o));
    } else {
      const dq_f64x2 t = {(double)x0, (double)x1};
      __builtin_nontemporal_store(t, reinterpret_cast<dq_f64x2*>(o));
    }
  }
}

// v[0, len / NB) = the values of the codes s[0, len) (s at any alignment, v
// 16-byte aligned, len a multiple of NB), by 256 lanes: lane l takes the
// dwords of codes l, l + 256, ..., each funnel-shifted from the two aligned
// dwords that cover it (the second lies inside the source whenever it is
// needed), 8 in flight before any store.
template <typename V, int NB, int U>
__device__ void dq_bytes(const uint8_t* __restrict__ s, V* __restrict__ v, uint32_t len, const V* lut,
                         const DqParams& P, uint32_t tid) {
  const uintptr_t sa = reinterpret_cast<uintptr_t>(s);
  const uint32_t sh = (uint32_t)(sa & 3) * 8;
  const auto a = gbl<uint32_t>(reinterpret_cast<const void*>(sa & ~(uintptr_t)3));  // global, not flat, loads
  const uint32_t ng = len >> 2;
  for (uint32_t g0 = 0; g0 < ng; g0 += U * 256) {
    uint32_t w0[U], w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t g = min(g0 + u * 256 + tid, ng - 1);
      w0[u] = a[g];
      w1[u] = a[sh ? g + 1 : g];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t g = g0 + u * 256 + tid;
      const uint32_t w = sh ? __builtin_amdgcn_alignbit(w1[u], w0[u], sh) : w0[u];
      if (g < ng) dq_store<V, NB>(v + (size_t)g * (4 / NB), w, lut, P);
    }
  }
  for (uint32_t i = (ng << 2) / NB + tid; i < len / NB; i += 256) {  // the array's last len % 4 bytes
    uint32_t r = 0;
    for (int j = 0; j < NB; ++j) r |= (uint32_t)s[i * NB + j] << (8 * j);
    v[i] = NB == 1 ? lut[r] : dequant_q<V>(r, P.ratio, P.inv, P.bin, P.min_v);
  }
}

// The workgroup's LDS table (nb = 1) for stream D; called by all 256 lanes,
// ends with a barrier.
__device__ __forceinline__ void dq_prepare(const DJob& D, double* lut64, uint32_t tid) {
  const DqParams P = dq_params(D);
  if (D.fnb == 1) {
    if (D.fdbl) dq_lut<double>(lut64, P, tid);
    else dq_lut<float>(reinterpret_cast<float*>(lut64), P, tid);
  }
  __syncthreads();
}

// Output fragment bytes [o0, o0 + len) of stream D, whose codes are at s, to
// their values (after dq_prepare).  U = code dwords in flight per lane: K-spec
// (global loads, C5 + COMPRESSING) measured 4 / 8 / 12 / 16 / 32 at
// 119 / 113 / 112 / 110 / 110 us (tools/ab_dq.sh); K4 keeps 8 (its decoder's
// registers set its occupancy).
template <int U = 16>
__device__ __forceinline__ void dq_frag(const DJob& D, const uint8_t* s, uint64_t o0, uint32_t len,
                                        const double* lut64, uint32_t tid) {
  const DqParams P = dq_params(D);
  const uint64_t first = o0 / D.fnb;  // 65536 is a multiple of nb
  if (D.fdbl) {
    double* v = static_cast<double*>(D.fv) + first;
    if (D.fnb == 1) dq_bytes<double, 1, U>(s, v, len, lut64, P, tid);
    else dq_bytes<double, 2, U>(s, v, len, lut64, P, tid);
  } else {
    float* v = static_cast<float*>(D.fv) + first;
    const float* lut = reinterpret_cast<const float*>(lut64);
    if (D.fnb == 1) dq_bytes<float, 1, U>(s, v, len, lut, P, tid);
    else dq_bytes<float, 2, U>(s, v, len, lut, P, tid);
  }
}

// K0: link the chain directly when the stream is mostly 64 KiB fragments
// stored as single literals (what a snappy 1.1.8 encoder emits for
// incompressible fragments, e.g. FIXING_FLOAT codes): lane k decodes the tags
// at p + (k + 64 j) * kFullLit for j < kLitRows, and the leading run of
// positions that hold a full literal is consumed in one step (512 fragments
// per memory latency); other tags take a single step.  After kLitBudget
// single steps the stream is handed to the window scan (K1) and its linker
// (K2) through kFlagScan.  K0 also records each output fragment's first tag
// and checks the tags it steps over one at a time as K3 would (the full
// literals have no copies); if it walks the whole stream, flags[1] = 1 tells
// K3 there is nothing left to index or validate.
// (One wave; its stores to a word are issued in program order, so the
// initialisation needs no barrier.)
constexpr int kLitRows = 8;
__device__ void dlit_body(const uint8_t* __restrict__ in, uint64_t C, uint32_t hdr, uint64_t dsize, uint32_t nwin,
                          uint64_t* __restrict__ wentry, uint64_t* __restrict__ woff, uint64_t* __restrict__ fragpos,
                          uint32_t* __restrict__ flags, uint32_t lane) {
  for (uint32_t i = lane; i < nwin; i += 64) wentry[i] = kNone;
  if (lane == 0) flags[1] = 0;
  if (!header_matches(in, C, hdr, dsize)) {
    if (lane == 0) *flags = kFlagHeader;
    return;
  }
  uint64_t p = hdr, o = 0;
  int64_t last_w = -1;
  uint32_t singles = 0;
  bool bad = false, serial = false, wide = true;
  while (p < C) {
    bool full[kLitRows];
    uint64_t pk[kLitRows];
    Tag t0;
#pragma unroll
    for (int j = 0; j < kLitRows; ++j) {
      pk[j] = p + (uint64_t)(lane + 64 * j) * kFullLit;
      full[j] = false;
      if (j == 0 || wide) {  // after a single step, probe one row only
        const Tag t = decode_tag(tag_bytes(in, C, pk[j]), pk[j]);
        full[j] = pk[j] < C && t.lit && t.len == 65536 && t.hl == 3;
        if (j == 0) t0 = t;
      }
    }
    uint32_t c = 0;  // leading run of full literals over rows 0, 1, ...
    bool open = true;
#pragma unroll
    for (int j = 0; j < kLitRows; ++j) {
      const uint64_t m = __ballot(full[j]);
      if (open) {
        const uint32_t r = m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
        c += r;
        open = r == 64;
      }
    }
    if (c > 0) {
      const bool aligned = (o & (kFrag - 1)) == 0;
      serial = serial || !aligned;  // full literals across output fragments
#pragma unroll
      for (int j = 0; j < kLitRows; ++j) {
        const uint32_t idx = lane + 64 * j;
        if (idx < c) {
          const int64_t wk = (int64_t)((pk[j] - hdr) / kWin);
          if (idx > 0 || wk > last_w) {  // full literals are > kWin apart: one per window
            wentry[wk] = pk[j];
            woff[wk] = o + (uint64_t)idx * 65536;
          }
          if (aligned) fragpos[o / kFrag + idx] = pk[j];
        }
      }
      last_w = (int64_t)((p + (uint64_t)(c - 1) * kFullLit - hdr) / kWin);
      p += (uint64_t)c * kFullLit;
      o += (uint64_t)c * 65536;
      wide = true;
    } else {
      wide = false;
      const uint64_t t0next = __shfl(t0.next, 0, 64), t0len = __shfl(t0.len, 0, 64);
      const bool t0lit = __shfl((int)t0.lit, 0, 64) != 0;
      const uint32_t t0off = __shfl(t0.off, 0, 64);
      const int64_t w0 = (int64_t)((p - hdr) / kWin);
      if (lane == 0) {
        if (w0 > last_w) {
          wentry[w0] = p;
          woff[w0] = o;
        }
        if ((o & (kFrag - 1)) == 0) fragpos[o / kFrag] = p;  // the tag that starts an output fragment
      }
      // what K3 checks, for the tags seen one at a time (the full literals
      // of the wide steps have no copies): a copy within the output so far,
      // and no tag or copy across output fragments (else the one-lane decoder)
      if (!t0lit) {
        if (t0off == 0 || t0off > o) bad = true;
        else if (o - t0off < (o & ~(uint64_t)(kFrag - 1))) serial = true;
      }
      if (o / kFrag != (o + t0len - 1) / kFrag) serial = true;
      if (w0 > last_w) last_w = w0;
      p = t0next;
      o += t0len;
      if (++singles > kLitBudget) {
        if (lane == 0) *flags = kFlagScan;
        return;
      }
    }
    if (o > dsize) {
      bad = true;
      break;
    }
  }
  const bool ok = !(bad || p != C || o != dsize);
  if (lane == 0) {
    *flags = !ok ? kFlagInvalid : serial ? kFlagSerial : 0u;
    flags[1] = ok ? 1u : 0u;  // every tag seen: K3 has nothing to add
  }
}

constexpr uint32_t kFewTags = 8;  // fragments of at most this many tags are decoded without LDS

struct FewLds {
  uint32_t n, o[kFewTags], len[kFewTags], off[kFewTags];
  uint64_t src[kFewTags], next;
};

// Output fragment d[0, end) from the tags at p, when they are at most
// kFewTags, end exactly at the fragment's end and copy only from inside it
// (stored data with a match or two): one lane walks the tags (checking each as
// RawUncompress would), all 256 lanes copy the literals global to global, then
// the copies run in order.  Returns the position after the fragment's last
// tag, or kNone (nothing written) when the fragment is not of that kind.
// Called by the whole workgroup.  U: copy_g2g's dwords in flight per lane.
template <int U = 16>
__device__ uint64_t decode_few(const uint8_t* __restrict__ in, uint64_t C, uint64_t p, uint32_t end,
                               uint8_t* __restrict__ d, uint32_t tid, FewLds& F) {
  if (tid == 0) {
    uint32_t o = 0, n = 0;
    bool good = p < C;
    while (good && o < end && n < kFewTags) {
      const Tag t = decode_tag(tag_bytes(in, C, p), p);
      if (t.lit ? t.next > C : (t.off == 0 || t.off > o)) good = false;
      F.o[n] = o;
      F.len[n] = (uint32_t)t.len;
      F.off[n] = t.off;
      F.src[n] = t.lit ? p + t.hl : kNone;
      o += (uint32_t)min(t.len, (uint64_t)kFrag + 1);
      p = t.next;
      ++n;
    }
    F.n = good && o == end ? n : 0;
    F.next = p;
  }
  __syncthreads();
  const uint32_t nt = F.n;
  if (nt == 0) return kNone;
  for (uint32_t i = 0; i < nt; ++i)
    if (F.src[i] != kNone) copy_g2g<U>(d + F.o[i], in + F.src[i], F.len[i], tid);
  __syncthreads();
  for (uint32_t i = 0; i < nt; ++i) {
    if (F.src[i] != kNone) continue;
    const uint32_t o = F.o[i], L = F.len[i], off = F.off[i];
    for (uint32_t j = tid; j < L; j += 256) d[o + j] = d[o - off + (off >= L ? j : j % off)];
    __syncthreads();
  }
  return F.next;
}

// K-spec: every output fragment k is first taken to be stored as one literal
// at hdr + k * (65536 + 3) -- what a 1.1.8 encoder writes for a stream of
// incompressible fragments (FIXING_FLOAT codes).  A workgroup checks its
// fragment's tag there and, if it is the literal that fills the fragment,
// copies it at once; a fragment found a few bytes off that place (after one
// with a match) is copied from there, and the first fragment with a few tags
// is decoded where assumed.  If every fragment was placed and each ends where
// the next begins (the first after the header, the last at the end of the
// stream), the stream is exactly that chain: decoded and valid, as the last
// workgroup to finish records.  One more workgroup
// runs K0 alongside (its verdict and index agree with that on such a stream);
// otherwise the kernels after this one redo every fragment whose true
// position differs from the one assumed here (specpos).
__global__ __launch_bounds__(256) void snappy_dspec(const SnappyDJobs J) {
  __shared__ uint32_t s_last, s_checked;
  __shared__ double s_lut[256];  // fused decode, nb = 1
  const uint32_t tid = threadIdx.x;
  if (J.znext)  // the next launch's control words (this launch's were cleared by the one before)
    for (uint32_t i = blockIdx.x * 256 + tid; i < J.zwords; i += gridDim.x * 256) J.znext[i] = 0;
  if (blockIdx.x < J.njobs) {  // one more workgroup per stream links it meanwhile (K0), needed or not
    const uint32_t i = blockIdx.x;  // dispatched first: its walk overlaps the copies
    const DJob& D = J.j[i];
    const DScr S = dscr(J, D, i);
    if (tid < 64) dlit_body(D.in, D.C, D.hdr, D.dsize, D.nwin, S.wentry, S.woff, S.fragpos, S.flags, tid);
    return;
  }
  const uint32_t b = blockIdx.x - J.njobs;
  const uint32_t ji = djob_frag(J, b);
  const DJob& D = J.j[ji];
  const DScr S = dscr(J, D, ji);
  const uint8_t* __restrict__ in = D.in;
  uint8_t* __restrict__ out = D.out;
  const uint64_t C = D.C, dsize = D.dsize;
  const uint32_t hdr = D.hdr, nfo = D.nfo, ticket = D.ticket;
  uint64_t* __restrict__ specpos = S.specpos;
  uint32_t* __restrict__ flags = S.flags;
  uint32_t* __restrict__ ctr = S.ctr;
  PubSlot* pub = J.pub ? J.pub + D.slot : nullptr;
  const uint32_t k = b - D.fo0, nspec = nfo ? nfo : 1;
  const uint64_t o0 = (uint64_t)k * kFrag;
  const uint32_t end = (uint32_t)min((uint64_t)kFrag, dsize - o0);  // 0 only for an empty output
  const uint64_t p = hdr + (uint64_t)k * kFullLit;
  bool ok = k > 0 || header_matches(in, C, hdr, dsize);
  uint32_t hl = 0;
  if (end == 0) {
    ok = ok && C == hdr;
  } else {
    hl = end - 1 < 60 ? 1 : ((31 - __builtin_clz(end - 1)) >> 3) + 2;
    const Tag t = decode_tag(tag_bytes(in, C, p), p);
    ok = ok && p < C && t.lit && t.len == end && t.hl == hl && t.next <= C && (k + 1 < nfo || t.next == C);
  }
  if (D.fv) dq_prepare(D, s_lut, tid);  // the range load overlaps the tag's
  // A fragment after one that is not stored (a 1.1.8 encoder found a match in
  // it) sits a few bytes off its assumed place: look for its literal within
  // +-128 bytes and copy it from there too.  That is a guess only (it does not
  // count as checked); K4 redoes the fragment unless K0/K3 find it there.
  uint64_t at = ok ? p : kNone;
  if (!ok && end && k > 0) {
    __shared__ uint32_t s_best;
    if (tid == 0) s_best = 0xffffffffu;
    __syncthreads();
    const int32_t dl = (int32_t)tid - 128;
    const uint64_t q = p + dl;
    if (dl != 0 && q < C) {
      const Tag t = decode_tag(tag_bytes(in, C, q), q);
      if (t.lit && t.len == end && t.hl == hl && t.next <= C && (k + 1 < nfo || t.next == C))
        atomicMin(&s_best, ((uint32_t)abs(dl) << 9) | tid);
    }
    __syncthreads();
    if (s_best != 0xffffffffu) at = p + (int32_t)(s_best & 511) - 128;
  }
  uint64_t e = kNone;  // where this fragment's tags end
  uint32_t vdone = 0;   // fused decode: this fragment's values written here
  if (at != kNone) {
    if (D.fv) {
      dq_frag(D, in + at + hl, o0, end, s_lut, tid);
      vdone = 1;
    } else {
      copy_g2g(out + o0, in + at + hl, end, tid);
    }
    e = at + hl + end;
  } else if (end && (k > 0 || header_matches(in, C, hdr, dsize))) {
    // not stored: a fragment with a few tags, right after stored ones that
    // all sit where assumed (the first such fragment of the stream), is
    // decoded here too
    __shared__ FewLds F;
    e = decode_few(in, C, p, end, out + o0, tid, F);
    if (e != kNone) {
      at = p;
      if (D.fv) {  // the codes just written (L2-hot) to their values (decode_few ends with a barrier)
        dq_frag(D, out + o0, o0, end, s_lut, tid);
        vdone = 1;
      }
    }
  } else if (ok) {
    e = C;  // the empty output: the header is the stream
  }
  // device-scope stores: the last workgroup reads them from another XCD
  if (tid == 0) {
    __hip_atomic_store(&specpos[k], at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&S.specend[k], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.fdone[k] = vdone;  // read by K4 (a later launch)
  }
  // one counter for both: workgroups done (high word) and fragments placed
  const bool placed = e != kNone;
  __syncthreads();
  if (tid == 0) {
    const unsigned long long old =
        atomicAdd(reinterpret_cast<unsigned long long*>(ctr), (1ull << 32) | (placed ? 1ull : 0ull));
    s_last = (uint32_t)(old >> 32) == nspec - 1;
    s_checked = (uint32_t)old + (placed ? 1u : 0u);
  }
  __syncthreads();
  if (!s_last) return;
  // every fragment placed somewhere: the stream is that chain if each one
  // ends where the next begins, the first begins after the header and the
  // last ends the stream
  __shared__ uint32_t s_chain;
  if (tid == 0) s_chain = s_checked == nspec ? 1u : 0u;
  __syncthreads();
  if (s_chain) {
    for (uint32_t i = tid; i < nspec; i += 256) {
      const uint64_t pos = __hip_atomic_load(&specpos[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t prev = i ? __hip_atomic_load(&S.specend[i - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (uint64_t)hdr;
      bool good = pos == prev;
      if (i + 1 == nspec)
        good = good && __hip_atomic_load(&S.specend[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == C;
      if (!good) s_chain = 0;  // any lane may clear it
    }
  }
  __syncthreads();
  if (s_chain) {
    if (tid == 0) {
      flags[0] = 0;
      flags[1] = 1;
      flags[2] = 1;  // decoded: the kernels after this one have nothing to do
      if (pub) {
        pub_store(&pub->status, (int32_t)kOk);
        pub_store(&pub->size, (uint64_t)dsize);
        publish_ticket(pub, ticket);
      }
    }
  }
}


// K2: link the windows along the true chain.  The walk is one chain (every
// lane holds the same values); K1's tables of the next kLinkAhead windows
// (exit and output count per start offset) are copied into LDS together, so a
// window entered at one of its first 64 bytes costs one LDS read and one
// memory latency per kLinkAhead windows.  Other entries step tag by tag until
// they meet lane 0's chain (bitmap word and the next tag's bytes loaded
// together).  Windows are entered in increasing order, so the first-entry
// bookkeeping stays in registers.
constexpr uint32_t kLinkAhead = 16;
__device__ void dlink_body(const uint8_t* __restrict__ in, uint64_t C, uint32_t hdr, uint64_t dsize,
                           const uint32_t* __restrict__ bitmap, const uint32_t* __restrict__ cum,
                           const uint64_t* __restrict__ wexit, const uint64_t* __restrict__ wtotal, uint32_t nwin,
                           uint64_t* __restrict__ wentry, uint64_t* __restrict__ woff, uint32_t* __restrict__ flags,
                           uint64_t* lex, uint64_t* ltot) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < nwin; i += 64) wentry[i] = kNone;
  __syncthreads();
  uint64_t p = hdr, o = 0;
  int64_t last_w = -1;  // highest window whose entry is recorded
  bool bad = false;
  const uintptr_t ia = reinterpret_cast<uintptr_t>(in);
  uint32_t tw = 0;  // first window of the tables in LDS
  bool have = false;
  while (p < C) {
    const uint64_t rel = p - hdr;
    const uint32_t w = (uint32_t)(rel / kWin);
    const uint64_t off = rel - (uint64_t)w * kWin;
    if ((int64_t)w > last_w) {
      if (lane == 0) {
        wentry[w] = p;
        woff[w] = o;
      }
      last_w = w;
    }
    if (off < kStarts) {  // parsed exactly by K1's lane `off`
      if (!have || w - tw >= kLinkAhead) {
        have = true;
        tw = w;
        uint64_t e[kLinkAhead], t[kLinkAhead];
#pragma unroll
        for (uint32_t j = 0; j < kLinkAhead; ++j) {
          const size_t r = (size_t)min(w + j, nwin - 1) * kStarts + lane;
          e[j] = wexit[r];
          t[j] = wtotal[r];
        }
#pragma unroll
        for (uint32_t j = 0; j < kLinkAhead; ++j) {
          lex[j * kStarts + lane] = e[j];
          ltot[j * kStarts + lane] = t[j];
        }
      }
      const uint32_t q = (w - tw) * kStarts + (uint32_t)off;
      o += ltot[q];
      p = lex[q];
    } else {
      // bitmap word and the 8 bytes at p, loaded together
      const uint32_t bw = bitmap[rel >> 5];
      const uint64_t a = (ia + p) & ~(uintptr_t)3;  // aligned dword address
      const uint64_t ai = a - ia;                    // its input offset (may be < p)
      uint32_t d0 = 0, d1 = 0, d2 = 0;
      if (ai + 12 <= C) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(a);
        d0 = q[0];
        d1 = q[1];
        d2 = q[2];
      } else {
        for (int i = 0; i < 12; ++i) {
          const uint64_t r = ai + i;
          const uint32_t b = r < C ? in[r] : 0;
          if (i < 4) d0 |= b << (8 * i); else if (i < 8) d1 |= b << (8 * (i - 4)); else d2 |= b << (8 * (i - 8));
        }
      }
      if ((bw >> (rel & 31)) & 1) {  // met lane 0's chain
        o += wtotal[(size_t)w * kStarts] - cum[p];
        p = wexit[(size_t)w * kStarts];
      } else {  // one tag, then look again
        const uint32_t sh = (uint32_t)(p - ai) * 8;  // 0..24
        const uint64_t lo = ((uint64_t)d1 << 32) | d0;
        const uint64_t x = sh ? (lo >> sh) | ((uint64_t)d2 << (64 - sh)) : lo;
        const Tag t = decode_tag(x, p);
        o += t.len;
        p = t.next;
      }
    }
    if (o > dsize) {
      bad = true;
      break;
    }
  }
  if (lane == 0) *flags = (bad || p != C || o != dsize) ? kFlagInvalid : 0;
}

// K1: speculative parse of each window from each of its first 64 byte offsets
// (lane l from offset l).  A window's true entry is one of them unless a literal
// carried the chain further in; for those K2 walks until it meets lane 0's chain.
constexpr uint32_t kEarly = 1024;  // bytes of a window where K1's starts are expected to meet lane 0's chain

// The chain of tags from p (relative to the staged window) to the first
// position >= wl, walked by the wave in batches: every lane decodes the tag
// that would start at p + lane, one scalar walk picks the chain's tags in
// [p, p + 64).  Adds the output to o, returns the exit position.  kRecord:
// lane 0's chain of K1 -- each tag into the bitmap, its output count before
// it into cum.
template <bool kRecord>
__device__ uint64_t scan_walk(const uint32_t* b32, uint32_t s, uint32_t wl, uint64_t p, uint64_t& o, uint32_t lane,
                              uint32_t* bm, uint32_t* __restrict__ cum) {
  while (p < wl) {
    const uint64_t pl = min(p + lane, (uint64_t)wl);
    const Tag tl = lds_tag(b32, s + pl, pl);
    const uint64_t adv = tl.next - pl;
    const uint64_t M = batch_mask((uint32_t)min(adv, (uint64_t)64), wl - p, ~0ull);
    const bool tag = (M >> lane) & 1;
    // a tag's output offset in the batch: every tag before the last has a
    // length <= 64 (it ends inside the batch)
    const uint32_t rel = wave_excl_sum(tag ? (uint32_t)min(tl.len, (uint64_t)64) : 0u, lane);
    if (kRecord && tag) {
      const uint64_t r = p + lane;
      atomicOr(&bm[r >> 5], 1u << (r & 31));
      cum[r] = (uint32_t)(o + rel);
    }
    const uint32_t last = 63 - __builtin_clzll(M);
    o += lane_of32(rel, last) + lane_of64(tl.len, last);
    p += last + lane_of64(adv, last);
  }
  return p;
}

__device__ void dscan_body(const SnappyDJobs& J, uint32_t ji, uint32_t w, uint32_t* b32, uint32_t* bm) {
  const DJob& D = J.j[ji];
  const DScr S = dscr(J, D, ji);
  if (!(*S.flags & kFlagScan)) return;  // K0 linked the stream already
  const uint8_t* __restrict__ in = D.in;
  const uint64_t C = D.C;
  const uint32_t hdr = D.hdr;
  uint32_t* __restrict__ bitmap = S.bitmap;
  uint32_t* __restrict__ cum = S.cum;
  uint64_t* __restrict__ wexit = S.wexit;
  uint64_t* __restrict__ wtotal = S.wtotal;
  const uint32_t lane = threadIdx.x;
  const uint64_t base = hdr + (uint64_t)w * kWin;
  const uint32_t wl = (uint32_t)min((uint64_t)kWin, C - base);
  const uint32_t s = stage(b32, in, C, base, wl + 16, lane);
  for (uint32_t i = lane; i < kWin / 32; i += 64) bm[i] = 0;
  __syncthreads();
  // ---- lane 0's chain (from offset 0) in batches: its tags into the
  // bitmap, each tag's output count before it into cum (K2; the other starts
  // read it back where they meet the chain)
  uint64_t o = 0;
  const uint64_t exit0 = scan_walk<true>(b32, s, wl, 0, o, lane, bm, cum + base);
  const uint64_t total0 = o;
  __syncthreads();
  // ---- the other starts: each lane steps its own chain until it lands on
  // lane 0's (its exit is then lane 0's and its total follows from cum),
  // leaves the window, or passes kEarly bytes.  Starts on one chain that
  // never meets lane 0's (sorted keys: the chain that reads every copy's
  // offset byte as a 3-byte literal) stop at the same first position past
  // kEarly; each such position is walked to the end once, in batches.
  uint64_t p = lane;
  o = 0;
  bool alive = lane > 0 && p < wl;
  bool pending = false, met = false;
  uint64_t ex = lane == 0 ? exit0 : p, tot = lane == 0 ? total0 : 0;
  while (__ballot(alive)) {
    if (alive) {
      if (p < kEarly && ((bm[p >> 5] >> (p & 31)) & 1)) {
        ex = exit0;
        tot = o + total0;  // - cum[p], below
        met = true;
        alive = false;
      } else {
        const Tag t = lds_tag(b32, s + p, p);
        o += t.len;
        p = t.next;
        if (p >= wl) {
          ex = p;
          tot = o;
          alive = false;
        } else if (p >= kEarly) {
          pending = true;
          alive = false;
        }
      }
    }
  }
  // cum[p] where a start met the chain: this wave's own stores above, read
  // once they have landed in L2 (agent scope: not from a line the CU cached)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (met) tot -= __hip_atomic_load(cum + base + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint64_t pm = __ballot(pending); pm; pm = __ballot(pending)) {
    const uint64_t P = lane_of64(p, (uint32_t)__builtin_ctzll(pm));
    uint64_t oP = 0;
    const uint64_t eP = scan_walk<false>(b32, s, wl, P, oP, lane, nullptr, nullptr);
    if (pending && p == P) {
      ex = eP;
      tot = o + oP;
      pending = false;
    }
  }
  wexit[(size_t)w * kStarts + lane] = base + ex;
  wtotal[(size_t)w * kStarts + lane] = tot;
  __syncthreads();
  uint32_t* gb = bitmap + (size_t)w * (kWin / 32);
  for (uint32_t i = lane; i < kWin / 32; i += 64) gb[i] = bm[i];
}


// K3: validate copies and index the tag that starts each output fragment
__device__ void dindex_body(const SnappyDJobs& J, uint32_t ji, uint32_t w, uint32_t* b32) {
  const DJob& D = J.j[ji];
  const DScr S = dscr(J, D, ji);
  uint32_t* __restrict__ flags = S.flags;
  if (flags[1]) return;  // K0 walked and indexed the whole stream
  const uint8_t* __restrict__ in = D.in;
  const uint64_t C = D.C;
  const uint32_t hdr = D.hdr;
  const uint64_t* __restrict__ wentry = S.wentry;
  const uint64_t* __restrict__ woff = S.woff;
  uint64_t* __restrict__ fragpos = S.fragpos;
  const uint32_t lane = threadIdx.x;
  const uint64_t e = wentry[w];
  if (e == kNone || (*flags & kFlagInvalid)) return;
  const uint64_t base = hdr + (uint64_t)w * kWin;
  const uint32_t wl = (uint32_t)min((uint64_t)kWin, C - base);
  {  // the entry tag is a literal that leaves the window (a stored fragment): no staging
    const uint64_t o = woff[w];
    const Tag t = decode_tag(tag_bytes(in, C, e), e);
    if (t.lit && t.next >= base + wl) {
      if (lane == 0) {
        uint32_t fl = 0;
        if ((o & (kFrag - 1)) == 0) fragpos[o / kFrag] = e;
        if (o / kFrag != (o + t.len - 1) / kFrag) fl |= kFlagSerial;
        if (fl) atomicOr(flags, fl);
      }
      return;
    }
  }
  const uint32_t s = stage(b32, in, C, base, wl + 16, lane);
  __syncthreads();
  uint64_t p = e - base, o = woff[w];
  uint32_t fl = 0;
  while (p < wl) {
    // a batch (as in K1): lane l checks the chain's tag at p + l, if any
    const uint64_t pl = min(p + lane, (uint64_t)wl);
    const Tag tl = lds_tag(b32, s + pl, pl);
    const uint64_t adv = tl.next - pl;
    const uint64_t M = batch_mask((uint32_t)min(adv, (uint64_t)64), wl - p, ~0ull);
    const bool tag = (M >> lane) & 1;
    const uint64_t vo = o + wave_excl_sum(tag ? (uint32_t)min(tl.len, (uint64_t)64) : 0u, lane);
    bool inval = false, serial = false;
    if (tag) {
      if (!tl.lit) {
        if (tl.off == 0 || tl.off > vo) inval = true;
        else if (vo - tl.off < (vo & ~(uint64_t)(kFrag - 1))) serial = true;
      }
      if ((vo & (kFrag - 1)) == 0) fragpos[vo / kFrag] = base + pl;
      if (vo / kFrag != (vo + tl.len - 1) / kFrag) serial = true;
    }
    if (__ballot(inval)) fl |= kFlagInvalid;
    if (__ballot(serial)) fl |= kFlagSerial;
    const uint32_t last = 63 - __builtin_clzll(M);
    o = lane_of64(vo, last) + lane_of64(tl.len, last);
    p += last + lane_of64(adv, last);
  }
  if (fl && lane == 0) atomicOr(flags, fl);
}

// K1, K2 and K3 as three ordinary launches: stream order is the barrier
// between them (K1's tables feed K2, K2's window entries feed K3), so no
// workgroup ever waits for another and no co-residency is assumed.  Each
// returns at once when no stream of the batch needs it.
__device__ __forceinline__ void dslow_needs(const SnappyDJobs& J, bool& scan, bool& index) {
  scan = index = false;
  for (uint32_t i = 0; i < J.njobs; ++i) {
    const uint32_t f0 = J.ctrl[8 * i], f1 = J.ctrl[8 * i + 1];
    scan = scan || (f0 & kFlagScan);
    index = index || (!f1 && !(f0 & (kFlagInvalid | kFlagHeader)));
  }
}
// K1: windows of the streams K0 handed over
__global__ __launch_bounds__(64) void snappy_dscan(const SnappyDJobs J) {
  __shared__ uint32_t b32[(kWin + 32) / 4];
  __shared__ uint32_t bm[kWin / 32];
  bool scan, index;
  dslow_needs(J, scan, index);
  if (!scan) return;
  for (uint32_t w = blockIdx.x; w < J.nwin; w += gridDim.x) {
    const uint32_t ji = djob_win(J, w);
    dscan_body(J, ji, w - J.j[ji].win0, b32, bm);
  }
}
// K2: one workgroup per stream links its windows
__global__ __launch_bounds__(64) void snappy_dlink(const SnappyDJobs J) {
  __shared__ uint64_t lex[kLinkAhead * kStarts], ltot[kLinkAhead * kStarts];
  for (uint32_t ji = blockIdx.x; ji < J.njobs; ji += gridDim.x) {
    const DScr S = dscr(J, J.j[ji], ji);
    if (*S.flags & kFlagScan) {
      const DJob& D = J.j[ji];
      dlink_body(D.in, D.C, D.hdr, D.dsize, S.bitmap, S.cum, S.wexit, S.wtotal, D.nwin, S.wentry, S.woff, S.flags,
                 lex, ltot);
    }
  }
}
// K2p: the windows linked in parallel, for a stream whose chain enters every
// window at one of its first 64 bytes (tag-dense data: every tag is short).
// Window w's K1 tables are a function on entry offsets: F_w(l) = the next
// window's entry offset (or the stream's end), with T_w(l) output bytes; the
// chain's entries are the prefix compositions of these functions from
// window 0's offset 0.  Three launches compose them in two levels: K2a, one
// wave per block of kLinkPer windows, composes its block's function (lane l
// follows the chain entered at offset l of the block's first window: one lane
// permute per window); K2b, one workgroup per stream, composes the blocks'
// functions into at most kLinkMaxBlocks superblocks (a wave each), walks
// those along the true chain and then re-walks each superblock's blocks to
// record every block's entry; K2c, one wave per block again, re-walks the
// block's windows from its entry and records each window's entry and output
// offset -- what K2's one-chain walk records.  A chain that leaves a window
// anywhere else (a long literal, an entry past the first 64 bytes) leaves the
// stream to K2.  (Round 4: one workgroup per stream did both levels, 0.47 ms
// for 128 MiB of sorted keys in 8 KiB windows, its waves' table loads one
// memory latency per 8 windows.)
constexpr uint32_t kLinkWaves = 16;
constexpr uint32_t kLinkMaxBlocks = 128;
constexpr uint32_t kLinkPer = 16;
constexpr uint32_t kLinkEnd = 64, kLinkOdd = 65;  // F codes besides an entry offset 0..63
__device__ __forceinline__ uint32_t link_code(uint64_t x, uint32_t w, uint32_t nwin, uint32_t hdr, uint64_t C) {
  if (w + 1 == nwin) return x == C ? kLinkEnd : kLinkOdd;
  if (x < hdr) return kLinkOdd;
  const uint64_t r = x - hdr, w2 = r / kWin, off = r - w2 * kWin;
  return (w2 == (uint64_t)w + 1 && off < kStarts) ? (uint32_t)off : kLinkOdd;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)l, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)l, 64);
  return ((uint64_t)hi << 32) | lo;
}
// a stream's linker blocks: F (u8 codes) and T rows, each block's entry and
// output offset; after cum in the stream's scratch (djob_bytes)
struct LinkBlk {
  uint64_t *T, *out;
  uint32_t* entry;
  uint8_t* F;
};
__device__ __forceinline__ uint32_t link_nblk(uint32_t nwin) { return (nwin + kLinkPer - 1) / kLinkPer; }
__device__ __forceinline__ LinkBlk link_blk(const DJob& D, const DScr& S) {
  const size_t nb = link_nblk(D.nwin) + 1;
  LinkBlk B;
  B.T = reinterpret_cast<uint64_t*>(S.cum + ((D.C + 1) & ~(uint64_t)1));
  B.out = B.T + nb * kStarts;
  B.entry = reinterpret_cast<uint32_t*>(B.out + nb);
  B.F = reinterpret_cast<uint8_t*>(B.entry + nb);
  return B;
}
__device__ __forceinline__ uint32_t djob_blk(const SnappyDJobs& J, uint32_t b) {
  uint32_t i = 0;
  while (i + 1 < J.njobs && b >= J.j[i + 1].blk0) ++i;
  return i;
}
// The composition of windows [w0, w1)'s functions applied from entry `cur`
// (lane l: cur = l), with its output count; 8 windows' tables in flight.
__device__ __forceinline__ void link_compose(const DScr& S, uint32_t w0, uint32_t w1, uint32_t nwin, uint32_t hdr,
                                             uint64_t C, uint32_t lane, uint32_t& cur, uint64_t& acc) {
  for (uint32_t wc = w0; wc < w1; wc += 8) {
    uint64_t x[8], t[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t w = min(wc + k, w1 - 1);
      x[k] = S.wexit[(size_t)w * kStarts + lane];
      t[k] = S.wtotal[(size_t)w * kStarts + lane];
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      if (wc + k >= w1) break;
      const uint32_t code = link_code(x[k], wc + k, nwin, hdr, C);
      const uint32_t nc = (uint32_t)__shfl((int)code, (int)(cur & 63), 64);
      const uint64_t nt = shfl64(t[k], cur & 63);
      if (cur < kStarts) {
        acc += nt;
        cur = nc;
      } else {
        cur = kLinkOdd;  // (the end is only ever the last window's)
      }
    }
  }
}
// K2a: one wave per linker block
__global__ __launch_bounds__(64) void snappy_dlinka(const SnappyDJobs J) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t g = blockIdx.x; g < J.nblk; g += gridDim.x) {
    const uint32_t ji = djob_blk(J, g);
    const DJob& D = J.j[ji];
    const DScr S = dscr(J, D, ji);
    if (!(*S.flags & kFlagScan)) continue;
    const uint32_t b = g - D.blk0, w0 = b * kLinkPer, w1 = min(D.nwin, w0 + kLinkPer);
    if (w0 >= w1) continue;
    uint32_t cur = lane;
    uint64_t acc = 0;
    link_compose(S, w0, w1, D.nwin, D.hdr, D.C, lane, cur, acc);
    const LinkBlk B = link_blk(D, S);
    B.F[(size_t)b * kStarts + lane] = (uint8_t)cur;
    B.T[(size_t)b * kStarts + lane] = acc;
  }
}
// K2b: one workgroup per stream: the blocks' entries along the true chain
__global__ __launch_bounds__(kLinkWaves * 64) void snappy_dlinkb(const SnappyDJobs J) {
  __shared__ uint8_t sF[kLinkMaxBlocks][kStarts];
  __shared__ uint64_t sT[kLinkMaxBlocks][kStarts];
  __shared__ uint32_t s_entry[kLinkMaxBlocks];
  __shared__ uint64_t s_out[kLinkMaxBlocks];
  __shared__ uint32_t s_ok;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t ji = blockIdx.x; ji < J.njobs; ji += gridDim.x) {
    const DJob& D = J.j[ji];
    const DScr S = dscr(J, D, ji);
    if (!(*S.flags & kFlagScan)) continue;  // (uniform: every wave reads the same word)
    const uint32_t nb = link_nblk(D.nwin);
    if (nb == 0) continue;
    const LinkBlk B = link_blk(D, S);
    const uint32_t per = max(8u, (nb + kLinkMaxBlocks - 1) / kLinkMaxBlocks);
    const uint32_t ns = (nb + per - 1) / per;
    // ---- each superblock's composed function
    for (uint32_t sb = wave; sb < ns; sb += kLinkWaves) {
      const uint32_t b0 = sb * per, b1 = min(nb, b0 + per);
      uint32_t cur = lane;
      uint64_t acc = 0;
      for (uint32_t bc = b0; bc < b1; bc += 8) {
        uint32_t f[8];
        uint64_t t[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          const uint32_t b = min(bc + k, b1 - 1);
          f[k] = B.F[(size_t)b * kStarts + lane];
          t[k] = B.T[(size_t)b * kStarts + lane];
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          if (bc + k >= b1) break;
          const uint32_t nc = (uint32_t)__shfl((int)f[k], (int)(cur & 63), 64);
          const uint64_t nt = shfl64(t[k], cur & 63);
          if (cur < kStarts) {
            acc += nt;
            cur = nc;
          } else {
            cur = kLinkOdd;
          }
        }
      }
      sF[sb][lane] = (uint8_t)cur;
      sT[sb][lane] = acc;
    }
    __syncthreads();
    // ---- the superblocks' entries along the true chain
    if (threadIdx.x == 0) {
      uint32_t e = 0;
      uint64_t o = 0;
      for (uint32_t sb = 0; sb < ns && e < kStarts; ++sb) {
        s_entry[sb] = e;
        s_out[sb] = o;
        o += sT[sb][e];
        e = sF[sb][e];
      }
      s_ok = e == kLinkEnd ? (o == D.dsize ? 1u : 2u) : 0u;  // 0: K2 walks it
    }
    __syncthreads();
    const uint32_t ok = s_ok;
    if (ok == 1) {
      // ---- every block's entry, from its superblock's
      for (uint32_t sb = wave; sb < ns; sb += kLinkWaves) {
        const uint32_t b0 = sb * per, b1 = min(nb, b0 + per);
        uint32_t e = s_entry[sb];
        uint64_t o = s_out[sb];
        for (uint32_t bc = b0; bc < b1; bc += 8) {
          uint32_t f[8];
          uint64_t t[8];
#pragma unroll
          for (uint32_t k = 0; k < 8; ++k) {
            const uint32_t b = min(bc + k, b1 - 1);
            f[k] = B.F[(size_t)b * kStarts + lane];
            t[k] = B.T[(size_t)b * kStarts + lane];
          }
#pragma unroll
          for (uint32_t k = 0; k < 8; ++k) {
            if (bc + k >= b1) break;
            if (lane == 0) {
              B.entry[bc + k] = e;
              B.out[bc + k] = o;
            }
            o += lane_of64(t[k], e);
            e = lane_of32(f[k], e);
          }
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      S.flags[3] = ok == 1 ? 1u : 0u;  // K2c's cue
      if (ok) *S.flags = ok == 2 ? kFlagInvalid : 0;  // (K2 then skips the stream)
    }
    __syncthreads();
  }
}
// K2c: one wave per linker block of a stream K2b linked: its windows' entries
// K2c's work for linker block g of the union grid
__device__ void dlinkc_block(const SnappyDJobs& J, uint32_t g) {
  const uint32_t lane = threadIdx.x;
  const uint32_t ji = djob_blk(J, g);
  const DJob& D = J.j[ji];
  const DScr S = dscr(J, D, ji);
  if (S.flags[3] != 1) return;
  const uint32_t b = g - D.blk0, w0 = b * kLinkPer, w1 = min(D.nwin, w0 + kLinkPer);
  if (w0 >= w1) return;
  const LinkBlk B = link_blk(D, S);
  uint32_t e = B.entry[b];
  uint64_t o = B.out[b];
  const uint32_t nwin = D.nwin, hdr = D.hdr;
  for (uint32_t wc = w0; wc < w1; wc += 8) {
    uint64_t x[8], t[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t w = min(wc + k, w1 - 1);
      x[k] = S.wexit[(size_t)w * kStarts + lane];
      t[k] = S.wtotal[(size_t)w * kStarts + lane];
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      if (wc + k >= w1) break;
      const uint32_t w = wc + k;
      if (lane == 0) {
        S.wentry[w] = hdr + (uint64_t)w * kWin + e;
        S.woff[w] = o;
      }
      const uint32_t code = link_code(x[k], w, nwin, hdr, D.C);
      o += lane_of64(t[k], e);
      e = lane_of32(code, e);
    }
  }
}

__global__ __launch_bounds__(64) void snappy_dlinkc(const SnappyDJobs J) {
  for (uint32_t g = blockIdx.x; g < J.nblk; g += gridDim.x) dlinkc_block(J, g);
}
// K3: windows indexed (streams K0 did not walk to the end)
__global__ __launch_bounds__(64) void snappy_dindex(const SnappyDJobs J) {
  __shared__ uint32_t b32[(kWin + 32) / 4];
  bool scan, index;
  dslow_needs(J, scan, index);
  if (!scan && !index) return;
  for (uint32_t w = blockIdx.x; w < J.nwin; w += gridDim.x) {
    const uint32_t ji = djob_win(J, w);
    dindex_body(J, ji, w - J.j[ji].win0, b32);
  }
}

// A literal too long for the staging window, read straight into the LDS
// fragment: 16-byte LDS stores to the aligned chunks, each composed from the
// two aligned 16-byte source blocks it straddles; 8 chunks per lane in
// flight (8 KiB per memory latency for the wave), bytes at the edges.
__device__ void literal_to_lds(uint8_t* ob, uint32_t o, const uint8_t* __restrict__ in, uint64_t src, uint32_t L,
                               uint32_t lane) {
  constexpr uint32_t M = kRing - 1;  // ob is the ring: 16-byte chunks never straddle its end
  const uint32_t head = (16 - (o & 15)) & 15;
  if (head >= L) {
    for (uint32_t i = lane; i < L; i += 64) ob[(o + i) & M] = in[src + i];
    return;
  }
  if (lane < head) ob[(o + lane) & M] = in[src + lane];
  const uint32_t nc = (L - head) >> 4;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(in + src + head);
  typedef uint32_t V4 __attribute__((ext_vector_type(4)));
  const auto s16 = gbl<V4>(reinterpret_cast<const void*>(sp & ~(uintptr_t)15));  // global, not flat, loads
  const uint32_t sh = (uint32_t)(sp & 15);
  const uint32_t o16 = o + head;  // 16-aligned
  constexpr int U = 2;  // (registers: K4's occupancy)
  for (uint32_t c0 = 0; c0 < nc; c0 += U * 64) {
    uint4 lo[U], hi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + u * 64 + lane;
      V4 x = {0, 0, 0, 0};
      if (c < nc) x = s16[c];
      V4 y = x;
      if (c < nc && sh) y = s16[c + 1];
      lo[u] = make_uint4(x[0], x[1], x[2], x[3]);
      hi[u] = make_uint4(y[0], y[1], y[2], y[3]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + u * 64 + lane;
      if (c < nc) *reinterpret_cast<uint4*>(ob + ((o16 + 16 * c) & M)) = funnel16(lo[u], hi[u], sh);
    }
  }
  const uint32_t t0 = head + 16 * nc;
  if (lane < L - t0) ob[(o + t0 + lane) & M] = in[src + t0 + lane];
}

// The ring's bytes [from, to) of the fragment to d (from a multiple of 16 or
// to the fragment's end), by one wave.
__device__ __forceinline__ void ring_flush(const uint8_t* ring, uint8_t* __restrict__ d, uint32_t from, uint32_t to,
                                           uint32_t lane) {
  constexpr uint32_t M = kRing - 1;
  uint32_t i = from;
  if ((reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const uint32_t c1 = to >> 4;
    for (uint32_t c = (from >> 4) + lane; c < c1; c += 64)
      reinterpret_cast<uint4*>(d)[c] = *reinterpret_cast<const uint4*>(ring + ((16 * c) & M));
    i = max(from, c1 << 4);
  }
  for (i += lane; i < to; i += 64) d[i] = ring[i & M];
}
// Byte x of the fragment d, flushed from the ring by this wave before: an
// agent-scope load after the wave's stores have landed in L2 (a plain load
// could hit a line this CU cached while the byte was not yet written).
__device__ __forceinline__ uint8_t flushed_byte(const uint8_t* d, uint32_t x) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uintptr_t a = reinterpret_cast<uintptr_t>(d + x);
  const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return (uint8_t)(w >> (8 * (a & 3)));
}

// K5 body: the verdict; one-lane decode of valid streams K4 could not split
__device__ void dserial_body(const uint8_t* __restrict__ in, uint64_t C, uint32_t hdr, uint8_t* __restrict__ out) {
  uint64_t p = hdr, o = 0;
  while (p < C) {
    const Tag t = decode_tag(tag_bytes(in, C, p), p);
    if (t.lit) {
      for (uint64_t i = 0; i < t.len; ++i) out[o + i] = in[p + t.hl + i];
    } else {
      for (uint64_t i = 0; i < t.len; ++i) out[o + i] = out[o - t.off + i];
    }
    o += t.len;
    p = t.next;
  }
}
__device__ void dverdict(uint32_t f, uint64_t dsize, PubSlot* pub, uint32_t ticket) {
  if (pub) {
    pub_store(&pub->status, (int32_t)((f & kFlagHeader) ? kErrHeaderHint : (f & kFlagInvalid) ? kErrCheck : kOk));
    pub_store(&pub->size, (uint64_t)dsize);
    publish_ticket(pub, ticket);
  }
}

// K4: one workgroup per 64 KiB output fragment whose true position differs
// from the one K-spec assumed.  A fragment stored as one literal is copied by
// all 256 lanes; any other is decoded by wave 0 through an 8 KiB LDS ring of
// its output (tags and short literals read from a staged window of the
// compressed bytes; the ring flushed to the output as it fills).  The small
// LDS footprint and 64 registers let 8 workgroups share a CU: a decode is one
// wave's dependent chain of LDS and lane operations, so the chip's 2048
// decoders (one round for 128 MiB) set the rate -- with the whole fragment in
// LDS, 2 per CU, sorted keys decoded at 11.2 GB/s, with the ring 18.3
// (tools/ab_ring2.sh).  The last workgroup to finish gives the verdict (K5).
__global__ __launch_bounds__(256, 8) void snappy_dfrag(const SnappyDJobs J) {
  __shared__ uint32_t ob32[kRing / 4];
  __shared__ uint32_t ib32[(kInWin + 32) / 4];
  __shared__ uint32_t s_last;
  __shared__ FewLds F;
  __shared__ double s_lut[256];  // fused decode, nb = 1
  const uint32_t ji = djob_frag(J, blockIdx.x);
  const DJob& D = J.j[ji];
  const DScr S = dscr(J, D, ji);
  const uint32_t* __restrict__ flags = S.flags;
  const uint8_t* __restrict__ in = D.in;
  uint8_t* __restrict__ out = D.out;
  const uint64_t C = D.C, dsize = D.dsize;
  const uint32_t hdr = D.hdr, ticket = D.ticket;
  const uint32_t tid = threadIdx.x, k = blockIdx.x - D.fo0;
  const uint64_t o0 = (uint64_t)k * kFrag;
  const uint32_t end = (uint32_t)min((uint64_t)kFrag, dsize - o0);
  if (flags[2]) {  // K-spec decoded the whole stream and gave the verdict
    if (D.fv && end && !S.fdone[k]) {  // a fragment it placed as codes: their values
      dq_prepare(D, s_lut, tid);
      dq_frag<8>(D, out + o0, o0, end, s_lut, tid);
    }
    return;
  }
  const uint64_t* __restrict__ fragpos = S.fragpos;
  const uint64_t* __restrict__ specpos = S.specpos;
  PubSlot* pub = J.pub ? J.pub + D.slot : nullptr;
  const uint32_t f = flags[0];
  uint8_t* ob = reinterpret_cast<uint8_t*>(ob32);
  PSF_DTRACE(k, 0);
  const uint64_t p0 = end ? fragpos[k] : kNone;
  const bool redo = f == 0 && end && p0 != specpos[k];
  if (redo) {
    PSF_DTRACE(k, 1);
    const Tag t0 = decode_tag(tag_bytes(in, C, p0), p0);
    if (decode_few<4>(in, C, p0, end, out + o0, tid, F) != kNone) {
      // (a fragment of a few tags: done)
    } else if (t0.lit && t0.len == end) {
      copy_g2g<4>(out + o0, in + p0 + t0.hl, end, tid);
    } else {
      if (tid < 64) {
        const uint32_t lane = tid;
        constexpr uint32_t kSpan = kInWin + 16;  // staged bytes [wb, wb + kSpan)
        constexpr uint32_t RM = kRing - 1;
        uint8_t* const d = out + o0;
        uint64_t p = p0, wb = p0;
        uint32_t s = stage(ib32, in, C, wb, kSpan, lane);
        uint32_t o = 0, flushed = 0;
        const uint8_t* ibb = reinterpret_cast<const uint8_t*>(ib32);
        while (o < end) {
          if (o - flushed > kRingFlushAt) {
            ring_flush(ob, d, flushed, o & ~15u, lane);
            flushed = o & ~15u;
          }
          if (p + kBatchMargin > wb + kSpan) {
            wb = p;
            s = stage(ib32, in, C, wb, kSpan, lane);
          }
          // ---- a batch: the tags that start in [p, p + 64).  Every lane
          // decodes the tag that would start at p + lane; one scalar walk
          // marks the chain's tag starts (batch_mask) and one wave prefix sum
          // gives each its output offset; then every literal of the batch is
          // written at once (by the lane of its tag) and the copies one after
          // another in tag order (a
          // copy reads only output before it: earlier literals, done, and
          // earlier copies, done in order).  The walk stops at the
          // fragment's end and before a tag it does not take (a literal
          // longer than kBatchLit bytes); that one goes the single way below.
          {
            const uint32_t qb = s + (uint32_t)(p - wb);
            const Tag tl = lds_tag(ib32, qb + lane, p + lane);
            const uint32_t adv = (uint32_t)min(tl.next - (p + lane), (uint64_t)64);
            const uint32_t tlen = (uint32_t)min(tl.len, (uint64_t)64);
            const uint64_t M0 = batch_mask(adv, 64, __ballot(!tl.lit || tl.len <= kBatchLit));
            const bool tag0 = (M0 >> lane) & 1;
            const uint32_t vo = o + wave_excl_sum(tag0 ? tlen : 0u, lane);
            const uint64_t M = M0 & __ballot(vo < end);  // tags past the fragment's end are not its own
            if (M) {
              const bool tag = (M >> lane) & 1;
              const uint32_t last = 63 - __builtin_clzll(M);
              const uint32_t oend = lane_of32(vo, last) + lane_of32(tlen, last);
              if (tag && tl.lit) {
                const uint8_t* q = ibb + qb + lane + tl.hl;
                for (uint32_t j = 0; j < tlen; ++j) ob[(vo + j) & RM] = q[j];
              }
              for (uint64_t cm = __ballot(tag && !tl.lit); cm; cm &= cm - 1) {
                const uint32_t k = (uint32_t)__builtin_ctzll(cm);
                const uint32_t ko = lane_of32(vo, k), L = lane_of32(tlen, k), off = lane_of32(tl.off, k);
                if (off >= L) {
                  if (ko - off + kRing >= oend) {
                    if (lane < L) ob[(ko + lane) & RM] = ob[(ko - off + lane) & RM];
                  } else {  // older than the ring: flushed
                    const uint8_t b = flushed_byte(d, ko - off + min(lane, L - 1));
                    if (lane < L) ob[(ko + lane) & RM] = b;
                  }
                } else if (lane < L) {
                  ob[(ko + lane) & RM] = ob[(ko - off + lane % off) & RM];
                }
              }
              o = oend;
              p += last + lane_of32(adv, last);
              if (o >= end || last + lane_of32(adv, last) >= 64) continue;
            }
          }
          // ---- one tag the general way (a step of its own)
          if (o - flushed > kRingFlushAt) {
            ring_flush(ob, d, flushed, o & ~15u, lane);
            flushed = o & ~15u;
          }
          const Tag t = lds_tag(ib32, s + (p - wb), p);
          const uint32_t L = (uint32_t)t.len;
          if (t.lit) {
            const uint64_t src = p + t.hl;
            if (src + L > wb + kSpan && L <= kInWin) {
              wb = src;
              s = stage(ib32, in, C, wb, kSpan, lane);
            }
            const bool staged = src + L <= wb + kSpan;
            for (uint32_t q0 = 0; q0 < L; q0 += kRingStep) {  // pieces of one step each
              const uint32_t n = min(L - q0, kRingStep), oq = o + q0;
              if (oq - flushed > kRingFlushAt) {
                ring_flush(ob, d, flushed, oq & ~15u, lane);
                flushed = oq & ~15u;
              }
              if (staged) {
                const uint8_t* q = reinterpret_cast<const uint8_t*>(ib32) + s + (src - wb) + q0;
                for (uint32_t i = lane; i < n; i += 64) ob[(oq + i) & RM] = q[i];
              } else {
                literal_to_lds(ob, oq, in, src + q0, n, lane);
              }
            }
          } else if (t.off >= L) {  // (L <= 64)
            if (o - t.off + kRing >= o + L) {
              if (lane < L) ob[(o + lane) & RM] = ob[(o - t.off + lane) & RM];
            } else {
              const uint8_t b = flushed_byte(d, o - t.off + min(lane, L - 1));
              if (lane < L) ob[(o + lane) & RM] = b;
            }
          } else if (lane < L) {
            ob[(o + lane) & RM] = ob[(o - t.off + lane % t.off) & RM];
          }
          o += L;
          p = t.next;
        }
        ring_flush(ob, d, flushed, end, lane);
      }
    }
  }
  if (D.fv && f == 0 && end && (redo || !S.fdone[k])) {  // values of the codes placed here or by K-spec
    __syncthreads();
    dq_prepare(D, s_lut, tid);
    dq_frag<8>(D, out + o0, o0, end, s_lut, tid);
  }
  PSF_DTRACE(k, 2);
  if (!last_block(S.ctr + 2, D.nfo ? D.nfo : 1, &s_last)) return;
  if (f == kFlagSerial) {
    if (tid == 0) dserial_body(in, C, hdr, out);
    if (D.fv) {
      __syncthreads();
      dq_prepare(D, s_lut, tid);
      for (uint64_t o = 0; o < dsize; o += kFrag) dq_frag<8>(D, out + o, o, (uint32_t)min((uint64_t)kFrag, dsize - o), s_lut, tid);
    }
    __syncthreads();
  }
  if (tid == 0) dverdict(f, dsize, pub, ticket);
}

}  // namespace

size_t snappy_max_compressed(size_t n) { return 32 + n + n / 6; }

// scratch: tag slots | finfo | offset (one each per fragment) | in_place (per
// job) | stash (per fragment)
size_t snappy_compress_batch_scratch(const SnappyCJob* jobs, int njobs) {
  size_t nfrag = 0;
  for (int i = 0; i < njobs; ++i) nfrag += (jobs[i].n + kFrag - 1) / kFrag;
  return nfrag * kSnappyFragOut + nfrag * 16 + 4 * kSnappyBatchMax + nfrag * kStash + 64;
}

size_t snappy_compress_scratch(size_t n) {
  const SnappyCJob j{nullptr, n, nullptr, 0, 0};
  return snappy_compress_batch_scratch(&j, 1);
}

int snappy_compress_batch_launch(const SnappyCJob* jobs, int njobs, void* scratch, hipStream_t st, Profiler* prof,
                                 PubSlot* pub_base) {
  if (njobs <= 0 || njobs > kSnappyBatchMax) return kErrArg;
  SnappyCJobs K{};
  K.pub = pub_base;
  K.njobs = (uint32_t)njobs;
  double bytes = 0;
  for (int i = 0; i < njobs; ++i) {
    const SnappyCJob& q = jobs[i];
    if (q.n == 0 || q.n > 0xffffffffull) return kErrArg;
    CJob& c = K.j[i];
    c.in = static_cast<const uint8_t*>(q.in);
    c.dst = static_cast<uint8_t*>(q.out);
    c.n = q.n;
    c.frag0 = K.nfrag;
    c.nfrag = (uint32_t)((q.n + kFrag - 1) / kFrag);
    c.hdr = 1;
    for (uint64_t v = q.n; v >= 128; v >>= 7) ++c.hdr;
    c.slot = (uint32_t)q.slot;
    c.ticket = q.ticket;
    c.stored = q.stored ? 1u : 0u;
    K.nfrag += c.nfrag;
    bytes += (double)q.n;
  }
  uint8_t* s = static_cast<uint8_t*>(scratch);
  uint8_t* p = s + (size_t)K.nfrag * kSnappyFragOut;
  K.finfo = reinterpret_cast<uint64_t*>(p);
  K.offset = K.finfo + K.nfrag;
  K.in_place = reinterpret_cast<uint32_t*>(K.offset + K.nfrag);  // (every word the kernels read is written first in the chain)
  K.stash = reinterpret_cast<uint8_t*>(K.in_place + kSnappyBatchMax);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return kErrHip;
  // K-parse: persistent workgroups, one per CU (the parse's LDS footprint allows no more)
  const uint32_t grid = K.nfrag < (uint32_t)cus ? K.nfrag : (uint32_t)cus;
  ProfScope ps(prof, kKSnappyCompress, st, bytes);
  uint32_t longest = 0;
  for (int i = 0; i < njobs; ++i) longest = std::max(longest, K.j[i].nfrag);
  if (longest <= kInlineScan) K.offset = nullptr;  // K-place sums the lengths itself
  hipLaunchKernelGGL(snappy_parse, dim3(grid), dim3(kCThreads), 0, st, K, s);
  if (K.offset) hipLaunchKernelGGL(snappy_scan, dim3(K.njobs), dim3(kScanT), 0, st, K);
  hipLaunchKernelGGL(snappy_place, dim3(K.nfrag), dim3(kPlaceT), 0, st, K, s);
  return launch_status();
}

int snappy_compress_launch(const void* in, size_t n, void* out, void* scratch, hipStream_t st, Profiler* prof,
                           PubSlot* pub, uint32_t ticket) {
  const SnappyCJob j{in, n, out, 0, ticket};
  return snappy_compress_batch_launch(&j, 1, scratch, st, prof, pub);
}

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// one stream's index arrays (DScr)
static size_t djob_bytes(size_t C, size_t dsize) {
  const size_t nwin = (C + kWin - 1) / kWin + 1;
  const size_t nfo = (dsize + kFrag - 1) / kFrag + 1;
  const size_t nblk = (nwin + kLinkPer - 1) / kLinkPer + 1;  // linker blocks (LinkBlk)
  return align256(nwin * (kWin / 8) + C * 4 + nwin * 8 * (2 * kStarts + 2) + 4 * nfo * 8 + 64 +
                  nblk * (kStarts * 9 + 12) + 16);
}

size_t snappy_uncompress_batch_scratch(const SnappyDJob* jobs, int njobs) {
  size_t b = align256((size_t)njobs * 32 + 4);
  for (int i = 0; i < njobs; ++i) b += djob_bytes(jobs[i].c, jobs[i].dsize);
  return b;
}

bool snappy_dequant_ok(const SnappyDequant& dq, size_t dsize) {
  return dq.values && (dq.nb == 1 || dq.nb == 2) && (dq.value_type == kFloat || dq.value_type == kDouble) &&
         dsize > 0 && dsize % (size_t)dq.nb == 0 && (reinterpret_cast<uintptr_t>(dq.values) & 15) == 0;
}

size_t snappy_uncompress_scratch(size_t C, size_t dsize) { return align256(32 + 4) + djob_bytes(C, dsize); }

// Launches for the whole batch: K-spec (+ K0 in one more workgroup per
// stream), K1, K2, K3 (one launch each), K4 (+ K5 in each stream's last
// workgroup).  On streams
// of stored fragments K-spec decodes everything and the others return at once.
static int launch_tail(const SnappyDJobs& K, hipStream_t st);

int snappy_uncompress_batch_launch(const SnappyDJob* jobs, int njobs, void* scratch, hipStream_t st,
                                   Profiler* prof, PubSlot* pub_base, const ZeroPair& z, SnappyTail* tail) {
  if (njobs <= 0 || njobs > kSnappyBatchMax) return kErrArg;
  SnappyDJobs K{};
  uint8_t* s = static_cast<uint8_t*>(scratch);
  K.ctrl = reinterpret_cast<uint32_t*>(s);  // 8 words per stream, then one spare word
  K.pub = pub_base;
  K.njobs = (uint32_t)njobs;
  uint8_t* data = s + align256((size_t)njobs * 32 + 4);
  double bytes = 0;
  for (int i = 0; i < njobs; ++i) {
    const SnappyDJob& q = jobs[i];
    if (q.hdr == 0 || q.hdr > q.c || q.hdr > 5) return kErrArg;
    DJob& D = K.j[i];
    D.in = static_cast<const uint8_t*>(q.in);
    D.out = static_cast<uint8_t*>(q.out);
    D.scratch = data;
    D.C = q.c;
    D.dsize = q.dsize;
    D.hdr = q.hdr;
    D.nwin = (uint32_t)((q.c - q.hdr + kWin - 1) / kWin);
    D.nfo = (uint32_t)((q.dsize + kFrag - 1) / kFrag);
    D.fo0 = K.nfo1;
    D.win0 = K.nwin;
    D.blk0 = K.nblk;
    D.slot = (uint32_t)q.slot;
    D.ticket = q.ticket;
    if (q.dq.values) {
      if (!snappy_dequant_ok(q.dq, q.dsize)) return kErrArg;
      D.fv = q.dq.values;
      D.frange = q.dq.range;
      D.fratio = ff_ratio(q.dq.nb);
      D.fmn = q.dq.mn;
      D.fmx = q.dq.mx;
      D.fnb = (uint32_t)q.dq.nb;
      D.fdbl = q.dq.value_type == kDouble ? 1u : 0u;
    }
    K.nfo1 += D.nfo ? D.nfo : 1;  // an empty output still takes one workgroup (header check, verdict)
    K.nwin += D.nwin;
    K.nblk += (D.nwin + kLinkPer - 1) / kLinkPer;
    data += djob_bytes(q.c, q.dsize);
    bytes += (double)q.c +
             (q.dq.values ? (double)(q.dsize / q.dq.nb) * (q.dq.value_type == kDouble ? 8 : 4) : (double)q.dsize);
  }
  const size_t zneed = (size_t)njobs * 32 + 4;
  if (z.cur && zneed <= z.bytes) {  // the context's region the previous launch cleared
    K.ctrl = static_cast<uint32_t*>(z.cur);
    K.znext = static_cast<uint32_t*>(z.next);
    K.zwords = (uint32_t)(z.bytes / 4);
  } else if (hipMemsetAsync(K.ctrl, 0, zneed, st) != hipSuccess) {
    return kErrHip;
  }
  if (tail) {
    std::shared_ptr<SnappyDJobs> keep = std::make_shared<SnappyDJobs>(K);
    {
      ProfScope ps(prof, kKSnappyDecompress, st, bytes);
      hipLaunchKernelGGL(snappy_dspec, dim3(K.nfo1 + K.njobs), dim3(256), 0, st, K);
    }
    tail->jobs = keep;
    tail->pending = true;
    return launch_status();
  }
  ProfScope ps(prof, kKSnappyDecompress, st, bytes);
  hipLaunchKernelGGL(snappy_dspec, dim3(K.nfo1 + K.njobs), dim3(256), 0, st, K);
  return launch_tail(K, st);
}

// PSF_LINK_PARALLEL (A/B knob, tools/): 0 leaves every stream to K2's walk
static bool link_parallel() {
  static const bool on = [] {
    const char* e = getenv("PSF_LINK_PARALLEL");
    return !(e && *e == '0');
  }();
  return on;
}

// K1-K3 and K4 (+ K5) of a batch whose fast path has run.  K2a / K2c / K3
// loop over their blocks / windows on grids capped at about twice what the
// chip holds at once (K3: 32 waves per CU), so a stream they have nothing to
// do for (stored fragments: K-spec decoded it) costs a few thousand
// workgroups, not one per 4 KiB window.  K1 keeps one workgroup per window:
// with a capped grid each workgroup's share of windows is fixed and the
// tag-dense scan lost its dynamic balance (sorted keys, 128 MiB: K1 0.83 ->
// 0.95 ms at twice its residency, 1.04 at once; tools/ab_dec.sh abcap / abcap2).
constexpr uint32_t kIndexGrid = 16384, kLinkGrid = 1024;
static int launch_tail(const SnappyDJobs& K, hipStream_t st) {
  if (K.nwin) {
    hipLaunchKernelGGL(snappy_dscan, dim3(K.nwin), dim3(64), 0, st, K);
    if (link_parallel()) {
      hipLaunchKernelGGL(snappy_dlinka, dim3(min(K.nblk, kLinkGrid)), dim3(64), 0, st, K);
      hipLaunchKernelGGL(snappy_dlinkb, dim3(K.njobs), dim3(kLinkWaves * 64), 0, st, K);
      hipLaunchKernelGGL(snappy_dlinkc, dim3(min(K.nblk, kLinkGrid)), dim3(64), 0, st, K);
    }
    hipLaunchKernelGGL(snappy_dlink, dim3(K.njobs), dim3(64), 0, st, K);
    hipLaunchKernelGGL(snappy_dindex, dim3(min(K.nwin, kIndexGrid)), dim3(64), 0, st, K);
  }
  hipLaunchKernelGGL(snappy_dfrag, dim3(K.nfo1), dim3(256), 0, st, K);
  return launch_status();
}

// (not bracketed by the profiler: the batch's bytes were counted with its fast
// path, whose launch the bench times)
int snappy_uncompress_tail_launch(SnappyTail* tail, hipStream_t st) {
  if (!tail || !tail->pending || !tail->jobs) return kErrArg;
  tail->pending = false;
  const SnappyDJobs& K = *static_cast<const SnappyDJobs*>(tail->jobs.get());
  return launch_tail(K, st);
}

int snappy_uncompress_launch(const void* in, size_t C, uint32_t hdr, size_t dsize, void* out, void* scratch,
                             hipStream_t st, Profiler* prof, PubSlot* pub, uint32_t ticket) {
  const SnappyDJob j{in, C, hdr, dsize, out, 0, ticket};
  return snappy_uncompress_batch_launch(&j, 1, scratch, st, prof, pub, ZeroPair{});
}

}  // namespace psf

#ifdef PSF_SNAPPY_TRACE
// diagnostic builds: copy the compress kernel's phase timestamps out
extern "C" int psf_debug_dfrag_trace(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(psf::g_dfrag_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -4;
}
extern "C" int psf_debug_snappy_trace(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(psf::g_snappy_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -4;
}
#endif
