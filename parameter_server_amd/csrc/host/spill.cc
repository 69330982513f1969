// The cross-range spill of the multi-GPU split, host side.
//
// The reference sends every per-server slice of a message as its own ZeroMQ
// multipart message [Task][key][value...] (executor.cc:135-146 ->
// Van::Send, van.cc:122-191) and the receiver rebuilds a Message from the
// frames (Van::Recv, van.cc:193-269).  Here the slices one rank sends in a
// step travel in ONE all-to-all-v over RCCL: SpillPlan lays every slice out
// in the per-peer segment of a single send buffer, and unpack() rebuilds the
// messages over the receive buffer, zero-copy, as Van::Recv does over zmq
// frames.
//
// Segment of one peer (every size a multiple of 256, so frames stay aligned):
//   [meta][payload]
//   meta    = records, one per message:
//             u32 magic 'PSSP', u32 server, u32 task_len, u32 nframes,
//             u64 frame_len[nframes], task bytes (the Task frame, protobuf wire
//             format), zero padding to 8
//   payload = the message's frames in order -- the key frame when the Task
//             has has_key, then one frame per value_type entry -- each at a
//             256-byte aligned offset
// The host builds the meta records (the Task is serialised here, as Van::Send
// does) and one gather launch assembles meta + frames in HBM.
#include "spill.h"

#include <string.h>

#include <algorithm>

#include "wire.h"

namespace psf {

namespace {
constexpr uint32_t kMagic = 0x50535350u;  // 'PSSP'
inline uint64_t up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
template <typename T> void put(std::vector<uint8_t>* b, T v) {
  const size_t at = b->size();
  b->resize(at + sizeof(T));
  memcpy(b->data() + at, &v, sizeof(T));
}
}  // namespace

SpillPlan::SpillPlan(Context* ctx, Message* const* msgs, const int* dest, const int* server, int n, int world)
    : ctx_(ctx) {
  if (world <= 0) throw CheckError(kErrArg, "world must be positive");
  sizes_.assign(2 * (size_t)world, 0);
  std::vector<std::vector<int>> by_rank(world);
  for (int i = 0; i < n; ++i) {
    if (dest[i] < 0 || dest[i] >= world) throw CheckError(kErrArg, "destination rank out of range");
    by_rank[dest[i]].push_back(i);
  }
  // pass 1: meta records of every rank (host blob) and the payload layout
  struct Frame { Buffer b; int rank; uint64_t off; };
  std::vector<Frame> frames;
  std::vector<uint64_t> meta_at(world);
  for (int r = 0; r < world; ++r) {
    meta_at[r] = blob_.size();
    uint64_t pay = 0;
    for (int i : by_rank[r]) {
      Message& m = *msgs[i];
      Task t = m.task;
      t.has_key = !m.key.empty();  // van.cc:131-137
      const std::string tb = serialize_task(t);
      std::vector<const Buffer*> fr;
      if (t.has_key) fr.push_back(&m.key);
      if (m.value.size() != t.value_type.size())
        throw CheckError(kErrCheck, "value frames != value_type entries");
      for (const Buffer& v : m.value) fr.push_back(&v);
      put<uint32_t>(&blob_, kMagic);
      put<uint32_t>(&blob_, (uint32_t)server[i]);
      put<uint32_t>(&blob_, (uint32_t)tb.size());
      put<uint32_t>(&blob_, (uint32_t)fr.size());
      for (const Buffer* b : fr) put<uint64_t>(&blob_, b->bytes);
      blob_.insert(blob_.end(), tb.begin(), tb.end());
      blob_.resize(up(blob_.size(), 8), 0);
      for (const Buffer* b : fr) {
        if (b->bytes) frames.push_back(Frame{*b, r, pay});
        pay += up(b->bytes, 256);
      }
    }
    blob_.resize(meta_at[r] + up(blob_.size() - meta_at[r], 256), 0);
    sizes_[2 * r] = (int64_t)(blob_.size() - meta_at[r]);
    sizes_[2 * r + 1] = (int64_t)pay;
  }
  // segment starts in the send buffer
  std::vector<uint64_t> seg(world + 1, 0);
  for (int r = 0; r < world; ++r) seg[r + 1] = seg[r] + (uint64_t)sizes_[2 * r] + (uint64_t)sizes_[2 * r + 1];
  total_ = seg[world];
  // pass 2: the copies; host-resident frames are staged behind the meta blob
  for (int r = 0; r < world; ++r)
    if (sizes_[2 * r]) copies_.push_back(Copy{nullptr, meta_at[r], seg[r], (uint64_t)sizes_[2 * r]});
  for (const Frame& f : frames) {
    const uint64_t dst = seg[f.rank] + (uint64_t)sizes_[2 * f.rank] + f.off;
    if (f.b.loc == Loc::kHost || ctx->device() < 0) {
      const uint64_t at = up(blob_.size(), 16);
      blob_.resize(at + f.b.bytes, 0);
      memcpy(blob_.data() + at, f.b.ptr, f.b.bytes);
      copies_.push_back(Copy{nullptr, at, dst, f.b.bytes});
    } else {
      copies_.push_back(Copy{f.b.ptr, 0, dst, f.b.bytes});
      keep_.push_back(f.b);  // alive until the gather has run
    }
  }
}

void SpillPlan::fill(void* sendbuf) {
  uint8_t* out = static_cast<uint8_t*>(sendbuf);
  if (total_ && !out) throw CheckError(kErrArg, "send buffer is null");
  if (ctx_->device() < 0) {  // host-only context (CPU exchange over gloo)
    for (const Copy& c : copies_) memcpy(out + c.dst_off, c.src ? c.src : blob_.data() + c.blob_off, c.len);
    return;
  }
  if (copies_.empty()) return;
  // one upload: [SpillCopy table | blob], then one gather launch
  const size_t tbl = up(copies_.size() * sizeof(SpillCopy), 256);
  Buffer d = ctx_->alloc(tbl + blob_.size());
  std::vector<uint8_t> host(tbl + blob_.size(), 0);
  uint64_t chunk = 0;
  SpillCopy* sc = reinterpret_cast<SpillCopy*>(host.data());
  for (size_t k = 0; k < copies_.size(); ++k) {
    const Copy& c = copies_[k];
    sc[k] = SpillCopy{c.src ? c.src : d.ptr + tbl + c.blob_off, c.dst_off, c.len, chunk};
    chunk += (c.len + kSpillChunk - 1) / kSpillChunk;
  }
  memcpy(host.data() + tbl, blob_.data(), blob_.size());
  hipStream_t st = ctx_->stream();
  PSF_HIP_CHECK(hipMemcpyAsync(d.ptr, host.data(), host.size(), hipMemcpyHostToDevice, st));
  int s = spill_gather_launch(reinterpret_cast<const SpillCopy*>(d.ptr), (int)copies_.size(), chunk, out, st);
  if (s != kOk) throw CheckError(s, "spill gather launch failed");
  keep_.push_back(d);  // freed stream-ordered after the launch
  keep_.clear();
}

Buffer own_copy(Context* ctx, const void* p, size_t bytes) {
  if (ctx->device() >= 0) {
    Buffer b = ctx->alloc(bytes);
    if (bytes) PSF_HIP_CHECK(hipMemcpyAsync(b.ptr, p, bytes, hipMemcpyDeviceToDevice, ctx->stream()));
    return b;
  }
  Buffer b;
  b.loc = Loc::kHost;
  b.bytes = bytes;
  if (!bytes) return b;
  uint8_t* q = new uint8_t[bytes];
  memcpy(q, p, bytes);
  b.owner = std::shared_ptr<void>(q, [](void* v) { delete[] static_cast<uint8_t*>(v); });
  b.ptr = q;
  return b;
}

int spill_unpack(Context* ctx, const Buffer& rbuf, int world, const int64_t* sizes, std::vector<Message>* out,
                 std::vector<int>* servers) {
  out->clear();
  servers->clear();
  const uint8_t* recv = rbuf.ptr;
  uint64_t at = 0;
  std::vector<uint8_t> meta;
  for (int s = 0; s < world; ++s) {
    const uint64_t mlen = (uint64_t)sizes[2 * s], plen = (uint64_t)sizes[2 * s + 1];
    if ((mlen | plen) & 255) throw CheckError(kErrCheck, "spill segment sizes must be 256-aligned");
    const uint8_t* seg = recv + at;
    const uint8_t* pay = seg + mlen;
    at += mlen + plen;
    if (!mlen) continue;
    meta.resize(mlen);
    if (ctx->device() < 0) {
      memcpy(meta.data(), seg, mlen);
    } else {
      PSF_HIP_CHECK(hipMemcpyAsync(meta.data(), seg, mlen, hipMemcpyDeviceToHost, ctx->stream()));
      ctx->sync();
    }
    uint64_t p = 0, poff = 0;
    auto need = [&](uint64_t k) {
      if (p + k > mlen) throw CheckError(kErrCheck, "truncated spill record");
    };
    while (p + 16 <= mlen) {
      uint32_t h[4];
      memcpy(h, meta.data() + p, 16);
      if (h[0] == 0) break;  // padding
      if (h[0] != kMagic) throw CheckError(kErrCheck, "bad spill record");
      p += 16;
      need(8ull * h[3] + h[2]);
      std::vector<uint64_t> fl(h[3]);
      memcpy(fl.data(), meta.data() + p, 8ull * h[3]);
      p += 8ull * h[3];
      out->emplace_back();
      Message& m = out->back();
      parse_task(meta.data() + p, h[2], &m.task);
      p = up(p + h[2], 8);
      size_t f = 0;
      auto frame = [&]() {
        Buffer b;
        b.owner = rbuf.owner;
        b.bytes = fl[f];
        b.ptr = b.bytes ? const_cast<uint8_t*>(pay + poff) : nullptr;
        if (!b.bytes) b.owner.reset();
        b.loc = ctx->device() < 0 ? Loc::kHost : Loc::kDevice;
        poff += up(fl[f], 256);
        if (poff > plen) throw CheckError(kErrCheck, "spill frames overrun the payload");
        ++f;
        return b;
      };
      const size_t want = (m.task.has_key ? 1 : 0) + m.task.value_type.size();
      if (fl.size() != want) throw CheckError(kErrCheck, "frame count != has_key + value_type entries");
      if (m.task.has_key) {
        m.key = frame();  // Van::Recv: the first data frame is the key (van.cc:240-250)
        m.key_frame_seen = true;
      }
      while (f < fl.size()) m.value.push_back(frame());
      servers->push_back((int)h[1]);
    }
  }
  return (int)out->size();
}

}  // namespace psf
