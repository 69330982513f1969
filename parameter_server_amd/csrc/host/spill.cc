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
//
// host_meta (the native exchange, exchange.h): the records stay on the host
// and travel through the node's mailbox; a rank's data segment is
//   [frames, 256-aligned as above][side-info block: 16 bytes per record]
// and a record is
//   u32 magic 'PSSN', u32 server, u32 task_len, u32 nframes, u32 nside, u32 0,
//   u64 frame_len[nframes], nside x {u16 filter, u16 fixed_point, u8 min,
//   u8 max, u16 0, u32 slot}, task bytes, zero padding to 8
// where each side entry names a FIXING_FLOAT fixed_point whose computed
// {min, max, status} (a RangeBatch record, context.h) sits in slot `slot` of
// the block: the Task travels without them (as if unset) and the receiver's
// decode reads them on the device -- no host wait for the encode.
#include "spill.h"

#include <string.h>

#include <algorithm>

#include "wire.h"

namespace psf {

namespace {
constexpr uint32_t kMagic = 0x50535350u;      // 'PSSP'
constexpr uint32_t kMagicHost = 0x5053534Eu;  // 'PSSN'
inline uint64_t up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
template <typename T> void put(std::vector<uint8_t>* b, T v) {
  const size_t at = b->size();
  b->resize(at + sizeof(T));
  memcpy(b->data() + at, &v, sizeof(T));
}
}  // namespace

SpillPlan::SpillPlan(Context* ctx, Message* const* msgs, const int* dest, const int* server, int n, int world,
                     bool host_meta)
    : ctx_(ctx) {
  if (world <= 0) throw CheckError(kErrArg, "world must be positive");
  sizes_.assign(2 * (size_t)world, 0);
  meta_at_.assign(world, 0);
  std::vector<std::vector<int>> by_rank(world);
  for (int i = 0; i < n; ++i) {
    if (dest[i] < 0 || dest[i] >= world) throw CheckError(kErrArg, "destination rank out of range");
    by_rank[dest[i]].push_back(i);
  }
  // pass 1: meta records of every rank (host blob) and the payload layout
  struct Frame { Buffer b; int rank; uint64_t off; };
  struct Side { const uint8_t* src; int rank; uint64_t slot; };
  std::vector<Frame> frames;
  std::vector<Side> sides;
  std::vector<uint64_t> side_at(world, 0);
  for (int r = 0; r < world; ++r) {
    meta_at_[r] = blob_.size();
    uint64_t pay = 0, nside = 0;
    for (int i : by_rank[r]) {
      Message& m = *msgs[i];
      Task t = m.task;
      t.has_key = !m.key.empty();  // van.cc:131-137
      // host_meta: device-resident side-info leaves the Task copy and rides
      // in the data segment
      struct Ent { uint16_t f, k; uint8_t mn, mx; uint16_t z; uint32_t slot; };
      std::vector<Ent> ents;
      if (host_meta && ctx->device() >= 0) {
        for (size_t f = 0; f < t.filter.size(); ++f) {
          FilterConfig& fc = t.filter[f];
          if (fc.type != FilterConfig::FIXING_FLOAT) continue;
          for (size_t k = 0; k < fc.fixed_point.size(); ++k) {
            FixedFloatConfig& fp = fc.fixed_point[k];
            if (!fp.pending || fp.pending->ctx != ctx || fp.pending->done) continue;
            if (f > 0xffff || k > 0xffff) throw CheckError(kErrArg, "too many filters to spill");
            ents.push_back(Ent{(uint16_t)f, (uint16_t)k, (uint8_t)fp.pending_min, (uint8_t)fp.pending_max, 0,
                               (uint32_t)nside});
            sides.push_back(Side{reinterpret_cast<const uint8_t*>(fp.device_range()), r, nside});
            ++nside;
            fp.pending.reset();  // (the copy's only: the message keeps its own)
            fp.pending_idx = -1;
            fp.pending_min = fp.pending_max = false;
          }
        }
      }
      const std::string tb = serialize_task(t);
      std::vector<const Buffer*> fr;
      if (t.has_key) fr.push_back(&m.key);
      if (m.value.size() != t.value_type.size())
        throw CheckError(kErrCheck, "value frames != value_type entries");
      for (const Buffer& v : m.value) fr.push_back(&v);
      put<uint32_t>(&blob_, host_meta ? kMagicHost : kMagic);
      put<uint32_t>(&blob_, (uint32_t)server[i]);
      put<uint32_t>(&blob_, (uint32_t)tb.size());
      put<uint32_t>(&blob_, (uint32_t)fr.size());
      if (host_meta) {
        put<uint32_t>(&blob_, (uint32_t)ents.size());
        put<uint32_t>(&blob_, 0u);
      }
      for (const Buffer* b : fr) put<uint64_t>(&blob_, b->bytes);
      for (const Ent& e : ents) {
        put<uint16_t>(&blob_, e.f);
        put<uint16_t>(&blob_, e.k);
        put<uint8_t>(&blob_, e.mn);
        put<uint8_t>(&blob_, e.mx);
        put<uint16_t>(&blob_, 0);
        put<uint32_t>(&blob_, e.slot);
      }
      blob_.insert(blob_.end(), tb.begin(), tb.end());
      blob_.resize(up(blob_.size(), 8), 0);
      for (const Buffer* b : fr) {
        if (b->bytes) frames.push_back(Frame{*b, r, pay});
        pay += up(b->bytes, 256);
      }
    }
    if (host_meta) {
      side_at[r] = pay;
      pay += up(16 * nside, 256);
      sizes_[2 * r] = (int64_t)(blob_.size() - meta_at_[r]);
    } else {
      blob_.resize(meta_at_[r] + up(blob_.size() - meta_at_[r], 256), 0);
      sizes_[2 * r] = (int64_t)(blob_.size() - meta_at_[r]);
    }
    sizes_[2 * r + 1] = (int64_t)pay;
  }
  // segment starts in the send buffer (host_meta: data only)
  seg_.assign(world + 1, 0);
  for (int r = 0; r < world; ++r)
    seg_[r + 1] = seg_[r] + (host_meta ? 0 : (uint64_t)sizes_[2 * r]) + (uint64_t)sizes_[2 * r + 1];
  total_ = seg_[world];
  // pass 2: the copies; host-resident frames are staged behind the meta blob
  if (!host_meta)
    for (int r = 0; r < world; ++r)
      if (sizes_[2 * r]) copies_.push_back(Copy{nullptr, meta_at_[r], seg_[r], (uint64_t)sizes_[2 * r]});
  for (const Frame& f : frames) {
    const uint64_t dst = seg_[f.rank] + (host_meta ? 0 : (uint64_t)sizes_[2 * f.rank]) + f.off;
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
  for (const Side& sd : sides) copies_.push_back(Copy{sd.src, 0, seg_[sd.rank] + side_at[sd.rank] + 16 * sd.slot, 16});
  // the side-info records stay alive with the messages that point into them
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

void spill_unpack_host(Context* ctx, const uint8_t* meta, uint64_t mlen, const Buffer& rbuf, uint64_t pay_at,
                       uint64_t plen, std::vector<Message>* out, std::vector<int>* servers) {
  if (plen & 255) throw CheckError(kErrCheck, "spill segment sizes must be 256-aligned");
  const uint8_t* pay = rbuf.ptr + pay_at;
  struct Pend { size_t msg; uint16_t f, k; uint8_t mn, mx; uint32_t slot; };
  std::vector<Pend> pend;
  uint32_t nslots = 0;
  uint64_t p = 0, poff = 0;
  auto need = [&](uint64_t k) {
    if (p + k > mlen) throw CheckError(kErrCheck, "truncated spill record");
  };
  while (p + 24 <= mlen) {
    uint32_t h[6];
    memcpy(h, meta + p, 24);
    if (h[0] != kMagicHost) throw CheckError(kErrCheck, "bad spill record");
    p += 24;
    need(8ull * h[3] + 12ull * h[4] + h[2]);
    std::vector<uint64_t> fl(h[3]);
    memcpy(fl.data(), meta + p, 8ull * h[3]);
    p += 8ull * h[3];
    const size_t mi = out->size();
    for (uint32_t e = 0; e < h[4]; ++e, p += 12) {
      Pend q;
      memcpy(&q.f, meta + p, 2);
      memcpy(&q.k, meta + p + 2, 2);
      q.mn = meta[p + 4];
      q.mx = meta[p + 5];
      memcpy(&q.slot, meta + p + 8, 4);
      q.msg = mi;
      nslots = std::max(nslots, q.slot + 1);
      pend.push_back(q);
    }
    out->emplace_back();
    Message& m = out->back();
    parse_task(meta + p, h[2], &m.task);
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
  if (p != mlen) throw CheckError(kErrCheck, "trailing bytes after the spill records");
  if (!nslots) return;
  // the side-info block after the frames: one RangeBatch over it, read by the
  // decodes on this context's stream (settled from the device on demand)
  if (ctx->device() < 0) throw CheckError(kErrCheck, "device side-info sent to a host-only context");
  if (poff + 16ull * nslots > plen) throw CheckError(kErrCheck, "spill side-info overruns the payload");
  auto rb = std::make_shared<RangeBatch>();
  rb->ctx = ctx;
  rb->dev.owner = rbuf.owner;
  rb->dev.ptr = const_cast<uint8_t*>(pay + poff);
  rb->dev.bytes = 16ull * nslots;
  rb->dev.loc = Loc::kDevice;
  rb->host.assign(4ull * nslots, 0u);
  ctx->adopt_device_records(rb);
  for (const Pend& q : pend) {
    Message& m = (*out)[q.msg];
    if (q.f >= m.task.filter.size() || m.task.filter[q.f].type != FilterConfig::FIXING_FLOAT ||
        q.k >= m.task.filter[q.f].fixed_point.size())
      throw CheckError(kErrCheck, "spill side-info names no FIXING_FLOAT fixed_point");
    FixedFloatConfig& fp = m.task.filter[q.f].fixed_point[q.k];
    fp.pending = rb;
    fp.pending_idx = (int)q.slot;
    fp.pending_min = q.mn != 0;
    fp.pending_max = q.mx != 0;
  }
}

int spill_unpack(Context* ctx, const Buffer& rbuf, int world, const int64_t* sizes, std::vector<Message>* out,
                 std::vector<int>* servers, std::vector<int>* srcs) {
  out->clear();
  servers->clear();
  if (srcs) srcs->clear();
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
      if (srcs) srcs->push_back(s);
    }
  }
  return (int)out->size();
}

void device_copies(Context* ctx, const std::vector<DeviceCopy>& copies, uint8_t* dst) {
  if (copies.empty()) return;
  if (ctx->device() < 0) {
    for (const DeviceCopy& c : copies) memcpy(dst + c.dst_off, c.src, c.len);
    return;
  }
  std::vector<SpillCopy> tbl(copies.size());
  uint64_t chunk = 0;
  for (size_t k = 0; k < copies.size(); ++k) {
    tbl[k] = SpillCopy{copies[k].src, copies[k].dst_off, copies[k].len, chunk};
    chunk += (copies[k].len + kSpillChunk - 1) / kSpillChunk;
  }
  const size_t bytes = tbl.size() * sizeof(SpillCopy);
  Buffer d = ctx->alloc(bytes);
  hipStream_t st = ctx->stream();
  PSF_HIP_CHECK(hipMemcpyAsync(d.ptr, tbl.data(), bytes, hipMemcpyHostToDevice, st));
  // (pageable source: the runtime has staged it when the call returns)
  int s = spill_gather_launch(reinterpret_cast<const SpillCopy*>(d.ptr), (int)tbl.size(), chunk, dst, st);
  if (s != kOk) throw CheckError(s, "device copy gather launch failed");
}

}  // namespace psf
