// Host side of COMPRESSING: buffer management around the snappy kernels
// (csrc/snappy.hip) with SArray::CompressTo / UncompressFrom semantics
// (reference src/util/shared_array_inl.h:232-255).
#include "snappy_host.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <string>

namespace psf {

// snappy::GetUncompressedLength -> Varint::Parse32WithLimit: at most 5 bytes,
// the 5th < 16.  Returns the header length, 0 when malformed.
uint32_t snappy_parse_header(const uint8_t* p, size_t n, uint64_t* len) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < 5; ++i) {
    if (i >= n) return 0;
    const uint32_t b = p[i];
    if (i == 4 && b >= 16) return 0;
    v |= (b & 127u) << (7 * i);
    if (b < 128) {
      *len = v;
      return i + 1;
    }
  }
  return 0;
}

uint32_t snappy_read_header(Context& c, const Buffer& in, uint64_t* len) {
  uint8_t h[5] = {0, 0, 0, 0, 0};
  const size_t k = std::min<size_t>(5, in.bytes);
  if (in.loc == Loc::kHost) {
    std::copy(in.ptr, in.ptr + k, h);
  } else {
    PSF_HIP_CHECK(hipMemcpyAsync(h, in.ptr, k, hipMemcpyDeviceToHost, c.stream()));
    PSF_HIP_CHECK(hipStreamSynchronize(c.stream()));
  }
  return snappy_parse_header(h, k, len);
}

void SnappyBatch::compress(const Buffer& src, Buffer* dst) {
  if (src.empty()) {  // "otherwise, snappy will add a 0 here": empty stays empty
    dst->clear();
    return;
  }
  if (src.bytes > 0xffffffffull) throw CheckError(kErrArg, "snappy: input longer than 4 GiB");
  if (jobs_.size() == (size_t)Context::kSyncSlots) flush();
  Job j;
  j.compress = true;
  j.in = c_.to_device(src);
  j.dst = dst;
  j.out = c_.alloc(snappy_max_compressed(src.bytes));
  j.slot = slot0_ + (int)jobs_.size();
  j.ticket = c_.next_ticket();
  jobs_.push_back(std::move(j));
}

static uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  for (; v >= 128; v >>= 7) ++n;
  return n;
}

void SnappyBatch::prepare_uncompress(Job& j, const Buffer& src, uint32_t hdr, uint64_t dsize) {
  j.in = c_.to_device(src);
  j.out = dsize ? c_.alloc(dsize) : Buffer{};
  j.out.bytes = dsize;
  j.hdr = hdr;
  j.ticket = c_.next_ticket();
}

void SnappyBatch::uncompress(const Buffer& src, Buffer* dst, const uint64_t* size_hint) {
  if (src.empty()) {  // UncompressFrom: src_size == 0 -> clear()
    dst->clear();
    return;
  }
  uint64_t dsize = 0;
  uint32_t hdr = 0;
  const bool hinted = size_hint && src.loc == Loc::kDevice && *size_hint <= 0xffffffffull &&
                      varint_len(*size_hint) <= src.bytes;
  if (hinted) {
    dsize = *size_hint;
    hdr = varint_len(dsize);
  } else {
    hdr = snappy_read_header(c_, src, &dsize);
    if (!hdr) throw CheckError(kErrCheck, "CHECK(snappy::GetUncompressedLength(src, src_size, &dsize))");
  }
  if (jobs_.size() == (size_t)Context::kSyncSlots) flush();
  Job j;
  j.dst = dst;
  j.slot = slot0_ + (int)jobs_.size();
  j.hinted = hinted;
  if (hinted) j.src = src;
  prepare_uncompress(j, src, hdr, dsize);
  jobs_.push_back(std::move(j));
}

void SnappyBatch::uncompress_dequant(const Buffer& src, Buffer* dst, uint64_t size_hint, const SnappyDequant& dq,
                                     bool* fused, int group) {
  const size_t before = jobs_.size();
  uncompress(src, dst, &size_hint);
  if (jobs_.size() != before + 1 || jobs_.back().dst != dst) return;  // empty source: nothing launched
  Job& j = jobs_.back();
  if (!j.hinted) return;  // the header was read: decoded unfused
  const size_t vsz = dq.value_type == kDouble ? 8 : 4;
  j.values = c_.alloc(j.out.bytes / (size_t)dq.nb * vsz);
  j.dq = dq;
  j.dq.values = j.values.ptr;
  if (!snappy_dequant_ok(j.dq, j.out.bytes)) {
    j.dq = SnappyDequant{};
    j.values = Buffer{};
    return;
  }
  j.fused = fused;
  j.group = group;
}

// every pending stream in as few launch chains as possible: compress and
// uncompress jobs each in groups of up to kSnappyBatchMax
void SnappyBatch::launch(size_t b, size_t e) {
  for (int pass = 0; pass < 2; ++pass) {
    const bool comp = pass == 0;
    std::vector<SnappyCJob> cj;
    std::vector<SnappyDJob> dj;
    std::vector<size_t> di;  // dj's jobs_ indices
    auto go = [&] {
      int st = kOk;
      if (comp && !cj.empty()) {
        Buffer scratch = c_.alloc(snappy_compress_batch_scratch(cj.data(), (int)cj.size()));
        st = snappy_compress_batch_launch(cj.data(), (int)cj.size(), scratch.ptr, c_.stream(), c_.prof(),
                                          c_.pub_dev(0));
        cj.clear();
      } else if (!comp && !dj.empty()) {
        Tail t;
        t.scratch = c_.alloc(snappy_uncompress_batch_scratch(dj.data(), (int)dj.size()));
        // the context's pre-zeroed control region serves the first batch
        // only: a later batch's fast path would clear it for the next launch
        // while this batch's tail may still need it
        const ZeroPair z = tails_.empty() ? c_.zero_pair(Context::kZeroUncompress, dj.size() * 32 + 4) : ZeroPair{};
        st = snappy_uncompress_batch_launch(dj.data(), (int)dj.size(), t.scratch.ptr, c_.stream(), c_.prof(),
                                            c_.pub_dev(0), z, &t.t);
        if (st != kOk) c_.zero_pair_unused(Context::kZeroUncompress, z);
        if (st == kOk) {
          t.done = c_.take_marker();
          PSF_HIP_CHECK(hipEventRecord(t.done, c_.stream()));
          t.jobs = di;
          tails_.push_back(std::move(t));
        }
        dj.clear();
        di.clear();
      }
      if (st != kOk) throw CheckError(st, comp ? "snappy compress launch failed" : "snappy uncompress launch failed");
    };
    for (size_t i = b; i < e; ++i) {
      Job& j = jobs_[i];
      if (j.compress != comp) continue;
      if (comp) cj.push_back(SnappyCJob{j.in.ptr, j.in.bytes, j.out.ptr, j.slot, j.ticket, (uint32_t)j.in.layout});
      else {
        dj.push_back(SnappyDJob{j.in.ptr, j.in.bytes, j.hdr, j.out.bytes, j.out.ptr, j.slot, j.ticket, j.dq});
        di.push_back(i);
      }
      if (cj.size() == (size_t)kSnappyBatchMax || dj.size() == (size_t)kSnappyBatchMax) go();
    }
    go();
  }
}

void SnappyBatch::launch_all() {
  launch(launched_, jobs_.size());
  launched_ = jobs_.size();
}

// psf_debug_force_snappy_tail (tests): the uncompress's tail kernels always
// run after the fast path -- what a completion marker that lands before the
// fast path's verdicts gives (the tail then finds the streams decoded)
static std::atomic<int> g_force_tail{0};
bool snappy_force_tail() { return g_force_tail.load(std::memory_order_relaxed) != 0; }

void SnappyBatch::finish() {
  launch_all();
  const bool force = snappy_force_tail();
  // uncompress batches: once the fast path has completed, the tail kernels
  // run only if a stream has not published its verdict (on FIXING_FLOAT
  // codes and other stored streams the fast path decodes everything)
  for (Tail& t : tails_) {
    // every verdict published (the fast path's last workgroups publish while
    // the rest of its grid drains), or the fast path complete without them
    auto published = [&] {
      for (size_t i : t.jobs) {
        const Job& j = jobs_[i];
        if (__atomic_load_n(&c_.pub_host(j.slot)->ticket, __ATOMIC_ACQUIRE) != j.ticket) return false;
      }
      return true;
    };
    bool all = !force && published();
    if (!all) {
      WaitTimer wt(&c_, Context::kWaitPublish);
      for (uint64_t spin = 0;; ++spin) {
        if (!force && (all = published())) break;
        const hipError_t q = hipEventQuery(t.done);
        if (q == hipSuccess) {
          all = !force && published();
          break;
        }
        if (q != hipErrorNotReady) throw CheckError(kErrHip, std::string("stream failed: ") + hipGetErrorString(q));
        if (spin > 4096) sched_yield();
      }
    }
    c_.give_marker(t.done);
    if (!all) {
      const int st = snappy_uncompress_tail_launch(&t.t, c_.stream());
      if (st != kOk) throw CheckError(st, "snappy uncompress launch failed");
    }
  }
  tails_.clear();  // (scratch freed stream-ordered, after the tails)
  int bad = kOk;
  // a fused stream whose header disagrees with its hint: every fused stream of
  // its group (one message's arrays) is decoded again unfused, so the
  // FIXING_FLOAT decode that follows sees the arrays the unfused chain gives
  std::vector<int> redo_groups;
  for (auto& j : jobs_) {
    c_.wait_ticket(j.slot, j.ticket);
    if (j.dq.values && c_.pub_host(j.slot)->status == kErrHeaderHint) redo_groups.push_back(j.group);
  }
  for (auto& j : jobs_) {
    const bool regroup = j.dq.values && std::find(redo_groups.begin(), redo_groups.end(), j.group) != redo_groups.end();
    if (regroup) {  // the codes, by the header (the slot is this job's own)
      j.dq = SnappyDequant{};
      j.values = Buffer{};
      uint64_t dsize = 0;
      const uint32_t hdr = snappy_read_header(c_, j.src, &dsize);
      if (!hdr) {
        bad = kErrCheck;
        continue;
      }
      prepare_uncompress(j, j.src, hdr, dsize);
      const SnappyDJob d{j.in.ptr, j.in.bytes, j.hdr, j.out.bytes, j.out.ptr, 0, j.ticket};
      Buffer scratch = c_.alloc(snappy_uncompress_batch_scratch(&d, 1));
      const int st = snappy_uncompress_batch_launch(&d, 1, scratch.ptr, c_.stream(), c_.prof(), c_.pub_dev(j.slot));
      if (st != kOk) throw CheckError(st, "snappy uncompress launch failed");
      c_.wait_ticket(j.slot, j.ticket);
    } else if (j.hinted && c_.pub_host(j.slot)->status == kErrHeaderHint) {
      // the stream's header disagrees with the size hint: decode by the
      // header, as UncompressFrom does (the slot is this job's own)
      uint64_t dsize = 0;
      const uint32_t hdr = snappy_read_header(c_, j.src, &dsize);
      if (!hdr) {
        bad = kErrCheck;
        continue;
      }
      prepare_uncompress(j, j.src, hdr, dsize);
      const SnappyDJob d{j.in.ptr, j.in.bytes, j.hdr, j.out.bytes, j.out.ptr, 0, j.ticket};
      Buffer scratch = c_.alloc(snappy_uncompress_batch_scratch(&d, 1));
      const int st = snappy_uncompress_batch_launch(&d, 1, scratch.ptr, c_.stream(), c_.prof(), c_.pub_dev(j.slot));
      if (st != kOk) throw CheckError(st, "snappy uncompress launch failed");
      c_.wait_ticket(j.slot, j.ticket);
    }
    const Slot& h = *c_.pub_host(j.slot);
    if (h.status != kOk) {
      bad = h.status;
      continue;
    }
    j.out.bytes = h.size;
    if (j.compress && h.pad == kStoredInPlace) {
      // every fragment came out stored: the stream FIXING_FLOAT wrote is the
      // result (snappy.hip K-place), the compressor's buffer goes unused
      Buffer o = j.in;
      o.bytes = h.size;
      o.layout = kLayoutPlain;
      *j.dst = o;
    } else if (j.dq.values) {
      *j.dst = j.values;
      *j.fused = true;
    } else {
      *j.dst = j.out;
    }
  }
  jobs_.clear();
  launched_ = 0;
  if (bad != kOk) throw CheckError(kErrCheck, "CHECK(snappy::RawUncompress(src, src_size, data_))");
}

}  // namespace psf

extern "C" int psf_debug_force_snappy_tail(int on) {
  psf::g_force_tail.store(on ? 1 : 0, std::memory_order_relaxed);
  return 0;
}
