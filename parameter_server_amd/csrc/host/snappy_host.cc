// Host side of COMPRESSING: buffer management around the snappy kernels
// (csrc/snappy.hip) with SArray::CompressTo / UncompressFrom semantics
// (reference src/util/shared_array_inl.h:232-255).
#include "snappy_host.h"

#include <algorithm>

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
  j.in = c_.to_device(src);
  j.dst = dst;
  j.out = c_.alloc(snappy_max_compressed(src.bytes));
  Buffer scratch = c_.alloc(snappy_compress_scratch(src.bytes));
  j.slot = (int)jobs_.size();
  j.ticket = c_.next_ticket();
  int st = snappy_compress_launch(j.in.ptr, j.in.bytes, j.out.ptr, scratch.ptr, c_.stream(), c_.prof(),
                                  c_.pub_dev(j.slot), j.ticket);
  if (st != kOk) throw CheckError(st, "snappy compress launch failed");
  jobs_.push_back(std::move(j));
}

static uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  for (; v >= 128; v >>= 7) ++n;
  return n;
}

void SnappyBatch::launch_uncompress(Job& j, const Buffer& src, uint32_t hdr, uint64_t dsize) {
  j.in = c_.to_device(src);
  j.out = dsize ? c_.alloc(dsize) : Buffer{};
  j.out.bytes = dsize;
  Buffer scratch = c_.alloc(snappy_uncompress_scratch(src.bytes, dsize));
  j.ticket = c_.next_ticket();
  int st = snappy_uncompress_launch(j.in.ptr, j.in.bytes, hdr, dsize, j.out.ptr, scratch.ptr, c_.stream(),
                                    c_.prof(), c_.pub_dev(j.slot), j.ticket);
  if (st != kOk) throw CheckError(st, "snappy uncompress launch failed");
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
  j.slot = (int)jobs_.size();
  j.hinted = hinted;
  if (hinted) j.src = src;
  launch_uncompress(j, src, hdr, dsize);
  jobs_.push_back(std::move(j));
}

void SnappyBatch::flush() {
  int bad = kOk;
  for (auto& j : jobs_) {
    c_.wait_ticket(j.slot, j.ticket);
    if (j.hinted && c_.pub_host(j.slot)->status == kErrHeaderHint) {
      // the stream's header disagrees with the size hint: decode by the
      // header, as UncompressFrom does (the slot is this job's own)
      uint64_t dsize = 0;
      const uint32_t hdr = snappy_read_header(c_, j.src, &dsize);
      if (!hdr) {
        bad = kErrCheck;
        continue;
      }
      launch_uncompress(j, j.src, hdr, dsize);
      c_.wait_ticket(j.slot, j.ticket);
    }
    const Slot& h = *c_.pub_host(j.slot);
    if (h.status != kOk) {
      bad = h.status;
      continue;
    }
    j.out.bytes = h.size;
    *j.dst = j.out;
  }
  jobs_.clear();
  if (bad != kOk) throw CheckError(kErrCheck, "CHECK(snappy::RawUncompress(src, src_size, data_))");
}

}  // namespace psf
