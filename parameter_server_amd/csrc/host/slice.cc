// Server key-range partition (the multi-GPU split) and the
// message slicer that feeds it (§8(f) f2).
//
//   even_divide     <- Range<T>::EvenDivide, src/util/range.h:100-107 (long
//                      double interval, truncating casts -- reproduced exactly)
//   slice_message   <- SliceKOFVMessage<K>, src/system/message.h:107-147
//                      (lower_bound at projected range ends, zero-copy key and
//                      value segments, `valid` when the range meets the
//                      message's key range)
#include <algorithm>
#include <vector>

#include "filter.h"
#include "slice.h"

namespace psf {

int lower_bound_launch(const void* keys, size_t n, int key_bytes, const uint64_t* d_bounds, int nb,
                       uint64_t* d_pos, hipStream_t st);

KeyRange even_divide(const KeyRange& r, uint64_t n, uint64_t i) {
  if (!(r.end >= r.begin)) throw CheckError(kErrCheck, "CHECK(valid())");
  if (n == 0) throw CheckError(kErrCheck, "CHECK_GT(n, 0)");
  if (i >= n) throw CheckError(kErrCheck, "CHECK_LT(i, n)");
  const long double itv = static_cast<long double>(r.end - r.begin) / static_cast<long double>(n);
  return KeyRange{static_cast<uint64_t>(r.begin + itv * i), static_cast<uint64_t>(r.begin + itv * (i + 1))};
}

static Buffer segment(const Buffer& b, size_t off, size_t len) {
  Buffer s = b;
  s.ptr = b.ptr ? b.ptr + off : nullptr;
  s.bytes = len;
  if (len == 0) s.clear();
  return s;
}

void slice_message(Context* ctx, const Message& msg, const std::vector<KeyRange>& krs,
                   int key_bytes, std::vector<Message>* outs, std::vector<bool>* valid) {
  if (key_bytes != 8 && key_bytes != 4) throw CheckError(kErrArg, "key type must be 32 or 64 bit");
  const size_t n = krs.size();
  outs->assign(n, Message());
  valid->assign(n, false);
  for (size_t i = 1; i < n; ++i)
    if (krs[i - 1].end != krs[i].begin) throw CheckError(kErrCheck, "CHECK_EQ(krs[i-1].end(), krs[i].begin())");
  const KeyRange mr = msg.task.has_key_range ? msg.task.key_range : KeyRange{0, 0};
  auto project = [&](uint64_t v) { return std::max(mr.begin, std::min(mr.end, v)); };
  const uint64_t kmask = key_bytes == 8 ? ~0ull : 0xFFFFFFFFull;  // (K) cast
  std::vector<uint64_t> bounds(n + 1);
  if (n) bounds[0] = project(krs[0].begin) & kmask;
  for (size_t i = 0; i < n; ++i) bounds[i + 1] = project(krs[i].end) & kmask;

  const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
  std::vector<uint64_t> pos(n + 1, 0);
  if (nkeys > 0 && n > 0) {
    if (msg.key.loc == Loc::kHost) {
      for (size_t i = 0; i <= n; ++i) {
        if (key_bytes == 8) {
          const uint64_t* k = reinterpret_cast<const uint64_t*>(msg.key.ptr);
          pos[i] = std::lower_bound(k, k + nkeys, bounds[i]) - k;
        } else {
          const uint32_t* k = reinterpret_cast<const uint32_t*>(msg.key.ptr);
          pos[i] = std::lower_bound(k, k + nkeys, (uint32_t)bounds[i]) - k;
        }
      }
    } else {
      if (n + 1 > (size_t)kMaxGrid) throw CheckError(kErrArg, "too many key ranges");
      uint64_t* d_b = static_cast<uint64_t*>(ctx->partials());
      uint64_t* d_p = d_b + (n + 1);
      hipStream_t st = ctx->stream();
      PSF_HIP_CHECK(hipMemcpyAsync(d_b, bounds.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
      int s = lower_bound_launch(msg.key.ptr, nkeys, key_bytes, d_b, (int)(n + 1), d_p, st);
      if (s != kOk) throw CheckError(s, "lower_bound launch failed");
      PSF_HIP_CHECK(hipMemcpyAsync(pos.data(), d_p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
      ctx->sync();
    }
  }

  for (size_t i = 0; i < n; ++i) {
    Message& ret = (*outs)[i];
    ret.task = msg.task;  // `new Message(msg->task)`, executor.cc:129
    const uint64_t ib = std::max(krs[i].begin, mr.begin), ie = std::min(krs[i].end, mr.end);
    if (ib >= ie) continue;  // SetIntersection(...).empty(): not sent
    (*valid)[i] = true;
    if (nkeys == 0) continue;  // "to void be divided by 0"
    const size_t lo = pos[i], hi = pos[i + 1];
    ret.set_key(segment(msg.key, lo * key_bytes, (hi - lo) * key_bytes));
    ret.task.key_type = key_bytes == 8 ? 8 : 7;  // EncodeType<K>: UINT64 / UINT32
    ret.task.has_key_type = true;
    for (const Buffer& v : msg.value) {
      const size_t k = v.bytes / nkeys;  // bytes per key
      if (nkeys * k != v.bytes) throw CheckError(kErrCheck, "CHECK_EQ(key.size() * k, v.size())");
      ret.value.push_back(segment(v, lo * k, (hi - lo) * k));
    }
  }
}

}  // namespace psf
