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
int lower_bound_batch_launch(const uint64_t* d_desc, int key_bytes, const uint64_t* d_bounds, int nb, int nmsg,
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

namespace {
// the (n + 1) lower_bound targets of one message: krs projected onto the
// message's key range, cast to K (message.h:111-116)
std::vector<uint64_t> slice_bounds(const Message& msg, const std::vector<KeyRange>& krs, int key_bytes) {
  const size_t n = krs.size();
  const KeyRange mr = msg.task.has_key_range ? msg.task.key_range : KeyRange{0, 0};
  auto project = [&](uint64_t v) { return std::max(mr.begin, std::min(mr.end, v)); };
  const uint64_t kmask = key_bytes == 8 ? ~0ull : 0xFFFFFFFFull;  // (K) cast
  std::vector<uint64_t> bounds(n + 1);
  if (n) bounds[0] = project(krs[0].begin) & kmask;
  for (size_t i = 0; i < n; ++i) bounds[i + 1] = project(krs[i].end) & kmask;
  return bounds;
}

void host_lower_bounds(const Message& msg, int key_bytes, const std::vector<uint64_t>& bounds, uint64_t* pos) {
  const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
  for (size_t i = 0; i < bounds.size(); ++i) {
    if (key_bytes == 8) {
      const uint64_t* k = reinterpret_cast<const uint64_t*>(msg.key.ptr);
      pos[i] = std::lower_bound(k, k + nkeys, bounds[i]) - k;
    } else {
      const uint32_t* k = reinterpret_cast<const uint32_t*>(msg.key.ptr);
      pos[i] = std::lower_bound(k, k + nkeys, (uint32_t)bounds[i]) - k;
    }
  }
}

// build the slices of one message from its split positions
void build_slices(const Message& msg, const std::vector<KeyRange>& krs, int key_bytes, const uint64_t* pos,
                  std::vector<Message>* outs, std::vector<bool>* valid) {
  const size_t n = krs.size();
  outs->assign(n, Message());
  valid->assign(n, false);
  const KeyRange mr = msg.task.has_key_range ? msg.task.key_range : KeyRange{0, 0};
  const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
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
}  // namespace

void slice_message(Context* ctx, const Message& msg, const std::vector<KeyRange>& krs,
                   int key_bytes, std::vector<Message>* outs, std::vector<bool>* valid) {
  std::vector<const Message*> one{&msg};
  std::vector<std::vector<Message>> o;
  std::vector<std::vector<bool>> v;
  slice_messages(ctx, one, krs, key_bytes, &o, &v);
  *outs = std::move(o[0]);
  *valid = std::move(v[0]);
}

// SliceKOFVMessage for many messages at once: the device lower_bounds of all
// of them are queued back to back and read back with one synchronisation.
void slice_messages(Context* ctx, const std::vector<const Message*>& msgs, const std::vector<KeyRange>& krs,
                    int key_bytes, std::vector<std::vector<Message>>* outs, std::vector<std::vector<bool>>* valid) {
  if (key_bytes != 8 && key_bytes != 4) throw CheckError(kErrArg, "key type must be 32 or 64 bit");
  const size_t n = krs.size();
  for (size_t i = 1; i < n; ++i)
    if (krs[i - 1].end != krs[i].begin) throw CheckError(kErrCheck, "CHECK_EQ(krs[i-1].end(), krs[i].begin())");
  const size_t M = msgs.size();
  outs->assign(M, {});
  valid->assign(M, {});
  std::vector<uint64_t> pos(M * (n + 1), 0), bounds(M * (n + 1), 0);
  std::vector<size_t> dev;
  for (size_t m = 0; m < M; ++m) {
    const Message& msg = *msgs[m];
    const std::vector<uint64_t> b = slice_bounds(msg, krs, key_bytes);
    std::copy(b.begin(), b.end(), bounds.begin() + m * (n + 1));
    const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
    if (nkeys == 0 || n == 0) continue;
    if (msg.key.loc == Loc::kHost) host_lower_bounds(msg, key_bytes, b, pos.data() + m * (n + 1));
    else dev.push_back(m);
  }
  if (!dev.empty()) {  // one upload, one launch, one read-back for all device-keyed messages
    hipStream_t st = ctx->stream();
    const size_t D = dev.size(), nb = n + 1;
    std::vector<uint64_t> up(D * nb + 2 * D);
    for (size_t q = 0; q < D; ++q) {
      const Message& msg = *msgs[dev[q]];
      std::copy(bounds.begin() + dev[q] * nb, bounds.begin() + (dev[q] + 1) * nb, up.begin() + q * nb);
      up[D * nb + 2 * q] = reinterpret_cast<uint64_t>(msg.key.ptr);
      up[D * nb + 2 * q + 1] = msg.key.bytes / (size_t)key_bytes;
    }
    Buffer d_up = ctx->alloc(up.size() * 8), d_p = ctx->alloc(D * nb * 8);
    PSF_HIP_CHECK(hipMemcpyAsync(d_up.ptr, up.data(), up.size() * 8, hipMemcpyHostToDevice, st));
    const uint64_t* d_b = reinterpret_cast<const uint64_t*>(d_up.ptr);
    int s = lower_bound_batch_launch(d_b + D * nb, key_bytes, d_b, (int)nb, (int)D,
                                     reinterpret_cast<uint64_t*>(d_p.ptr), st);
    if (s != kOk) throw CheckError(s, "lower_bound launch failed");
    std::vector<uint64_t> dpos(D * nb);
    PSF_HIP_CHECK(hipMemcpyAsync(dpos.data(), d_p.ptr, D * nb * 8, hipMemcpyDeviceToHost, st));
    ctx->sync();
    for (size_t q = 0; q < D; ++q)
      std::copy(dpos.begin() + q * nb, dpos.begin() + (q + 1) * nb, pos.begin() + dev[q] * nb);
  }
  for (size_t m = 0; m < M; ++m)
    build_slices(*msgs[m], krs, key_bytes, pos.data() + m * (n + 1), &(*outs)[m], &(*valid)[m]);
}

}  // namespace psf
