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

// whether slice i of msg is sent: the range meets the message's key range
// (SetIntersection(...).empty() means not sent)
bool slice_valid(const Message& msg, const KeyRange& kr) {
  const KeyRange mr = msg.task.has_key_range ? msg.task.key_range : KeyRange{0, 0};
  const uint64_t ib = std::max(kr.begin, mr.begin), ie = std::min(kr.end, mr.end);
  return ib < ie;
}

// fill the (task-copied) slice ret of a valid range from its split positions
void fill_slice(const Message& msg, int key_bytes, size_t lo, size_t hi, Message* ret) {
  const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
  if (nkeys == 0) return;  // "to void be divided by 0"
  // SArray::Segment (shared_array_inl.h:135): a range end that does not fit
  // K wraps in the (K) cast and lands before the range's begin
  if (lo > hi) throw CheckError(kErrCheck, "CHECK(range.valid())");
  ret->set_key(segment(msg.key, lo * key_bytes, (hi - lo) * key_bytes));
  ret->task.key_type = key_bytes == 8 ? 8 : 7;  // EncodeType<K>: UINT64 / UINT32
  ret->task.has_key_type = true;
  ret->value.reserve(msg.value.size());
  for (const Buffer& v : msg.value) {
    const size_t k = v.bytes / nkeys;  // bytes per key
    if (nkeys * k != v.bytes) throw CheckError(kErrCheck, "CHECK_EQ(key.size() * k, v.size())");
    ret->value.push_back(segment(v, lo * k, (hi - lo) * k));
  }
}

// build the slices of one message from its split positions
void build_slices(const Message& msg, const std::vector<KeyRange>& krs, int key_bytes, const uint64_t* pos,
                  std::vector<Message>* outs, std::vector<bool>* valid) {
  const size_t n = krs.size();
  outs->assign(n, Message());
  valid->assign(n, false);
  for (size_t i = 0; i < n; ++i) {
    Message& ret = (*outs)[i];
    ret.task = msg.task;  // `new Message(msg->task)`, executor.cc:129
    if (!slice_valid(msg, krs[i])) continue;
    (*valid)[i] = true;
    fill_slice(msg, key_bytes, pos[i], pos[i + 1], &ret);
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

// SliceKOFVMessage for many messages at once: one launch, one event wait.
void slice_messages(Context* ctx, const std::vector<const Message*>& msgs, const std::vector<KeyRange>& krs,
                    int key_bytes, std::vector<std::vector<Message>>* outs, std::vector<std::vector<bool>>* valid) {
  std::unique_ptr<SliceJob> job = slice_begin(ctx, msgs, krs, key_bytes);
  slice_end(*job, outs, valid);
}

static SliceJob::KeyId key_id(const Message& m) {
  return SliceJob::KeyId{m.key.ptr, m.key.bytes, m.task.has_key_range, m.task.key_range};
}

bool SliceJob::same_inputs(const Message* const* ms, int n) const {
  if ((size_t)n != msgs.size()) return false;
  for (int i = 0; i < n; ++i) {
    if (ms[i] != msgs[i]) return false;
    const KeyId k = key_id(*ms[i]);
    const KeyId& o = ids[i];
    if (k.ptr != o.ptr || k.bytes != o.bytes || k.has_range != o.has_range || !(k.range == o.range)) return false;
  }
  return true;
}

SliceJob::~SliceJob() {
  if (!ev) return;
  if (!ended) (void)hipEventSynchronize(ev);  // the pinned records go back to the pool
  ctx->give_event(ev);
}

std::unique_ptr<SliceJob> slice_begin(Context* ctx, const std::vector<const Message*>& msgs,
                                      const std::vector<KeyRange>& krs, int key_bytes, hipEvent_t after) {
  if (key_bytes != 8 && key_bytes != 4) throw CheckError(kErrArg, "key type must be 32 or 64 bit");
  const size_t n = krs.size();
  for (size_t i = 1; i < n; ++i)
    if (krs[i - 1].end != krs[i].begin) throw CheckError(kErrCheck, "CHECK_EQ(krs[i-1].end(), krs[i].begin())");
  std::unique_ptr<SliceJob> job(new SliceJob());
  job->ctx = ctx;
  job->msgs = msgs;
  job->krs = krs;
  job->key_bytes = key_bytes;
  const size_t M = msgs.size(), nb = n + 1;
  job->pos.assign(M * nb, 0);
  job->ids.reserve(M);
  std::vector<std::vector<uint64_t>> bounds(M);
  for (size_t m = 0; m < M; ++m) {
    const Message& msg = *msgs[m];
    job->ids.push_back(key_id(msg));
    bounds[m] = slice_bounds(msg, krs, key_bytes);
    const size_t nkeys = msg.key.bytes / (size_t)key_bytes;
    if (nkeys == 0 || n == 0) continue;
    if (msg.key.loc == Loc::kHost) host_lower_bounds(msg, key_bytes, bounds[m], job->pos.data() + m * nb);
    else job->dev.push_back(m);
  }
  const size_t D = job->dev.size();
  if (D == 0) return job;
  // host-mapped layout: desc[2D] | bounds[D nb] | pos[D nb] (u64) | sig[D n] (u32)
  const size_t desc_b = 16 * D, bnd_b = 8 * D * nb, pos_b = 8 * D * nb, sig_b = 4 * D * n;
  job->buf = ctx->pinned(desc_b + bnd_b + pos_b + sig_b);
  uint64_t* h = reinterpret_cast<uint64_t*>(job->buf.host);
  for (size_t q = 0; q < D; ++q) {
    const Message& msg = *msgs[job->dev[q]];
    h[2 * q] = reinterpret_cast<uint64_t>(msg.key.ptr);
    h[2 * q + 1] = msg.key.bytes / (size_t)key_bytes;
    std::copy(bounds[job->dev[q]].begin(), bounds[job->dev[q]].end(), h + 2 * D + q * nb);
  }
  uint8_t* d = job->buf.dev;
  SliceSigParams p{};
  p.desc = reinterpret_cast<const uint64_t*>(d);
  p.bounds = reinterpret_cast<const uint64_t*>(d + desc_b);
  p.nslices = (int)n;
  p.nmsg = (int)D;
  p.pos = reinterpret_cast<uint64_t*>(d + desc_b + bnd_b);
  p.sig = reinterpret_cast<uint32_t*>(d + desc_b + bnd_b + pos_b);
  hipStream_t st = ctx->stream();
  if (after) {
    st = ctx->side_stream();
    PSF_HIP_CHECK(hipStreamWaitEvent(st, after, 0));
  }
  int s = slice_sig_launch(p, key_bytes, st);
  if (s != kOk) throw CheckError(s, "slice launch failed");
  job->ev = ctx->take_event();
  PSF_HIP_CHECK(hipEventRecord(job->ev, st));
  return job;
}

// the device pass's results into job.pos; returns the signatures (or null)
static const uint32_t* slice_collect(SliceJob& job) {
  if (job.ended) throw CheckError(kErrArg, "slice job already ended");
  const size_t n = job.krs.size(), nb = n + 1, D = job.dev.size();
  const uint32_t* sig = nullptr;
  if (D) {
    job.ctx->wait_event(job.ev, Context::kWaitSlice);
    const uint8_t* h = job.buf.host;
    const uint64_t* pos = reinterpret_cast<const uint64_t*>(h + 16 * D + 8 * D * nb);
    sig = reinterpret_cast<const uint32_t*>(h + 16 * D + 16 * D * nb);
    for (size_t q = 0; q < D; ++q) std::copy(pos + q * nb, pos + (q + 1) * nb, job.pos.begin() + job.dev[q] * nb);
  }
  job.ended = true;
  return sig;
}

void slice_end_flat(SliceJob& job, std::vector<Message>* out, std::vector<int>* stream, std::vector<int>* server,
                    std::vector<KeySigHint>* hints, std::vector<uint64_t>* first_key) {
  const uint32_t* sig = slice_collect(job);
  const size_t M = job.msgs.size(), n = job.krs.size(), nb = n + 1;
  std::vector<int> dev_index(M, -1);
  for (size_t q = 0; q < job.dev.size(); ++q) dev_index[job.dev[q]] = (int)q;
  out->reserve(out->size() + M * n);
  for (size_t m = 0; m < M; ++m) {
    const Message& msg = *job.msgs[m];
    const uint64_t* pos = job.pos.data() + m * nb;
    for (size_t i = 0; i < n; ++i) {
      if (!slice_valid(msg, job.krs[i])) continue;
      out->emplace_back();
      Message& ret = out->back();
      ret.task = msg.task;  // `new Message(msg->task)`, executor.cc:129
      fill_slice(msg, job.key_bytes, pos[i], pos[i + 1], &ret);
      stream->push_back((int)m);
      server->push_back((int)i);
      first_key->push_back(ret.key.bytes ? pos[i] : 0);
      KeySigHint h;
      if (sig && dev_index[m] >= 0 && !ret.key.empty())
        h = KeySigHint{ret.key.ptr, ret.key.bytes, sig[(size_t)dev_index[m] * n + i]};
      hints->push_back(h);
    }
  }
}

void slice_end(SliceJob& job, std::vector<std::vector<Message>>* outs, std::vector<std::vector<bool>>* valid,
               std::vector<std::vector<KeySigHint>>* hints) {
  const uint32_t* sig = slice_collect(job);
  const size_t M = job.msgs.size(), n = job.krs.size(), nb = n + 1, D = job.dev.size();
  outs->assign(M, {});
  valid->assign(M, {});
  for (size_t m = 0; m < M; ++m)
    build_slices(*job.msgs[m], job.krs, job.key_bytes, job.pos.data() + m * nb, &(*outs)[m], &(*valid)[m]);
  if (!hints) return;
  hints->assign(M, std::vector<KeySigHint>(n));
  for (size_t q = 0; q < D; ++q) {
    const size_t m = job.dev[q];
    for (size_t i = 0; i < n; ++i) {
      const Message& sl = (*outs)[m][i];
      if (!(*valid)[m][i] || sl.key.empty()) continue;
      (*hints)[m][i] = KeySigHint{sl.key.ptr, sl.key.bytes, sig[q * n + i]};
    }
  }
}

}  // namespace psf
