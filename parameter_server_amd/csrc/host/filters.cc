// Codec filters of libpsf (host side).  Each method cites the reference lines
// whose behaviour it keeps; the element work runs in the HIP kernels of
// ff_codec.hip / crc32c.hip / snappy.hip / noise.hip.
#include <math.h>

#include <algorithm>
#include <functional>
#include <map>
#include <vector>

#include "filter.h"
#include <cstring>
#include "snappy_host.h"

namespace psf {

// ------------------------------------------------------------- factory ----
Filter* Filter::create(const FilterConfig& conf, Context* ctx) {
  switch (conf.type) {  // filter.cc:9-23
    case FilterConfig::KEY_CACHING: return new KeyCachingFilter(ctx);
    case FilterConfig::COMPRESSING: return new CompressingFilter(ctx);
    case FilterConfig::FIXING_FLOAT: return new FixingFloatFilter(ctx);
    case FilterConfig::NOISE: return new AddNoiseFilter(ctx);
    default: throw CheckError(kErrArg, "unknow filter type");
  }
}

FilterConfig* Filter::find(FilterConfig::Type type, Task* task) {  // filter.cc:26-31
  for (auto& f : task->filter)
    if (f.type == type) return &f;
  return nullptr;
}

// --------------------------------------------------------- KEY_CACHING ----
uint32_t KeyCachingFilter::signature(const Buffer& key) {
  const size_t len = std::min(key.bytes, kMaxSigLen);  // key_caching.h:18
  if (key.loc == Loc::kHost) return crc32c_host(key.ptr, len);
  // <= 2 KiB: one workgroup, result published straight to host-mapped memory
  const uint32_t ticket = ctx_->next_ticket();
  int st = crc32c_launch(key.ptr, len, &ctx_->d_slots()[0].crc, ctx_->stream(), ctx_->prof(),
                         ctx_->pub_dev(0), ticket);
  if (st != kOk) throw CheckError(st, "crc32c launch failed");
  return ctx_->wait_crc(0, ticket);
}

void KeyCachingFilter::encode(Message* msg) {  // key_caching.h:9-34
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf) return;
  encode_with(msg, msg->has_key() ? signature(msg->key) : 0u);
}

bool KeyCachingFilter::needs_signature(Message* msg, bool encode) {
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf || !msg->has_key()) return false;
  return encode || conf->has_signature;
}

void KeyCachingFilter::encode_with(Message* msg, uint32_t sig) {
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf) return;
  if (!msg->has_key()) {
    conf->has_signature = false;
    conf->signature = 0;
    return;
  }
  conf->has_signature = true;
  conf->signature = sig;
  CacheKey ck{msg->task.key_channel, msg->task.key_range};
  std::lock_guard<std::mutex> l(mu_);
  Entry& e = cache_[ck];
  const bool was = !e.key.empty();
  const bool hit = e.sig == sig && e.key.bytes == msg->key.bytes;
  if (hit) {
    msg->clear_key();
  } else {
    e.sig = sig;
    e.key = msg->key;
  }
  // cache_.erase(ck): the entry is reset instead (an absent entry and a reset
  // one read the same, sig 0 with no key, and the node is not freed and
  // reallocated every round trip); account() erases reset entries in bulk
  if (conf->clear_cache_if_done && is_done(msg->task)) e = Entry{};
  account(was, e);
}

void KeyCachingFilter::account(bool was, const Entry& e) {
  const bool now = !e.key.empty();
  live_ = live_ + (now ? 1 : 0) - (was ? 1 : 0);
  const size_t idle = cache_.size() - live_;
  if (idle <= kMaxIdle || idle <= live_) return;
  for (auto it = cache_.begin(); it != cache_.end();) {
    if (it->second.key.empty()) it = cache_.erase(it);
    else ++it;
  }
}

void KeyCachingFilter::decode(Message* msg) {  // key_caching.h:36-60
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf || !conf->has_signature) return;
  decode_with(msg, msg->has_key() ? signature(msg->key) : 0u);
}

void KeyCachingFilter::decode_with(Message* msg, uint32_t got) {
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf || !conf->has_signature) return;
  const uint32_t sig = conf->signature;
  if (msg->has_key()) {
    if (got != sig) throw CheckError(kErrCheck, "KEY_CACHING: key signature mismatch");
  }
  CacheKey ck{msg->task.key_channel, msg->task.key_range};
  std::lock_guard<std::mutex> l(mu_);
  Entry& e = cache_[ck];
  const bool was = !e.key.empty();
  if (msg->has_key()) {
    e.sig = sig;
    e.key = msg->key;
  } else {
    // "the cache is invalid... may ask the sender to resend this task"
    if (sig != e.sig) {
      account(was, e);  // (a new, empty entry)
      throw CheckError(kErrCheck, "KEY_CACHING: cache miss on decode");
    }
    msg->set_key(e.key);
  }
  if (conf->clear_cache_if_done && is_done(msg->task)) e = Entry{};  // (as in encode_with)
  account(was, e);
}

// -------------------------------------------------------- FIXING_FLOAT ----
void FixingFloatFilter::convert(Message* msg, bool encode) {  // fixing_float.h:24-47
  std::vector<FfMessage> one{FfMessage{msg, defer_dequant_}};
  if (encode) encode_messages(ctx_, one);
  else decode_messages(ctx_, one);
}

namespace {
struct FfJob {
  Message* msg;
  int i;     // value index
  int type;  // FLOAT / DOUBLE
  int nb;
  FixedFloatConfig* fp;
  Buffer in, out;
  size_t elems;
  const float* range = nullptr;  // decode: the encode's device {min, max}
  bool stored = false;           // encode: codes into a stored snappy stream (COMPRESSING next)
};

// Whether msg's COMPRESSING encode comes right after its FIXING_FLOAT encode
// on the values (only KEY_CACHING, which touches keys, in between): then the
// codes are written in the stored-stream layout the compressor leaves in
// place when no fragment has a match (psf_internal.h StoredLayout).
bool compressing_follows(const Message* msg) {
  bool after = false;
  for (const auto& f : msg->task.filter) {
    if (f.type == FilterConfig::FIXING_FLOAT) {
      after = true;
    } else if (after) {
      if (f.type == FilterConfig::COMPRESSING) return true;
      if (f.type != FilterConfig::KEY_CACHING) return false;
    }
  }
  return false;
}

// the value arrays FixingFloatFilter::convert touches in one message
// (fixing_float.h:24-47); false when num_bytes == 0 (the filter does nothing)
bool collect_jobs(Message* msg, std::vector<FfJob>* jobs) {
  FilterConfig* conf = Filter::find(FilterConfig::FIXING_FLOAT, msg);
  if (!conf) throw CheckError(kErrCheck, "CHECK_NOTNULL(find(FIXING_FLOAT))");
  if (conf->num_bytes == 0) return false;
  const int n = (int)msg->value.size();
  if (n != (int)msg->task.value_type.size())
    throw CheckError(kErrCheck, "CHECK_EQ(value.size(), value_type_size())");
  const size_t first = jobs->size();
  int k = 0;
  for (int i = 0; i < n; ++i) {
    if (msg->value[i].empty()) continue;
    const int type = msg->task.value_type[i];
    if ((int)conf->fixed_point.size() <= k) conf->fixed_point.emplace_back();
    if (type == kFloat || type == kDouble)
      jobs->push_back(FfJob{msg, i, type, conf->num_bytes, &conf->fixed_point[k++], {}, {}, 0, nullptr});
  }
  if (jobs->size() > first) {
    const int nb = conf->num_bytes;
    if (nb <= 0 || nb >= 8) throw CheckError(kErrNbytes, "CHECK_GT(nbytes,0) / CHECK_LT(nbytes,8)");
  }
  return true;
}

// Outputs of jobs [b, e): one HBM block carved into 256-byte aligned
// sub-buffers that share its owner when there are several (one allocator call
// per batch instead of one per message), a plain buffer for one.
void alloc_outputs(Context* ctx, std::vector<FfJob>& jobs, size_t b, size_t e,
                   const std::vector<size_t>& bytes) {
  if (e - b == 1) {
    jobs[b].out = ctx->alloc(bytes[0]);
    return;
  }
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t total = 0;
  for (size_t q = b; q < e; ++q) total += up(bytes[q - b]);
  Buffer blk = ctx->alloc(total);
  size_t off = 0;
  for (size_t q = b; q < e; ++q) {
    Buffer& o = jobs[q].out;
    o.owner = blk.owner;
    o.ptr = blk.ptr + off;
    o.bytes = bytes[q - b];
    o.loc = Loc::kDevice;
    off += up(bytes[q - b]);
  }
}

// jobs [b, e) grouped for batched launches: same (type, nb), batchable
// (groups in a flat list: a batch almost always has one)
template <typename F, typename G>
void for_each_batch(std::vector<FfJob>& jobs, size_t b, size_t e, bool encode, F&& launch_one, G&& launch_batch) {
  struct Group {
    int type, nb;
    std::vector<size_t> q;
  };
  std::vector<Group> groups;
  for (size_t q = b; q < e; ++q) {
    FfJob& j = jobs[q];
    // a stored-layout output is written by the batched kernel only, even alone
    if ((e - b > 1 || j.stored) && ff_batchable(j.in.ptr, j.out.ptr, j.elems, j.nb, j.type, encode)) {
      Group* g = nullptr;
      for (auto& x : groups)
        if (x.type == j.type && x.nb == j.nb) g = &x;
      if (!g) {
        groups.push_back(Group{j.type, j.nb, {}});
        g = &groups.back();
        g->q.reserve(e - b);
      }
      g->q.push_back(q);
    } else {
      launch_one(q);
    }
  }
  std::sort(groups.begin(), groups.end(),  // (type, nb) order, as before
            [](const Group& x, const Group& y) { return x.type != y.type ? x.type < y.type : x.nb < y.nb; });
  for (auto& g : groups) {
    if (g.q.size() <= (size_t)kFfBatchMax) {
      if (g.q.size() == 1 && !jobs[g.q[0]].stored) launch_one(g.q[0]);
      else launch_batch(g.q);
      continue;
    }
    for (size_t k = 0; k < g.q.size(); k += kFfBatchMax) {
      std::vector<size_t> part(g.q.begin() + k, g.q.begin() + std::min(g.q.size(), k + (size_t)kFfBatchMax));
      if (part.size() == 1 && !jobs[part[0]].stored) launch_one(part[0]);
      else launch_batch(part);
    }
  }
}
}  // namespace

// FIXING_FLOAT encode (fixing_float.h:50-88) of every value array of `msgs`.
// Computed min/max (and the CHECK_GT(bin,0) outcome) are published by
// workgroup 0 of each array's encode to a host-mapped slot as soon as it has
// folded the partials; the FilterConfigs are filled from there while the
// grids are still streaming.  One array: the single-array kernels; several:
// batched launches of up to kFfBatchMax arrays (one launch per kernel for a
// whole batch of small messages).
void FixingFloatFilter::encode_messages(Context* ctx, std::vector<FfMessage>& msgs, bool lazy) {
  std::vector<FfJob> jobs;
  jobs.reserve(msgs.size());
  for (auto& m : msgs) collect_jobs(m.msg, &jobs);
  if (jobs.empty()) return;
  if (ctx->device() < 0) lazy = false;
  hipStream_t st = ctx->stream();
  // publish slots serve kSyncSlots arrays at a time; lazy encodes use none
  const size_t chunk = lazy ? std::max<size_t>(jobs.size(), 1) : (size_t)Context::kSyncSlots;
  for (size_t base = 0; base < jobs.size(); base += chunk) {
    const size_t end = std::min(jobs.size(), base + chunk);
    std::vector<uint32_t> tickets(end - base, 0);
    std::vector<FixedPoint> presets(end - base);
    std::vector<uint32_t> seeds(end - base);
    std::vector<int> lazy_idx(end - base, -1);
    std::vector<size_t> out_bytes(end - base);
    int nlazy = 0;
    for (size_t q = base; q < end; ++q) {
      FfJob& j = jobs[q];
      j.fp->settle();  // a config still pending from an earlier encode
      const size_t vsz = j.type == kFloat ? 4 : 8;
      j.in = ctx->to_device(j.msg->value[j.i]);
      j.elems = j.in.bytes / vsz;
      if (j.elems == 0) throw CheckError(kErrArg, "value array shorter than one element");
      FixedPoint& preset = presets[q - base];
      preset = FixedPoint{j.fp->has_min, j.fp->has_max, j.fp->min_value, j.fp->max_value};
      if (preset.has_min && preset.has_max) {
        if (!((double)preset.max_value - (double)preset.min_value > 0))
          throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      } else if (lazy) {
        lazy_idx[q - base] = nlazy++;
      } else {
        tickets[q - base] = ctx->next_ticket();
      }
      out_bytes[q - base] = j.elems * (size_t)j.nb;
      j.stored = ctx->device() >= 0 && (j.nb == 1 || j.nb == 2) && out_bytes[q - base] < (1ull << 32) &&
                 j.in.loc == Loc::kDevice && (reinterpret_cast<uintptr_t>(j.in.ptr) % (j.type == kFloat ? 4 : 8)) == 0 &&
                 compressing_follows(j.msg);
      // the whole stored stream (64 bytes to spare for the compressor's
      // aligned reads past a fragment's end)
      if (j.stored) out_bytes[q - base] = stored_alloc_bytes(stored_layout((uint32_t)out_bytes[q - base]));
      seeds[q - base] = (uint32_t)ff_clock_seed();  // `int seed = time(NULL)`, per array
    }
    alloc_outputs(ctx, jobs, base, end, out_bytes);
    for (size_t q = base; q < end; ++q) {
      FfJob& j = jobs[q];
      if (!j.stored) continue;
      j.out.bytes = j.elems * (size_t)j.nb;  // the payload; COMPRESSING reads it in the stream layout
      j.out.layout = j.nb == 1 ? kLayoutStored1 : kLayoutStored2;
    }
    std::shared_ptr<RangeBatch> rb;
    float* ring_dev = nullptr;
    if (nlazy) {
      rb = std::make_shared<RangeBatch>();
      rb->ctx = ctx;
      rb->dev = ctx->alloc(16 * (size_t)nlazy);
      rb->host.assign(4 * (size_t)nlazy, 0u);
      ring_dev = ctx->claim_lazy(rb, nlazy);
    }
    auto range_of = [&](size_t q) -> float* {
      const int k = lazy_idx[q - base];
      return k < 0 ? nullptr : reinterpret_cast<float*>(rb->dev.ptr + 16 * (size_t)k);
    };
    auto ring_of = [&](size_t q) -> float* {
      const int k = lazy_idx[q - base];
      return k < 0 ? nullptr : ring_dev + 4 * k;
    };
    auto one = [&](size_t q) {
      FfJob& j = jobs[q];
      if (j.stored) {  // (not batchable after all: plain codes, in the larger buffer)
        j.stored = false;
        j.out.layout = kLayoutPlain;
      }
      const uint32_t t = tickets[q - base];
      float* r = range_of(q);
      int s = ff_encode_launch(j.in.ptr, j.elems, j.type, j.nb, presets[q - base], seeds[q - base], j.out.ptr,
                               ctx->partials(), r, r ? reinterpret_cast<int*>(r + 2) : nullptr, st, ctx->prof(),
                               t ? ctx->pub_dev((int)(q - base)) : nullptr, t, ring_of(q));
      if (s != kOk) throw CheckError(s, "ff_encode launch failed");
    };
    auto batch = [&](std::vector<size_t>& part) {
      std::vector<FfArray> arrs;
      arrs.reserve(part.size());
      for (size_t q : part) {
        const FfJob& j = jobs[q];
        const uint32_t t = tickets[q - base];
        arrs.push_back(FfArray{j.in.ptr, j.out.ptr, j.elems, presets[q - base], seeds[q - base],
                               t ? (int)(q - base) : -1, t, range_of(q), ring_of(q), j.stored});
      }
      Buffer scratch = ctx->alloc(ff_batch_partials_bytes(arrs.data(), (int)arrs.size()));
      PSF_HPROF(9);
      // a held-back decode of the same value type goes along with this
      // batch's min/max pass (independent arrays)
      Context::DeferredDecode& d = ctx->deferred;
      const bool take = !d.arrs.empty() && d.value_type == jobs[part[0]].type;
      int s = ff_encode_batch_launch(jobs[part[0]].type, jobs[part[0]].nb, arrs.data(), (int)arrs.size(),
                                     scratch.ptr, ctx->pub_dev(0), st, ctx->prof(), take ? d.arrs.data() : nullptr,
                                     take ? (int)d.arrs.size() : 0, take ? d.nb : 0, ctx->fused());
      if (take) d.clear();
      if (s != kOk) throw CheckError(s, "ff_encode batch launch failed");
    };
    for_each_batch(jobs, base, end, true, one, batch);
    if (rb) ctx->track(rb);
    for (size_t q = base; q < end; ++q) {
      FfJob& j = jobs[q];
      if (tickets[q - base]) {
        ctx->wait_ticket((int)(q - base), tickets[q - base]);
        const Slot& hs = *ctx->pub_host((int)(q - base));
        if (!j.fp->has_min) j.fp->set_min(hs.range[0]);
        if (!j.fp->has_max) j.fp->set_max(hs.range[1]);
        if (hs.status == kErrHip) ctx->handoff_failed();
        if (hs.status != kOk) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      } else if (lazy_idx[q - base] >= 0) {
        j.fp->pending = rb;
        j.fp->pending_idx = lazy_idx[q - base];
        j.fp->pending_min = !j.fp->has_min;
        j.fp->pending_max = !j.fp->has_max;
      }
      j.msg->value[j.i] = j.out;
    }
  }
}

// Host side of a lazily encoded range (see FixedFloatConfig::pending).
void FixedFloatConfig::settle() {
  if (!pending) return;
  std::shared_ptr<RangeBatch> rb = std::move(pending);
  pending.reset();
  rb->resolve();
  const uint32_t* r = &rb->host[4 * (size_t)pending_idx];
  float mn, mx;
  memcpy(&mn, r, 4);
  memcpy(&mx, r + 1, 4);
  if (pending_min) set_min(mn);
  if (pending_max) set_max(mx);
  pending_idx = -1;
  pending_min = pending_max = false;
  if ((int32_t)r[2] == kErrHip) {
    if (rb->ctx) rb->ctx->handoff_failed();
    throw CheckError(kErrHip, "FIXING_FLOAT: in-launch min/max hand-off timed out");
  }
  if ((int32_t)r[2] != kOk) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
}

const float* FixedFloatConfig::device_range() const {
  return pending ? reinterpret_cast<const float*>(pending->dev.ptr + 16 * (size_t)pending_idx) : nullptr;
}

// FIXING_FLOAT decode (fixing_float.h:89-101) of every value array of `msgs`;
// a message whose node defers the dequantise keeps its codes pending
// (only where every filter listed before FIXING_FLOAT is KEY_CACHING, so
// nothing decoded after it reads values).
void FixingFloatFilter::decode_messages(Context* ctx, std::vector<FfMessage>& msgs) {
  std::vector<FfJob> jobs;
  jobs.reserve(msgs.size());
  for (auto& m : msgs) {
    const size_t first = jobs.size();
    if (!collect_jobs(m.msg, &jobs)) continue;
    bool defer = m.defer;
    for (const auto& f : m.msg->task.filter) {
      if (f.type == FilterConfig::FIXING_FLOAT) break;
      if (f.type != FilterConfig::KEY_CACHING) defer = false;
    }
    size_t keep = first;
    std::vector<uint8_t> pre;
    pre.swap(m.msg->predecoded);  // decoded by the COMPRESSING decode before (fused_ff_plan)
    for (size_t q = first; q < jobs.size(); ++q) {
      FfJob& j = jobs[q];
      FixedFloatConfig& fp = *j.fp;
      if ((size_t)j.i < pre.size() && pre[j.i]) continue;
      if (fp.pending && fp.pending->ctx == ctx && !fp.pending->done && !(defer && j.type == kFloat)) {
        // encoded on this context's stream: the kernel reads {min, max} where
        // the encode left them (CHECK_GT(bin, 0) is reported when settled)
        j.range = fp.device_range();
        if (keep != q) jobs[keep] = std::move(j);
        ++keep;
        continue;
      }
      fp.settle();
      if (!fp.has_min) throw CheckError(kErrCheck, "CHECK(conf->has_min_value())");
      if (!fp.has_max) throw CheckError(kErrCheck, "CHECK(conf->has_max_value())");
      const double bin = (double)fp.max_value - (double)fp.min_value;
      if (!(bin > 0)) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      if (defer && j.type == kFloat) {
        Message* msg = j.msg;
        if (msg->pending.size() < msg->value.size()) msg->pending.resize(msg->value.size());
        msg->pending[j.i] = PendingDequant{j.nb, fp.min_value, fp.max_value};
        continue;
      }
      if (keep != q) jobs[keep] = std::move(j);
      ++keep;
    }
    jobs.resize(keep);
  }
  if (jobs.empty()) return;
  hipStream_t st = ctx->stream();
  std::vector<size_t> out_bytes(jobs.size());
  for (size_t q = 0; q < jobs.size(); ++q) {
    FfJob& j = jobs[q];
    j.in = ctx->to_device(j.msg->value[j.i]);
    j.elems = j.in.bytes / (size_t)j.nb;
    out_bytes[q] = j.elems * (j.type == kFloat ? 4 : 8);
  }
  // outputs: the message's destination for the array when it names one of
  // the right size (Message::value_dest), else library memory
  std::vector<size_t> need;
  std::vector<size_t> need_bytes;
  for (size_t q = 0; q < jobs.size(); ++q) {
    FfJob& j = jobs[q];
    const Buffer* d = (size_t)j.i < j.msg->value_dest.size() ? &j.msg->value_dest[j.i] : nullptr;
    if (d && d->ptr && d->loc == Loc::kDevice && d->bytes == out_bytes[q]) {
      j.out = *d;
    } else {
      need.push_back(q);
      need_bytes.push_back(out_bytes[q]);
    }
  }
  if (need.size() == jobs.size()) {
    alloc_outputs(ctx, jobs, 0, jobs.size(), out_bytes);
  } else if (!need.empty()) {
    std::vector<FfJob> tmp;
    tmp.reserve(need.size());
    for (size_t q : need) tmp.push_back(jobs[q]);
    alloc_outputs(ctx, tmp, 0, tmp.size(), need_bytes);
    for (size_t t = 0; t < need.size(); ++t) jobs[need[t]].out = tmp[t].out;
  }
  auto one = [&](size_t q) {
    FfJob& j = jobs[q];
    int s = ff_decode_launch(j.in.ptr, j.elems, j.type, j.nb, j.range, j.fp->min_value, j.fp->max_value,
                             j.out.ptr, st, ctx->prof());
    if (s != kOk) throw CheckError(s, "ff_decode launch failed");
  };
  auto batch = [&](std::vector<size_t>& part) {
    std::vector<FfDecArray> arrs;
    arrs.reserve(part.size());
    for (size_t q : part) {
      const FfJob& j = jobs[q];
      arrs.push_back(FfDecArray{j.in.ptr, j.out.ptr, j.elems, j.fp->min_value, j.fp->max_value, j.range});
    }
    PSF_HPROF(10);
    const int type = jobs[part[0]].type, nb = jobs[part[0]].nb;
    Context::DeferredDecode& d = ctx->deferred;
    if (ctx->defers_here() && (d.arrs.empty() || (d.value_type == type && d.nb == nb)) &&
        d.arrs.size() + arrs.size() <= 64) {
      // held back: the next batched encode's min/max launch takes it along
      d.value_type = type;
      d.nb = nb;
      d.arrs.insert(d.arrs.end(), arrs.begin(), arrs.end());
      for (size_t q : part) {
        d.keep.push_back(jobs[q].in);
        d.keep.push_back(jobs[q].out);
        // the device {min, max} j.range points into this batch's records
        if (jobs[q].range && jobs[q].fp->pending) d.ranges.push_back(jobs[q].fp->pending);
      }
      return;
    }
    ctx->flush_deferred();
    int s = ff_decode_batch_launch(type, nb, arrs.data(), (int)arrs.size(), st, ctx->prof());
    if (s != kOk) throw CheckError(s, "ff_decode batch launch failed");
  };
  for_each_batch(jobs, 0, jobs.size(), false, one, batch);
  for (auto& j : jobs) j.msg->value[j.i] = j.out;
}

// --------------------------------------------------------- COMPRESSING ----
void CompressingFilter::encode(Message* msg) { encode_messages(ctx_, {msg}); }

void CompressingFilter::decode(Message* msg) { decode_messages(ctx_, {msg}); }

void CompressingFilter::encode_messages(Context* ctx, const std::vector<Message*>& msgs,
                                        std::unique_ptr<SnappyBatch>* defer) {  // compressing.h:8-19
  // (left in flight: its own publish slots, so the caller's decodes and the
  // next steps' synchronous launches may run meanwhile)
  std::unique_ptr<SnappyBatch> held(new SnappyBatch(*ctx, defer ? Context::kCompressSlot0 : 0));
  SnappyBatch& batch = *held;
  for (Message* msg : msgs) {
    FilterConfig* conf = find(FilterConfig::COMPRESSING, msg);
    if (!conf) continue;
    conf->uncompressed_size.clear();
    if (msg->has_key()) {
      conf->uncompressed_size.push_back(msg->key.bytes);
      batch.compress(msg->key, &msg->key);
    }
    for (auto& v : msg->value) {
      conf->uncompressed_size.push_back(v.bytes);
      batch.compress(v, &v);
    }
  }
  if (defer) {
    batch.launch_all();
    *defer = std::move(held);
    return;
  }
  batch.flush();
}

// The FIXING_FLOAT decode that follows message msg's COMPRESSING decode on
// `node`, as SnappyDequant parameters per value array (values == null: that
// array is decoded unfused).  Only where the decodes in between are
// KEY_CACHING (keys only) and FixingFloatFilter::decode_messages would take
// the array with nothing left to check: num_bytes 1 or 2, a float/double
// array whose codes fill whole values, its range known (set on the config, or
// left on the device by an encode on this context), and no deferred
// dequantise.  The fixed_point entry of an array is found as collect_jobs
// finds it, from the arrays' sizes after the uncompress (the recorded sizes).
static void fused_ff_plan(Context* ctx, RemoteNode* node, Message* msg, const FilterConfig* cz,
                          std::vector<SnappyDequant>* plan) {
  plan->assign(msg->value.size(), SnappyDequant{});
  const auto& fl = msg->task.filter;
  size_t c = fl.size();
  for (size_t q = 0; q < fl.size(); ++q)
    if (&fl[q] == cz) c = q;
  if (c == fl.size()) return;
  while (c > 0 && fl[c - 1].type == FilterConfig::KEY_CACHING) --c;
  if (c == 0 || fl[c - 1].type != FilterConfig::FIXING_FLOAT) return;
  FilterConfig* ff = Filter::find(FilterConfig::FIXING_FLOAT, msg);
  if (ff != &fl[c - 1]) return;
  const int nb = ff->num_bytes;
  if (nb != 1 && nb != 2) return;
  if (msg->value.size() != msg->task.value_type.size()) return;
  const size_t has_key = msg->has_key() ? 1 : 0;
  size_t k = 0;
  for (size_t i = 0; i < msg->value.size(); ++i) {
    const uint64_t dsize = msg->value[i].empty() ? 0 : cz->uncompressed_size[i + has_key];
    if (dsize == 0) continue;  // empty after the uncompress: collect_jobs skips it
    const int type = msg->task.value_type[i];
    if (type != kFloat && type != kDouble) continue;
    const size_t kk = k++;
    if (kk >= ff->fixed_point.size()) break;
    if (dsize % (uint64_t)nb || msg->value[i].loc != Loc::kDevice) continue;
    if (node->defer_dequant() && type == kFloat) continue;
    const FixedFloatConfig& fp = ff->fixed_point[kk];
    SnappyDequant d;
    d.nb = nb;
    d.value_type = type;
    if (fp.pending) {
      if (fp.pending->ctx != ctx || fp.pending->done) continue;  // decode_messages would settle it
      d.range = fp.device_range();
    } else {
      if (!fp.has_min || !fp.has_max || !((double)fp.max_value - (double)fp.min_value > 0)) continue;
      d.mn = fp.min_value;
      d.mx = fp.max_value;
    }
    d.values = reinterpret_cast<void*>(1);  // taken; the buffer is SnappyBatch's
    (*plan)[i] = d;
  }
}

void CompressingFilter::decode_messages(Context* ctx, const std::vector<Message*>& msgs,
                                        const std::vector<RemoteNode*>* nodes) {  // compressing.h:20-37
  DecodeInFlight st;
  decode_launch(ctx, msgs, nodes, &st, 0);
  decode_finish(&st);
}

void CompressingFilter::decode_launch(Context* ctx, const std::vector<Message*>& msgs,
                                      const std::vector<RemoteNode*>* nodes, DecodeInFlight* st, int slot0) {
  st->batch.reset(new SnappyBatch(*ctx, slot0));
  SnappyBatch& batch = *st->batch;
  std::vector<SnappyDequant> plan;
  std::vector<std::unique_ptr<bool[]>>& fused = st->fused;  // one flag per value array of each message in owners
  std::vector<Message*>& owners = st->owners;
  for (size_t m = 0; m < msgs.size(); ++m) {
    Message* msg = msgs[m];
    FilterConfig* conf = find(FilterConfig::COMPRESSING, msg);
    if (!conf) continue;
    const int has_key = msg->has_key() ? 1 : 0;
    if (conf->uncompressed_size.size() != msg->value.size() + has_key)
      throw CheckError(kErrCheck, "CHECK_EQ(conf->uncompressed_size_size(), msg->value.size() + has_key)");
    plan.clear();
    if (nodes && ctx->device() >= 0) fused_ff_plan(ctx, (*nodes)[m], msg, conf, &plan);
    bool* flags = nullptr;
    for (const SnappyDequant& d : plan)
      if (d.values && !flags) {
        fused.emplace_back(new bool[msg->value.size()]());
        owners.push_back(msg);
        flags = fused.back().get();
      }
    // the recorded sizes size the launches (the device checks them against
    // each stream's header; snappy_host.cc)
    size_t k = 0;
    if (has_key) batch.uncompress(msg->key, &msg->key, &conf->uncompressed_size[k++]);
    for (size_t i = 0; i < msg->value.size(); ++i, ++k) {
      Buffer& v = msg->value[i];
      if (flags && plan[i].values) batch.uncompress_dequant(v, &v, conf->uncompressed_size[k], plan[i], &flags[i], (int)m);
      else batch.uncompress(v, &v, &conf->uncompressed_size[k]);
    }
  }
  batch.launch_all();
}

void CompressingFilter::decode_finish(DecodeInFlight* st) {
  if (!st->batch) return;
  std::unique_ptr<SnappyBatch> batch = std::move(st->batch);
  batch->finish();
  const std::vector<Message*>& owners = st->owners;
  const std::vector<std::unique_ptr<bool[]>>& fused = st->fused;
  for (size_t f = 0; f < owners.size(); ++f) {  // the flags finish() set
    Message* msg = owners[f];
    msg->predecoded.assign(msg->value.size(), 0);
    bool any = false;
    for (size_t i = 0; i < msg->value.size(); ++i) {
      msg->predecoded[i] = fused[f][i] ? 1 : 0;
      any = any || fused[f][i];
    }
    if (!any) msg->predecoded.clear();
  }
}

// --------------------------------------------------------------- NOISE ----
void AddNoiseFilter::encode(Message* msg) {  // add_noise.h:11-25
  FilterConfig* conf = find(FilterConfig::NOISE, msg);
  if (!conf) throw CheckError(kErrCheck, "CHECK_NOTNULL(find(NOISE))");
  const int n = (int)msg->value.size();
  if (n != (int)msg->task.value_type.size())
    throw CheckError(kErrCheck, "CHECK_EQ(value.size(), value_type_size())");
  hipStream_t st = ctx_->stream();
  for (int i = 0; i < n; ++i) {
    Buffer& v = msg->value[i];
    if (v.empty()) continue;
    const int type = msg->task.value_type[i];
    if (type != kFloat && type != kDouble) continue;
    const size_t elems = v.bytes / (type == kFloat ? 4 : 8);
    if (elems == 0) continue;
    const void* z = ctx_->noise_table(type, elems);
    // in place on the caller's buffer, as the reference (add_noise.h:33-37)
    Buffer d = ctx_->to_device(v);
    int s = noise_apply_launch(d.ptr, z, elems, type, conf->mean, conf->std, st, ctx_->prof());
    if (s != kOk) throw CheckError(s, "noise launch failed");
    if (v.loc == Loc::kHost) {
      PSF_HIP_CHECK(hipMemcpyAsync(v.ptr, d.ptr, elems * (type == kFloat ? 4 : 8),
                                   hipMemcpyDeviceToHost, st));
      ctx_->sync();
    }
  }
}

// ---------------------------------------------------------- RemoteNode ----
Filter* RemoteNode::FindFilterOrCreate(const FilterConfig& conf) {  // remote_node.cc:7-15
  auto it = filters_.find(conf.type);
  if (it == filters_.end()) {
    it = filters_.emplace(conf.type, Filter::create(conf, ctx_)).first;
    it->second->set_defer_dequant(defer_dequant_);
  }
  return it->second;
}

void RemoteNode::EncodeMessage(Message* msg) {  // remote_node.cc:17-22
  for (size_t i = 0; i < msg->task.filter.size(); ++i)
    FindFilterOrCreate(msg->task.filter[i])->encode(msg);
}

void RemoteNode::DecodeMessage(Message* msg) {  // remote_node.cc:23-29, reverse order
  msg->predecoded.clear();
  for (int i = (int)msg->task.filter.size() - 1; i >= 0; --i)
    FindFilterOrCreate(msg->task.filter[i])->decode(msg);
}

// KEY_CACHING signatures (CRC32C of the first min(bytes, 2048) key bytes,
// key_caching.h:18) of many messages: device keys in batched launches whose
// results land in publish slots, host keys on the host.  finish() waits and
// fills sigs[k] for idx[k].  With `defer`, the batches use the context's
// deferred slot range, so the caller can launch further work (FIXING_FLOAT of
// the next chain position) before waiting; otherwise each batch is waited
// for before the next reuses the slots.
namespace {
struct SigBatch {
  struct Chunk {
    Context* ctx;
    int slot0;
    std::vector<size_t> ks;
    std::vector<uint32_t> tk;
  };
  std::vector<uint32_t> sigs;
  std::vector<Chunk> chunks;
  void finish_chunk(const Chunk& c) {
    for (size_t q = 0; q < c.ks.size(); ++q) {
      sigs[c.ks[q]] = c.ctx->wait_crc(c.slot0 + (int)q, c.tk[q]);
    }
  }
  void finish() {
    for (const Chunk& c : chunks) finish_chunk(c);
    chunks.clear();
  }
};
}  // namespace

// The distinct contexts of a batch, in order of first appearance (a batch
// almost always has one: a linear scan beats a map).
static int ctx_index(std::vector<Context*>& ctxs, Context* c) {
  for (size_t i = 0; i < ctxs.size(); ++i)
    if (ctxs[i] == c) return (int)i;
  ctxs.push_back(c);
  return (int)ctxs.size() - 1;
}

static void launch_signatures(RemoteNode* const* nodes, Message* const* msgs, const std::vector<int>& idx,
                              bool defer, SigBatch* sb, const KeySigHint* hints = nullptr) {
  sb->sigs.assign(idx.size(), 0u);
  sb->chunks.clear();
  std::vector<Context*> ctxs;
  std::vector<std::vector<size_t>> dev;
  for (size_t k = 0; k < idx.size(); ++k) {
    const Buffer& key = msgs[idx[k]]->key;
    const size_t len = std::min(key.bytes, (size_t)2048);
    if (hints && hints[idx[k]].matches(key)) {
      sb->sigs[k] = hints[idx[k]].crc;
    } else if (key.loc == Loc::kHost || nodes[idx[k]]->ctx()->device() < 0) {
      sb->sigs[k] = crc32c_host(key.ptr, len);
    } else {
      const int c = ctx_index(ctxs, nodes[idx[k]]->ctx());
      if ((size_t)c >= dev.size()) dev.emplace_back();
      dev[c].push_back(k);
    }
  }
  constexpr size_t kDeferCap = (size_t)(Context::kPresignSlot0 - Context::kDeferSlot0);
  for (size_t ci = 0; ci < dev.size(); ++ci) {
    Context* ctx = ctxs[ci];
    const std::vector<size_t>& ks = dev[ci];
    const bool keep = defer && ks.size() <= kDeferCap;  // all of this context's batches in flight at once
    for (size_t b = 0; b < ks.size(); b += (size_t)kCrcBatchMax) {
      const size_t e = std::min(ks.size(), b + (size_t)kCrcBatchMax);
      SigBatch::Chunk c{ctx, keep ? Context::kDeferSlot0 + (int)b : 0, {}, {}};
      std::vector<const void*> d;
      std::vector<uint32_t> n;
      std::vector<int> slot;
      for (size_t q = b; q < e; ++q) {
        const Buffer& key = msgs[idx[ks[q]]]->key;
        d.push_back(key.ptr);
        n.push_back((uint32_t)std::min(key.bytes, (size_t)2048));
        slot.push_back((int)(q - b));
        c.ks.push_back(ks[q]);
        c.tk.push_back(ctx->next_ticket());
      }
      PSF_HPROF(11);
      int s = crc32c_batch_launch(d.data(), n.data(), slot.data(), c.tk.data(), (int)d.size(),
                                  ctx->pub_dev(c.slot0), ctx->stream(), ctx->prof());
      if (s != kOk) throw CheckError(s, "crc32c batch launch failed");
      if (keep) sb->chunks.push_back(std::move(c));
      else sb->finish_chunk(c);
    }
  }
}

PresignJob presign_launch(RemoteNode* const* nodes, const Message* const* msgs, int n, bool ahead,
                          bool after_main) {
  PresignJob J;
  J.bufs.reserve(n);
  J.next.assign(n, -1);
  // key buffer -> J.bufs index: open addressing over (ptr, bytes, context)
  size_t cap = 16;
  while (cap < 2 * (size_t)n) cap <<= 1;
  std::vector<int> tab(cap, -1);
  for (int i = 0; i < n; ++i) {
    const Message& m = *msgs[i];
    if (!m.has_key() || m.key.loc != Loc::kDevice || !Filter::find(FilterConfig::KEY_CACHING, const_cast<Message*>(&m)))
      continue;
    Context* ctx = nodes[i]->ctx();
    if (ctx->device() < 0) continue;
    const uint64_t h0 = (uint64_t)reinterpret_cast<uintptr_t>(m.key.ptr) * 0x9E3779B97F4A7C15ull ^ m.key.bytes;
    for (size_t h = (size_t)(h0 >> 17) & (cap - 1);; h = (h + 1) & (cap - 1)) {
      const int q = tab[h];
      if (q < 0) {
        tab[h] = (int)J.bufs.size();
        J.bufs.push_back(PresignJob::Buf{ctx, m.key.ptr, m.key.bytes, i, i, {0, 0}, -1});
        break;
      }
      PresignJob::Buf& b = J.bufs[q];
      if (b.ptr == m.key.ptr && b.bytes == m.key.bytes && b.ctx == ctx) {
        J.next[b.last] = i;
        b.last = i;
        break;
      }
    }
  }
  // ahead (the next iteration's, waited for later): the presign slot range,
  // when all of it fits; else the synchronous slots, waited for chunk by chunk
  std::vector<Context*> ctxs;
  std::vector<size_t> per;
  for (const auto& b : J.bufs) {
    const int c = ctx_index(ctxs, b.ctx);
    if ((size_t)c >= per.size()) per.push_back(0);
    ++per[c];
  }
  size_t most = 0;
  for (size_t k : per) most = std::max(most, k);
  J.ahead = ahead && 2 * most <= (size_t)(Context::kPresignEnd - Context::kPresignSlot0);
  if (!J.ahead) return J;  // launched and waited for in presign_finish
  std::vector<const void*> d;
  std::vector<uint32_t> len, tk;
  std::vector<int> slot;
  d.reserve(2 * J.bufs.size());
  len.reserve(2 * J.bufs.size());
  tk.reserve(2 * J.bufs.size());
  slot.reserve(2 * J.bufs.size());
  for (Context* ctx : ctxs) {
    d.clear();
    len.clear();
    tk.clear();
    slot.clear();
    // after_main: after what the main stream has queued so far (a decode or
    // copy there may be producing these keys) -- the driver's first presign;
    // its later ones read the same template keys, which nothing it queues
    // writes, and stay free of the iterations in between
    hipStream_t side = after_main ? ctx->side_stream_after_main() : ctx->side_stream();
    int s = Context::kPresignSlot0;
    for (PresignJob::Buf& b : J.bufs) {
      if (b.ctx != ctx) continue;
      b.slot0 = s;
      for (int r = 0; r < 2; ++r) {
        b.tk[r] = ctx->next_ticket();
        d.push_back(b.ptr);
        len.push_back((uint32_t)std::min(b.bytes, (size_t)2048));
        tk.push_back(b.tk[r]);
        slot.push_back(s - Context::kPresignSlot0 + r);
      }
      s += 2;
    }
    for (size_t c = 0; c < d.size(); c += (size_t)kCrcBatchMax) {
      const int cnt = (int)std::min(d.size() - c, (size_t)kCrcBatchMax);
      // on the context's side stream: the CRCs are read back through the
      // publish slots, so they run beside the current iteration instead of
      // queueing behind its encodes (ordered only after the main stream's
      // position at this launch)
      int st = crc32c_batch_launch(d.data() + c, len.data() + c, slot.data() + c, tk.data() + c, cnt,
                                   ctx->pub_dev(Context::kPresignSlot0), side, ctx->prof());
      if (st != kOk) throw CheckError(st, "crc32c batch launch failed");
    }
  }
  return J;
}

void presign_finish(PresignJob& J, KeySigHint* enc, KeySigHint* dec) {
  auto fill = [&](const PresignJob::Buf& b, uint32_t se, uint32_t sd) {
    for (int i = b.first; i >= 0; i = J.next[i]) {
      enc[i] = KeySigHint{b.ptr, b.bytes, se};
      if (dec) dec[i] = KeySigHint{b.ptr, b.bytes, sd};
    }
  };
  if (J.ahead) {
    for (const auto& b : J.bufs) fill(b, b.ctx->wait_crc(b.slot0, b.tk[0]), b.ctx->wait_crc(b.slot0 + 1, b.tk[1]));
    J.bufs.clear();
    return;
  }
  // now: chunks of the synchronous slots, each launched and waited for
  constexpr size_t kPer = (size_t)Context::kSyncSlots / 2;  // buffers (x2 CRCs) in flight per wait
  std::map<Context*, std::vector<size_t>> order;
  for (size_t q = 0; q < J.bufs.size(); ++q) order[J.bufs[q].ctx].push_back(q);
  for (auto& kv : order) {
    Context* ctx = kv.first;
    const std::vector<size_t>& qs = kv.second;
    for (size_t b0 = 0; b0 < qs.size(); b0 += kPer) {
      const size_t e = std::min(qs.size(), b0 + kPer);
      // CRC 2q: the sender's signature of buffer q; CRC 2q + 1: the receiver's check
      std::vector<const void*> d;
      std::vector<uint32_t> len, tk;
      std::vector<int> slot;
      for (size_t i = b0; i < e; ++i) {
        PresignJob::Buf& b = J.bufs[qs[i]];
        for (int r = 0; r < 2; ++r) {
          b.tk[r] = ctx->next_ticket();
          d.push_back(b.ptr);
          len.push_back((uint32_t)std::min(b.bytes, (size_t)2048));
          tk.push_back(b.tk[r]);
          slot.push_back((int)(2 * (i - b0) + r));
        }
      }
      for (size_t c = 0; c < d.size(); c += (size_t)kCrcBatchMax) {
        const int cnt = (int)std::min(d.size() - c, (size_t)kCrcBatchMax);
        int st = crc32c_batch_launch(d.data() + c, len.data() + c, slot.data() + c, tk.data() + c, cnt,
                                     ctx->pub_dev(0), ctx->stream(), ctx->prof());
        if (st != kOk) throw CheckError(st, "crc32c batch launch failed");
      }
      for (size_t i = b0; i < e; ++i) {
        const PresignJob::Buf& b = J.bufs[qs[i]];
        fill(b, ctx->wait_crc((int)(2 * (i - b0)), b.tk[0]), ctx->wait_crc((int)(2 * (i - b0) + 1), b.tk[1]));
      }
    }
  }
  J.bufs.clear();
}

void presign_roundtrip(RemoteNode* const* nodes, const Message* const* msgs, int n, KeySigHint* enc,
                       KeySigHint* dec) {
  PresignJob J = presign_launch(nodes, msgs, n, false, true);
  presign_finish(J, enc, dec);
}

// Encode in filter order, position by position over all chains.  The
// KEY_CACHING signatures of a position stay in flight while a following
// all-FIXING_FLOAT position launches (the two touch disjoint parts of a
// message: keys vs values); the cache logic then runs in message order, so
// the result equals sequential EncodeMessage calls.
void encode_batch(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints,
                  PendingEncode* later) {
  size_t maxlen = 0;
  for (int i = 0; i < n; ++i) maxlen = std::max(maxlen, msgs[i]->task.filter.size());
  struct PendingKc {
    bool active = false;
    size_t pos = 0;
    std::vector<int> kc, kc_sig;
    SigBatch sb;
  } pend;
  auto finish_kc = [&] {
    if (!pend.active) return;
    PSF_HPROF(4);
    pend.active = false;
    pend.sb.finish();
    size_t k = 0;
    for (int i : pend.kc) {
      const uint32_t sig = (k < pend.kc_sig.size() && pend.kc_sig[k] == i) ? pend.sb.sigs[k++] : 0u;
      static_cast<KeyCachingFilter*>(nodes[i]->FindFilterOrCreate(msgs[i]->task.filter[pend.pos]))
          ->encode_with(msgs[i], sig);
    }
  };
  for (size_t pos = 0; pos < maxlen; ++pos) {  // filter position pos of every chain
    bool only_ff = true;
    for (int i = 0; i < n && only_ff; ++i)
      if (pos < msgs[i]->task.filter.size() && msgs[i]->task.filter[pos].type != FilterConfig::FIXING_FLOAT)
        only_ff = false;
    if (!only_ff) finish_kc();
    // per context (in order of first appearance; a batch almost always has one)
    std::vector<Context*> ffc, czc;
    std::vector<std::vector<FfMessage>> ff;
    std::vector<std::vector<Message*>> cz;
    std::vector<int> kc, kc_sig;
    for (int i = 0; i < n; ++i) {
      if (pos >= msgs[i]->task.filter.size()) continue;
      const FilterConfig& conf = msgs[i]->task.filter[pos];
      Filter* f = nodes[i]->FindFilterOrCreate(conf);
      if (conf.type == FilterConfig::FIXING_FLOAT) {
        const int c = ctx_index(ffc, nodes[i]->ctx());
        if ((size_t)c >= ff.size()) ff.emplace_back().reserve(n);
        ff[c].push_back(FfMessage{msgs[i], false});
      } else if (conf.type == FilterConfig::KEY_CACHING) {
        kc.push_back(i);
        if (KeyCachingFilter::needs_signature(msgs[i], true)) kc_sig.push_back(i);
      } else if (conf.type == FilterConfig::COMPRESSING) {
        const int c = ctx_index(czc, nodes[i]->ctx());
        if ((size_t)c >= cz.size()) cz.emplace_back();
        cz[c].push_back(msgs[i]);
      } else {
        f->encode(msgs[i]);
      }
    }
    for (size_t c = 0; c < cz.size(); ++c) {
      if (later && pos + 1 == maxlen) {  // the last position: left in flight for the caller
        later->snappy.emplace_back();
        CompressingFilter::encode_messages(czc[c], cz[c], &later->snappy.back());
      } else {
        CompressingFilter::encode_messages(czc[c], cz[c]);
      }
    }
    if (!kc.empty()) {  // signatures launched now, the caches after the next position's launches
      pend.pos = pos;
      pend.kc = std::move(kc);
      pend.kc_sig = std::move(kc_sig);
      {
        PSF_HPROF(2);
        launch_signatures(nodes, msgs, pend.kc_sig, true, &pend.sb, hints);
      }
      pend.active = true;
    }
    {
      PSF_HPROF(3);
      for (size_t c = 0; c < ff.size(); ++c) FixingFloatFilter::encode_messages(ffc[c], ff[c], /*lazy=*/true);
    }
  }
  finish_kc();
}

// positions [r0, maxlen) of decode_batch (r-th filter from the end of every chain)
static void decode_positions(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints,
                             size_t r0);

void decode_batch(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints,
                  PendingDecode* later) {
  for (int i = 0; i < n; ++i) msgs[i]->predecoded.clear();
  if (later && n > 0) {
    if (later->active) later->finish();
    // every chain ends in COMPRESSING of value arrays only: its launches now,
    // the rest in finish().  (A message with keys -- a KEY_CACHING miss,
    // keys compressed -- is decoded at once: tag-dense key streams need the
    // uncompress's tail kernels, which finish() would queue behind whatever
    // the caller launches meanwhile; measured slower, r05u2.)
    bool all_cz = true;
    for (int i = 0; i < n && all_cz; ++i)
      all_cz = !msgs[i]->task.filter.empty() && msgs[i]->task.filter.back().type == FilterConfig::COMPRESSING &&
               !msgs[i]->has_key();
    if (all_cz) {
      std::vector<Context*> czc;
      std::vector<std::vector<Message*>> cz;
      std::vector<std::vector<RemoteNode*>> cz_nodes;
      for (int i = 0; i < n; ++i) {
        nodes[i]->FindFilterOrCreate(msgs[i]->task.filter.back());
        const int c = ctx_index(czc, nodes[i]->ctx());
        if ((size_t)c >= cz.size()) {
          cz.emplace_back();
          cz_nodes.emplace_back();
        }
        cz[c].push_back(msgs[i]);
        cz_nodes[c].push_back(nodes[i]);
      }
      later->nodes.assign(nodes, nodes + n);
      later->msgs.assign(msgs, msgs + n);
      later->hints.clear();
      if (hints) later->hints.assign(hints, hints + n);
      later->cz.clear();
      later->cz.resize(cz.size());
      later->active = true;
      for (size_t c = 0; c < cz.size(); ++c)
        CompressingFilter::decode_launch(czc[c], cz[c], &cz_nodes[c], &later->cz[c], Context::kDecodeSlot0);
      return;
    }
  }
  decode_positions(nodes, msgs, n, hints, 0);
}

void PendingDecode::finish() {
  if (!active) return;
  active = false;
  for (auto& c : cz) CompressingFilter::decode_finish(&c);
  cz.clear();
  decode_positions(nodes.data(), msgs.data(), (int)msgs.size(), hints.empty() ? nullptr : hints.data(), 1);
}

PendingDecode::~PendingDecode() {
  try {
    finish();
  } catch (...) {  // (a destructor does not throw; the caller that cared finished it)
  }
}

static void decode_positions(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints,
                             size_t r0) {
  size_t maxlen = 0;
  for (int i = 0; i < n; ++i) maxlen = std::max(maxlen, msgs[i]->task.filter.size());
  for (size_t r = r0; r < maxlen; ++r) {  // r-th filter from the end of every chain
    std::vector<Context*> ffc, czc;
    std::vector<std::vector<FfMessage>> ff;
    std::vector<std::vector<Message*>> cz;
    std::vector<std::vector<RemoteNode*>> cz_nodes;
    std::vector<int> kc, kc_sig;
    for (int i = 0; i < n; ++i) {
      const size_t len = msgs[i]->task.filter.size();
      if (r >= len) continue;
      const FilterConfig& conf = msgs[i]->task.filter[len - 1 - r];
      Filter* f = nodes[i]->FindFilterOrCreate(conf);
      if (conf.type == FilterConfig::FIXING_FLOAT) {
        const int c = ctx_index(ffc, nodes[i]->ctx());
        if ((size_t)c >= ff.size()) ff.emplace_back().reserve(n);
        ff[c].push_back(FfMessage{msgs[i], f->defer_dequant()});
      } else if (conf.type == FilterConfig::KEY_CACHING) {
        kc.push_back(i);
        if (KeyCachingFilter::needs_signature(msgs[i], false)) kc_sig.push_back(i);
      } else if (conf.type == FilterConfig::COMPRESSING) {
        const int c = ctx_index(czc, nodes[i]->ctx());
        if ((size_t)c >= cz.size()) {
          cz.emplace_back();
          cz_nodes.emplace_back();
        }
        cz[c].push_back(msgs[i]);
        cz_nodes[c].push_back(nodes[i]);
      } else {
        f->decode(msgs[i]);
      }
    }
    for (size_t c = 0; c < cz.size(); ++c) CompressingFilter::decode_messages(czc[c], cz[c], &cz_nodes[c]);
    if (!kc.empty()) {
      PSF_HPROF(8);
      SigBatch sb;
      launch_signatures(nodes, msgs, kc_sig, false, &sb, hints);
      size_t k = 0;
      for (int i : kc) {
        const size_t len = msgs[i]->task.filter.size();
        const uint32_t sig = (k < kc_sig.size() && kc_sig[k] == i) ? sb.sigs[k++] : 0u;
        static_cast<KeyCachingFilter*>(nodes[i]->FindFilterOrCreate(msgs[i]->task.filter[len - 1 - r]))
            ->decode_with(msgs[i], sig);
      }
    }
    {
      PSF_HPROF(7);
      for (size_t c = 0; c < ff.size(); ++c) FixingFloatFilter::decode_messages(ffc[c], ff[c]);
    }
  }
}

void RemoteNode::set_defer_dequant(bool v) {
  defer_dequant_ = v;
  for (auto& f : filters_) f.second->set_defer_dequant(v);
}

void materialize(Context* ctx, Message* msg) {
  for (size_t i = 0; i < msg->pending.size(); ++i) {
    const PendingDequant pd = msg->pending[i];
    if (pd.nb == 0) continue;
    const int type = msg->task.value_type[i];
    const size_t vsz = type == kFloat ? 4 : 8;
    Buffer code = ctx->to_device(msg->value[i]);
    const size_t elems = code.bytes / (size_t)pd.nb;
    Buffer out = ctx->alloc(elems * vsz);
    int s = ff_decode_launch(code.ptr, elems, type, pd.nb, nullptr, pd.min_value, pd.max_value, out.ptr,
                             ctx->stream(), ctx->prof());
    if (s != kOk) throw CheckError(s, "ff_decode launch failed");
    msg->value[i] = out;
    msg->pending[i] = PendingDequant{};
  }
}

}  // namespace psf
