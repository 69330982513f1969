// Codec filters of libpsf (host side).  Each method cites the reference lines
// whose behaviour it keeps; the element work runs in the HIP kernels of
// ff_codec.hip / crc32c.hip / snappy.hip / noise.hip.
#include <math.h>

#include <algorithm>
#include <vector>

#include "filter.h"
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
  ctx_->wait_ticket(0, ticket);
  return ctx_->pub_host(0)->crc;
}

void KeyCachingFilter::encode(Message* msg) {  // key_caching.h:9-34
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf) return;
  if (!msg->has_key()) {
    conf->has_signature = false;
    conf->signature = 0;
    return;
  }
  const uint32_t sig = signature(msg->key);
  conf->has_signature = true;
  conf->signature = sig;
  CacheKey ck{msg->task.key_channel, msg->task.key_range};
  std::lock_guard<std::mutex> l(mu_);
  Entry& e = cache_[ck];
  const bool hit = e.sig == sig && e.key.bytes == msg->key.bytes;
  if (hit) {
    msg->clear_key();
  } else {
    e.sig = sig;
    e.key = msg->key;
  }
  if (conf->clear_cache_if_done && is_done(msg->task)) cache_.erase(ck);
}

void KeyCachingFilter::decode(Message* msg) {  // key_caching.h:36-60
  FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
  if (!conf || !conf->has_signature) return;
  const uint32_t sig = conf->signature;
  if (msg->has_key()) {
    const uint32_t got = signature(msg->key);
    if (got != sig) throw CheckError(kErrCheck, "KEY_CACHING: key signature mismatch");
  }
  CacheKey ck{msg->task.key_channel, msg->task.key_range};
  std::lock_guard<std::mutex> l(mu_);
  Entry& e = cache_[ck];
  if (msg->has_key()) {
    e.sig = sig;
    e.key = msg->key;
  } else {
    // "the cache is invalid... may ask the sender to resend this task"
    if (sig != e.sig) throw CheckError(kErrCheck, "KEY_CACHING: cache miss on decode");
    msg->set_key(e.key);
  }
  if (conf->clear_cache_if_done && is_done(msg->task)) cache_.erase(ck);
}

// -------------------------------------------------------- FIXING_FLOAT ----
void FixingFloatFilter::convert(Message* msg, bool encode) {  // fixing_float.h:24-47
  FilterConfig* conf = find(FilterConfig::FIXING_FLOAT, msg);
  if (!conf) throw CheckError(kErrCheck, "CHECK_NOTNULL(find(FIXING_FLOAT))");
  if (conf->num_bytes == 0) return;
  const int n = (int)msg->value.size();
  if (n != (int)msg->task.value_type.size())
    throw CheckError(kErrCheck, "CHECK_EQ(value.size(), value_type_size())");

  struct Job { int i; int type; FixedFloatConfig* fp; Buffer in, out; size_t elems; };
  std::vector<Job> jobs;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    if (msg->value[i].empty()) continue;
    const int type = msg->task.value_type[i];
    if ((int)conf->fixed_point.size() <= k) conf->fixed_point.emplace_back();
    if (type == kFloat || type == kDouble) jobs.push_back(Job{i, type, &conf->fixed_point[k++], {}, {}, 0});
  }
  if (jobs.empty()) return;
  const int nb = conf->num_bytes;
  if (nb <= 0 || nb >= 8) throw CheckError(kErrNbytes, "CHECK_GT(nbytes,0) / CHECK_LT(nbytes,8)");
  const double ratio = ff_ratio(nb);
  (void)ratio;
  hipStream_t st = ctx_->stream();

  if (!encode) {  // fixing_float.h:89-101
    // Deferral is only sound when nothing decoded after this filter reads the
    // values: decode runs in reverse order, so every filter listed before
    // FIXING_FLOAT must be KEY_CACHING (keys only).
    bool defer = defer_dequant_;
    for (const auto& f : msg->task.filter) {
      if (f.type == FilterConfig::FIXING_FLOAT) break;
      if (f.type != FilterConfig::KEY_CACHING) defer = false;
    }
    for (auto& j : jobs) {
      const FixedFloatConfig& fp = *j.fp;
      if (!fp.has_min) throw CheckError(kErrCheck, "CHECK(conf->has_min_value())");
      if (!fp.has_max) throw CheckError(kErrCheck, "CHECK(conf->has_max_value())");
      const double bin = (double)fp.max_value - (double)fp.min_value;
      if (!(bin > 0)) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      if (defer && j.type == kFloat) {
        if (msg->pending.size() < msg->value.size()) msg->pending.resize(msg->value.size());
        msg->pending[j.i] = PendingDequant{nb, fp.min_value, fp.max_value};
        continue;
      }
      const size_t vsz = j.type == kFloat ? 4 : 8;
      Buffer code = ctx_->to_device(msg->value[j.i]);
      const size_t elems = code.bytes / (size_t)nb;
      Buffer out = ctx_->alloc(elems * vsz);
      int s = ff_decode_launch(code.ptr, elems, j.type, nb, nullptr, fp.min_value, fp.max_value, out.ptr, st,
                               ctx_->prof());
      if (s != kOk) throw CheckError(s, "ff_decode launch failed");
      msg->value[j.i] = out;
    }
    return;
  }

  // encode, fixing_float.h:50-88.  Computed min/max (and the CHECK_GT(bin,0)
  // outcome) are published by workgroup 0 of each encode kernel to a
  // host-mapped slot as soon as it has folded the partials; the FilterConfig is
  // filled from there while the rest of the grid is still streaming.
  for (size_t base = 0; base < jobs.size(); base += Context::kSlots) {
    const size_t end = std::min(jobs.size(), base + (size_t)Context::kSlots);
    std::vector<uint32_t> tickets(end - base, 0);
    for (size_t q = base; q < end; ++q) {
      Job& j = jobs[q];
      const size_t vsz = j.type == kFloat ? 4 : 8;
      j.in = ctx_->to_device(msg->value[j.i]);
      j.elems = j.in.bytes / vsz;
      if (j.elems == 0) throw CheckError(kErrArg, "value array shorter than one element");
      FixedPoint preset{j.fp->has_min, j.fp->has_max, j.fp->min_value, j.fp->max_value};
      PubSlot* pub = nullptr;
      if (preset.has_min && preset.has_max) {
        if (!((double)preset.max_value - (double)preset.min_value > 0))
          throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      } else {
        tickets[q - base] = ctx_->next_ticket();
        pub = ctx_->pub_dev((int)(q - base));
      }
      j.out = ctx_->alloc(j.elems * (size_t)nb);
      const uint32_t seed = (uint32_t)ff_clock_seed();  // `int seed = time(NULL)`, per array
      int s = ff_encode_launch(j.in.ptr, j.elems, j.type, nb, preset, seed, j.out.ptr,
                               ctx_->partials(), nullptr, nullptr, st, ctx_->prof(), pub,
                               tickets[q - base]);
      if (s != kOk) throw CheckError(s, "ff_encode launch failed");
    }
    for (size_t q = base; q < end; ++q) {
      Job& j = jobs[q];
      if (tickets[q - base]) {
        ctx_->wait_ticket((int)(q - base), tickets[q - base]);
        const Slot& hs = *ctx_->pub_host((int)(q - base));
        if (!j.fp->has_min) j.fp->set_min(hs.range[0]);
        if (!j.fp->has_max) j.fp->set_max(hs.range[1]);
        if (hs.status != kOk) throw CheckError(kErrBin, "CHECK_GT(bin, 0)");
      }
      msg->value[j.i] = j.out;
    }
  }
}

// --------------------------------------------------------- COMPRESSING ----
void CompressingFilter::encode(Message* msg) {  // compressing.h:8-19
  FilterConfig* conf = find(FilterConfig::COMPRESSING, msg);
  if (!conf) return;
  conf->uncompressed_size.clear();
  SnappyBatch batch(*ctx_);
  if (msg->has_key()) {
    conf->uncompressed_size.push_back(msg->key.bytes);
    batch.compress(msg->key, &msg->key);
  }
  for (auto& v : msg->value) {
    conf->uncompressed_size.push_back(v.bytes);
    batch.compress(v, &v);
  }
  batch.flush();
}

void CompressingFilter::decode(Message* msg) {  // compressing.h:20-37
  FilterConfig* conf = find(FilterConfig::COMPRESSING, msg);
  if (!conf) return;
  const int has_key = msg->has_key() ? 1 : 0;
  if (conf->uncompressed_size.size() != msg->value.size() + has_key)
    throw CheckError(kErrCheck, "CHECK_EQ(conf->uncompressed_size_size(), msg->value.size() + has_key)");
  SnappyBatch batch(*ctx_);
  if (has_key) batch.uncompress(msg->key, &msg->key);
  for (auto& v : msg->value) batch.uncompress(v, &v);
  batch.flush();
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
  for (int i = (int)msg->task.filter.size() - 1; i >= 0; --i)
    FindFilterOrCreate(msg->task.filter[i])->decode(msg);
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
