// Server-side consumers: host side of kv_store.hip.
#include "kvstore.h"

#include <string.h>

namespace psf {

namespace {
size_t next_pow2(size_t v) {
  size_t c = 1;
  while (c < v) c <<= 1;
  return c;
}

// value-array element count under a (possibly pending) dequantise
size_t elements(const Buffer& b, const PendingDequant& pd, size_t vsz) {
  return pd.nb ? b.bytes / (size_t)pd.nb : b.bytes / vsz;
}
}  // namespace

KvMapFtrl::KvMapFtrl(Context* ctx, size_t capacity, const FtrlConfig& c) : ctx_(ctx) {
  if (ctx->device() < 0) throw CheckError(kErrArg, "KVMap needs a device context");
  // LearningRate<float> (learning_rate.h:9-12) and ElasticNet<float>
  // (penalty.h:43-46) take their parameters as V = float and CHECK them
  alpha_ = (float)c.alpha;
  beta_ = (float)c.beta;
  l1_ = (float)c.lambda1;
  l2_ = (float)c.lambda2;
  decay_ = c.lr_type == 1 ? 0 : 1;  // LearningRateConfig::CONSTANT = 1
  if (!(alpha_ > 0)) throw CheckError(kErrCheck, "CHECK_GT(alpha(), 0)");
  if (!(beta_ >= 0)) throw CheckError(kErrCheck, "CHECK_GE(beta(), 0)");
  if (!(l1_ >= 0) || !(l2_ >= 0)) throw CheckError(kErrCheck, "CHECK_GE(lambda, 0)");
  cap_ = next_pow2(2 * (capacity < 2048 ? 2048 : capacity));
  table_ = ctx_->alloc(cap_ * kvmap_slot_bytes());
  int s = kvmap_init_launch(table_.ptr, cap_, ctx_->stream());
  if (s != kOk) throw CheckError(s, "kvmap init failed");
  stats_ = ctx_->alloc(kvmap_stats_bytes());
  PSF_HIP_CHECK(hipMemsetAsync(stats_.ptr, 0, kvmap_stats_bytes(), ctx_->stream()));
}

KvMapFtrl::Stats KvMapFtrl::stats() {
  struct {
    long long nnz_delta;
    double weight_sum, delta_sum;
    unsigned long long inserted;
    int status, pad;
  } h;
  static_assert(sizeof(h) == 40, "KvStats mirror");
  if (kvmap_stats_bytes() != sizeof(h)) throw CheckError(kErrArg, "KvStats layout");
  PSF_HIP_CHECK(hipMemcpyAsync(&h, stats_.ptr, sizeof(h), hipMemcpyDeviceToHost, ctx_->stream()));
  ctx_->sync();
  if (h.status == kErrCheck) throw CheckError(kErrCheck, "CHECK_GT(eta, 0) (penalty.h:52)");
  if (h.status != kOk) throw CheckError(h.status, "KVMap table overflow");
  size_ub_ = h.inserted;
  return Stats{h.nnz_delta, h.weight_sum, h.delta_sum, h.inserted};
}

// Keep the load factor <= 1/2: grow (2x, rehash on the device) before a push
// could exceed it.  The host tracks an upper bound and reads the exact count
// (one sync) only when the bound says the table might be too full.
void KvMapFtrl::reserve(size_t incoming) {
  if ((size_ub_ + incoming) * 2 <= cap_) {
    size_ub_ += incoming;
    return;
  }
  const size_t size = stats().size;
  const size_t need = size + incoming;
  if (need * 2 > cap_) {
    size_t ncap = cap_;
    while (need * 2 > ncap) ncap <<= 1;
    Buffer nt = ctx_->alloc(ncap * kvmap_slot_bytes());
    int s = kvmap_init_launch(nt.ptr, ncap, ctx_->stream());
    if (s == kOk) s = kvmap_rehash_launch(table_.ptr, cap_, nt.ptr, ncap, ctx_->stream());
    if (s != kOk) throw CheckError(s, "kvmap rehash failed");
    table_ = nt;
    cap_ = ncap;
  }
  size_ub_ = need;
}

void KvMapFtrl::push(const uint64_t* keys, size_t n, const void* src, const PendingDequant& pd) {
  if (n == 0) return;
  reserve(n);
  int s = kvmap_push_launch(table_.ptr, cap_, keys, n, static_cast<const float*>(src), pd.nb ? src : nullptr,
                            pd.nb, pd.min_value, pd.max_value, alpha_, beta_, decay_, l1_, l2_, stats_.ptr,
                            ctx_->stream(), ctx_->prof());
  if (s != kOk) throw CheckError(s, "kvmap push launch failed");
}

void KvMapFtrl::pull(const uint64_t* keys, size_t n, float* out) {
  int s = kvmap_get_launch(table_.ptr, cap_, keys, n, out, ctx_->stream(), ctx_->prof());
  if (s != kOk) throw CheckError(s, "kvmap get launch failed");
}

void KvMapFtrl::set_value(const Message& msg) {  // kv_map.h:80-91
  const size_t n = msg.key.bytes / 8;
  if (msg.value.size() != 1) throw CheckError(kErrCheck, "CHECK_EQ(msg->value.size(), 1)");
  const PendingDequant pd = msg.is_pending(0) ? msg.pending[0] : PendingDequant{};
  if (elements(msg.value[0], pd, 4) != n) throw CheckError(kErrCheck, "CHECK_EQ(n * k_, val.size())");
  if (n == 0) return;
  Buffer k = ctx_->to_device(msg.key);
  Buffer v = ctx_->to_device(msg.value[0]);
  push(reinterpret_cast<const uint64_t*>(k.ptr), n, v.ptr, pd);
}

void KvMapFtrl::get_value(Message* msg) {  // kv_map.h:69-77
  const size_t n = msg->key.bytes / 8;
  Buffer out = ctx_->alloc(n * 4);
  if (n) {
    Buffer k = ctx_->to_device(msg->key);
    pull(reinterpret_cast<const uint64_t*>(k.ptr), n, reinterpret_cast<float*>(out.ptr));
  }
  msg->value.push_back(out);  // msg->add_value(val): value_type FLOAT
  msg->task.value_type.push_back(kFloat);
  if (!msg->pending.empty()) msg->pending.resize(msg->value.size());
}

void KvMapFtrl::get_values(Message* const* msgs, int n) {
  if (n == 1) return get_value(msgs[0]);
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t bytes = 0;
  for (int i = 0; i < n; ++i) bytes += up(msgs[i]->key.bytes / 8 * 4);
  Buffer blk = bytes ? ctx_->alloc(bytes) : Buffer();
  std::vector<KvGetJob> jobs;
  std::vector<Buffer> keep;
  uint64_t total = 0, off = 0;
  for (int i = 0; i < n; ++i) {
    Message* msg = msgs[i];
    const size_t k = msg->key.bytes / 8;
    Buffer out;
    if (k) {
      out = blk;
      out.ptr = blk.ptr + off;
      out.bytes = k * 4;
      Buffer kb = ctx_->to_device(msg->key);
      jobs.push_back(KvGetJob{reinterpret_cast<const uint64_t*>(kb.ptr), reinterpret_cast<float*>(out.ptr), total, k});
      keep.push_back(kb);
      total += k;
      off += up(k * 4);
    }
    msg->value.push_back(out);  // msg->add_value(val): value_type FLOAT
    msg->task.value_type.push_back(kFloat);
    if (!msg->pending.empty()) msg->pending.resize(msg->value.size());
  }
  if (jobs.empty()) return;
  Buffer d = ctx_->alloc(jobs.size() * sizeof(KvGetJob));
  PSF_HIP_CHECK(hipMemcpyAsync(d.ptr, jobs.data(), jobs.size() * sizeof(KvGetJob), hipMemcpyHostToDevice,
                               ctx_->stream()));
  int s = kvmap_get_batch_launch(table_.ptr, cap_, reinterpret_cast<const KvGetJob*>(d.ptr), (int)jobs.size(), total,
                                 ctx_->stream(), ctx_->prof());
  if (s != kOk) throw CheckError(s, "kvmap get launch failed");
  // (keep / d: released stream-ordered after the launch)
}

size_t ordered_match_raw(Context* ctx, const uint64_t* src_key, size_t nsrc, const void* src_val,
                         const PendingDequant& pd, const uint64_t* dst_key, size_t ndst, void* dst_val,
                         int value_type, int k, int op) {
  if (ctx->device() < 0) throw CheckError(kErrArg, "ordered match needs a device context");
  if (nsrc == 0 || ndst == 0) return 0;  // parallel_ordered_match.h:14
  Buffer cnt = ctx->alloc(sizeof(unsigned long long));
  PSF_HIP_CHECK(hipMemsetAsync(cnt.ptr, 0, sizeof(unsigned long long), ctx->stream()));
  Buffer scratch;
  if (k > 1) scratch = ctx->alloc(nsrc * sizeof(int64_t));
  int s = ordered_match_launch(src_key, nsrc, pd.nb ? nullptr : src_val, pd.nb ? src_val : nullptr, pd.nb,
                               pd.min_value, pd.max_value, dst_key, ndst, dst_val, k, value_type, op,
                               reinterpret_cast<int64_t*>(scratch.ptr),
                               reinterpret_cast<unsigned long long*>(cnt.ptr), ctx->stream(), ctx->prof());
  if (s != kOk) throw CheckError(s, "ordered match launch failed");
  unsigned long long matched = 0;
  PSF_HIP_CHECK(hipMemcpyAsync(&matched, cnt.ptr, sizeof(matched), hipMemcpyDeviceToHost, ctx->stream()));
  ctx->sync();
  return (size_t)matched * (size_t)k;
}

size_t ordered_match(Context* ctx, const Message& msg, int vi, const uint64_t* dst_key, size_t ndst,
                     void* dst_val, int value_type, int k, int op) {
  if (vi < 0 || vi >= (int)msg.value.size()) throw CheckError(kErrArg, "value index out of range");
  if (k <= 0) throw CheckError(kErrArg, "k must be positive");
  const size_t vsz = value_type == kFloat ? 4 : 8;
  const size_t nsrc = msg.key.bytes / 8;
  const PendingDequant pd = msg.is_pending(vi) ? msg.pending[vi] : PendingDequant{};
  if (pd.nb && value_type != kFloat) throw CheckError(kErrArg, "pending codes decode to float");
  // CHECK_EQ(src_key.size() * k, src_val.size()), parallel_ordered_match.h:68
  if (elements(msg.value[vi], pd, vsz) != nsrc * (size_t)k)
    throw CheckError(kErrCheck, "CHECK_EQ(src_key.size() * k, src_val.size())");
  Buffer kb = ctx->to_device(msg.key);
  Buffer vb = ctx->to_device(msg.value[vi]);
  return ordered_match_raw(ctx, reinterpret_cast<const uint64_t*>(kb.ptr), nsrc, vb.ptr, pd, dst_key, ndst,
                           dst_val, value_type, k, op);
}

}  // namespace psf
