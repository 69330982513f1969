// Server-side consumers of received messages, fed
// straight from the decode: a FIXING_FLOAT value array the decode left pending
// (RemoteNode::set_defer_dequant) is dequantised inside the consumer kernel.
//
//   KvMapFtrl       KVMap<Key, float, FTRLEntry, SGDState>
//                   (src/parameter/kv_map.h:32-91, async_sgd.h:42-154) on HBM
//   ordered_match   ParallelOrderedMatch (src/util/parallel_ordered_match.h:57-83)
//                   on one value array of a message (KVVector::SetValue,
//                   src/parameter/kv_vector.h:171-211)
#pragma once
#include "context.h"
#include "message.h"

namespace psf {

// LearningRateConfig (linear.proto:93-101) + PenaltyConfig (linear.proto:83-90)
// as the server's SGDState builds them (async_sgd.h:91-94, penalty.h:76-91).
struct FtrlConfig {
  int lr_type = 2;  // 1 CONSTANT, 2 DECAY
  double alpha = 0.01, beta = 10;
  double lambda1 = 0, lambda2 = 0;  // ElasticNet(l1, l2)
};

class KvMapFtrl {
 public:
  struct Stats {
    int64_t nnz;
    double weight_sum, delta_sum;
    uint64_t size;
  };
  KvMapFtrl(Context* ctx, size_t capacity, const FtrlConfig& conf);
  // Lifetime (as Context's): the C ABI's handle holds one reference, a router
  // serving pulls from the map one more; the last unref deletes the map and
  // drops its context reference.
  std::atomic<int> refs{1};
  static void ref(KvMapFtrl* m) {
    if (m) m->refs.fetch_add(1, std::memory_order_relaxed);
  }
  static void unref(KvMapFtrl* m) {
    if (!m || m->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    Context* c = m->ctx_;
    delete m;
    Context::unref(c);
  }
  Context* context() const { return ctx_; }

  // KVMap::SetValue (kv_map.h:80-91) of a push message: keys + one value array
  void set_value(const Message& msg);
  // KVMap::GetValue (kv_map.h:69-77): appends the float array of w
  void get_value(Message* msg);
  // get_value of n messages in one launch (their outputs share one block)
  void get_values(Message* const* msgs, int n);
  // raw device arrays (grad: float, or FIXING_FLOAT codes when pd.nb != 0)
  void push(const uint64_t* keys, size_t n, const void* src, const PendingDequant& pd);
  void pull(const uint64_t* keys, size_t n, float* out);
  Stats stats();
  size_t capacity() const { return cap_; }

 private:
  void reserve(size_t incoming);
  Context* ctx_;
  Buffer table_, stats_;
  size_t cap_ = 0;
  size_t size_ub_ = 0;  // upper bound on occupied slots (exact after a stats read)
  float alpha_, beta_, l1_, l2_;
  int decay_;
};

// ParallelOrderedMatch of value array `vi` of msg (keys = msg.key) into
// (dst_key, dst_val); returns *n as the reference does (matched keys * k).
size_t ordered_match(Context* ctx, const Message& msg, int vi, const uint64_t* dst_key, size_t ndst,
                     void* dst_val, int value_type, int k, int op);
size_t ordered_match_raw(Context* ctx, const uint64_t* src_key, size_t nsrc, const void* src_val,
                         const PendingDequant& pd, const uint64_t* dst_key, size_t ndst, void* dst_val,
                         int value_type, int k, int op);

}  // namespace psf
