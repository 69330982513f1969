#include "router.h"

#include <stdlib.h>

#include "slice.h"

namespace psf {

PushRouter::PushRouter(Context* ctx, const std::vector<KeyRange>& ranges, int rank, int world, bool loopback)
    : ctx_(ctx), ranges_(ranges), rank_(rank), world_(world), loopback_(loopback) {
  if (world <= 0 || rank < 0 || rank >= world) throw CheckError(kErrArg, "bad rank / world");
  if ((int)ranges.size() < world) throw CheckError(kErrArg, "need at least one server per rank");
  for (size_t i = 1; i < ranges.size(); ++i)
    if (ranges[i - 1].end != ranges[i].begin) throw CheckError(kErrArg, "server ranges must be contiguous");
}

PushRouter::~PushRouter() {
  if (step_start_) ctx_->give_marker(step_start_);
}

// The key width SliceKOFVMessage<K> slices with (message.h:107-147): the
// application's K, which the stream's task.key_type records (EncodeType<K>,
// message.h:70-76).  Streams without keys do not vote; the streams of one
// step must agree, and a key buffer must hold whole keys (SArray<K>'s CHECK).
static int step_key_bytes(const Message* const* streams, int n) {
  int kb = 0;
  for (int i = 0; i < n; ++i) {
    const Message& m = *streams[i];
    if (m.key.empty()) continue;
    int w = 0;
    if (m.task.has_key_type && m.task.key_type == 8) w = 8;       // UINT64
    else if (m.task.has_key_type && m.task.key_type == 7) w = 4;  // UINT32
    else throw CheckError(kErrArg, "router: stream keys must be UINT32 or UINT64 (task.key_type)");
    if (m.key.bytes % (size_t)w) throw CheckError(kErrCheck, "CHECK_EQ(key.size() % sizeof(K), 0): ragged key buffer");
    if (kb && kb != w) throw CheckError(kErrArg, "router: streams of one step must share a key type");
    kb = w;
  }
  return kb ? kb : 8;
}

RemoteNode* PushRouter::sender(int32_t stream, int server) {
  auto& p = senders_[{stream, server}];
  if (!p) p.reset(new RemoteNode(ctx_));
  return p.get();
}

RemoteNode* PushRouter::receiver(int server, int32_t stream) {
  auto& p = receivers_[{(int32_t)server, (int)stream}];
  if (!p) p.reset(new RemoteNode(ctx_));
  return p.get();
}

// Executor::Submit for a push to kServerGroup (executor.cc:127-146): slice
// (message.h:107-147), encode each valid slice on its per-peer node.  The
// slices copy the stream's Task and share its buffers, as `new
// Message(msg->task)` plus the zero-copy SArray segments do.
// PSF_SIDE_SLICE (A/B knob, tools/): 0 keeps the prefetched slicing on the main stream
static bool side_slice_mode() {
  static const bool on = [] {
    const char* e = getenv("PSF_SIDE_SLICE");
    return !(e && *e == '0');
  }();
  return on;
}

void PushRouter::encode_launch(const Message* const* streams, int n, bool origin) {
  t_launch_ = now_ns();
  results_.clear();
  enc_.clear();
  local_.clear();
  local_server_.clear();
  plan_.reset();
  pend_.finish();  // (a launch without its finish: complete it first)
  // where the main stream stands before this step's encode: the next step's
  // slicing (prefetch) waits for this point only -- everything the callers
  // enqueued before, not this step's encode and decode
  // (origin false: the multi-step driver's later steps, between which the
  // caller enqueues nothing -- the first step's point still orders them, and a
  // marker in the stream costs it ~3 us, tools/event_gap_probe.hip)
  if (ctx_->device() >= 0 && side_slice_mode() && (origin || !step_start_)) {  // (a host-only context slices on the host)
    if (!step_start_) step_start_ = ctx_->take_marker();
    PSF_HIP_CHECK(hipEventRecord(step_start_, ctx_->stream()));
  }
  std::unique_ptr<SliceJob> job;
  if (next_ && next_->same_inputs(streams, n)) job = std::move(next_);
  next_.reset();
  const int kb = step_key_bytes(streams, n);
  if (job && job->key_bytes != kb) job.reset();
  if (!job) job = slice_begin(ctx_, std::vector<const Message*>(streams, streams + n), ranges_, kb);
  std::vector<std::vector<Message>> parts;
  std::vector<std::vector<bool>> ok;
  std::vector<std::vector<KeySigHint>> hints;
  slice_end(*job, &parts, &ok, &hints);
  job.reset();
  const int S = (int)ranges_.size();
  slices_.clear();
  srv_.clear();
  slices_.reserve((size_t)n * S);
  std::vector<KeySigHint> sh;
  sh.reserve((size_t)n * S);
  std::vector<RemoteNode*> nodes;
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < S; ++d) {
      if (!ok[i][d]) continue;  // the range misses the message's key range: not sent
      slices_.push_back(std::move(parts[i][d]));
      sh.push_back(hints[i][d]);
      nodes.push_back(sender(streams[i]->task.key_channel, d));
      srv_.push_back(d);
    }
  std::vector<Message*> mp(slices_.size());
  for (size_t k = 0; k < slices_.size(); ++k) mp[k] = &slices_[k];
  encode_batch(nodes.data(), mp.data(), (int)slices_.size(), sh.data(), &pend_);
  stat_encode_ns += now_ns() - t_launch_;
}

void PushRouter::encode_finish(int64_t* sizes) {
  const int64_t t0 = now_ns();
  pend_.finish();
  std::vector<Message*> remote;
  std::vector<int> dest, rsrv;
  for (size_t k = 0; k < slices_.size(); ++k) {
    if (keep_enc_) enc_.push_back(Encoded{slices_[k].task.key_channel, srv_[k], slices_[k]});
    const int r = owner(srv_[k]);
    if (r == rank_ && !loopback_) {
      local_.push_back(std::move(slices_[k]));  // delivered (the sender keeps nothing of it)
      local_server_.push_back(srv_[k]);
    } else {
      remote.push_back(&slices_[k]);
      dest.push_back(r);
      rsrv.push_back(srv_[k]);
    }
  }
  plan_.reset(new SpillPlan(ctx_, remote.data(), dest.data(), rsrv.data(), (int)remote.size(), world_));
  for (int r = 0; r < 2 * world_; ++r) sizes[r] = plan_->sizes()[r];
  ++stat_steps;
  stat_encode_ns += now_ns() - t0;
}

// The next step's slicing on the side stream: it reads only the streams' key
// buffers (the callers' templates; no kernel of a step writes them) and
// writes host-mapped records, so it need not queue behind this step's encode
// and decode -- the host then finds it done when the next step starts instead
// of waiting for this step's kernels.
void PushRouter::prefetch(const Message* const* streams, int n) {
  next_ = slice_begin(ctx_, std::vector<const Message*>(streams, streams + n), ranges_, step_key_bytes(streams, n),
                      step_start_);
}

void PushRouter::fill(void* sendbuf) {
  if (!plan_) throw CheckError(kErrArg, "fill() before encode()");
  plan_->fill(sendbuf);
  plan_.reset();
}

void PushRouter::exchange_step() {
  if (!ex_) throw CheckError(kErrArg, "router: no exchange");
  if (ex_->world() != world_ || ex_->rank() != rank_) throw CheckError(kErrArg, "router: exchange of another world");
  int64_t t0 = now_ns();
  pend_.finish();  // COMPRESSING's lengths (the only device wait of the step)
  std::vector<Message*> remote;
  std::vector<int> dest, rsrv;
  for (size_t k = 0; k < slices_.size(); ++k) {
    if (keep_enc_) enc_.push_back(Encoded{slices_[k].task.key_channel, srv_[k], slices_[k]});
    const int r = owner(srv_[k]);
    if (r == rank_ && !loopback_) {
      local_.push_back(std::move(slices_[k]));
      local_server_.push_back(srv_[k]);
    } else {
      remote.push_back(&slices_[k]);
      dest.push_back(r);
      rsrv.push_back(srv_[k]);
    }
  }
  const int W = world_;
  SpillPlan plan(ctx_, remote.data(), dest.data(), rsrv.data(), (int)remote.size(), W, /*host_meta=*/true);
  std::vector<int64_t> meta(W), pay(W);
  std::vector<const uint8_t*> recs(W);
  std::vector<uint64_t> soff(W), roff(W);
  for (int r = 0; r < W; ++r) {
    meta[r] = plan.sizes()[2 * r];
    pay[r] = plan.sizes()[2 * r + 1];
    recs[r] = plan.records(r);
    soff[r] = plan.send_offset(r);
  }
  Buffer send;
  if (plan.total()) {
    if (ctx_->device() >= 0) {
      send = ctx_->alloc(plan.total());
    } else {
      send.loc = Loc::kHost;
      send.bytes = plan.total();
      uint8_t* q = new uint8_t[plan.total()];
      send.owner = std::shared_ptr<void>(q, [](void* v) { delete[] static_cast<uint8_t*>(v); });
      send.ptr = q;
    }
    plan.fill(send.ptr);
  }
  ++stat_steps;
  stat_encode_ns += now_ns() - t0;
  t0 = now_ns();
  ex_->post(meta.data(), pay.data(), recs.data(), send.ptr, soff.data());
  ex_->gather_meta();
  uint64_t total = 0;
  for (int s = 0; s < W; ++s) {
    roff[s] = total;
    total += (uint64_t)ex_->pay_in()[s];
  }
  Buffer recv;
  if (total) {
    if (ctx_->device() >= 0) {
      recv = ctx_->alloc(total);
    } else {
      recv.loc = Loc::kHost;
      recv.bytes = total;
      uint8_t* q = new uint8_t[total];
      recv.owner = std::shared_ptr<void>(q, [](void* v) { delete[] static_cast<uint8_t*>(v); });
      recv.ptr = q;
    }
  }
  std::vector<Message> ms;
  std::vector<int> sv;
  for (int s = 0; s < W; ++s)
    if (ex_->meta_in()[s])
      spill_unpack_host(ctx_, ex_->records_in(s), (uint64_t)ex_->meta_in()[s], recv, roff[s],
                        (uint64_t)ex_->pay_in()[s], &ms, &sv);
  const int S = (int)ranges_.size();
  for (int s : sv)
    if (s < 0 || s >= S || owner(s) != rank_) throw CheckError(kErrCheck, "spill record for a server this rank does not own");
  ex_->move(send.ptr, soff.data(), recv.ptr, roff.data());
  decode_into_results(local_, local_server_);  // beside the transfer
  local_.clear();
  local_server_.clear();
  ex_->join_data();
  // (released only now: the allocator orders reuse on the context's stream,
  // which has just been made to wait for the transfer that reads it)
  send.clear();
  decode_into_results(ms, sv);
  stat_decode_ns += now_ns() - t0;
}

// PickActiveMsg on each server (executor.cc:178-219): decode on the server's
// node for that stream, all of them in one batch.
void PushRouter::decode_into_results(std::vector<Message>& ms, const std::vector<int>& servers) {
  std::vector<RemoteNode*> nodes(ms.size());
  std::vector<Message*> mp(ms.size());
  for (size_t k = 0; k < ms.size(); ++k) {
    nodes[k] = receiver(servers[k], ms[k].task.key_channel);
    mp[k] = &ms[k];
  }
  decode_batch(nodes.data(), mp.data(), (int)ms.size());
  for (size_t k = 0; k < ms.size(); ++k) results_.emplace_back(servers[k], std::move(ms[k]));
}

void PushRouter::decode_local() {
  const int64_t t0 = now_ns();
  decode_into_results(local_, local_server_);
  stat_decode_ns += now_ns() - t0;
  local_.clear();
  local_server_.clear();
}

void PushRouter::decode_local_launch() {
  const int64_t t0 = now_ns();
  decode_local_finish();  // (a launch without its finish: complete it first)
  dec_msgs_ = std::move(local_);
  dec_servers_ = std::move(local_server_);
  local_.clear();
  local_server_.clear();
  dec_nodes_.resize(dec_msgs_.size());
  dec_ptrs_.resize(dec_msgs_.size());
  for (size_t k = 0; k < dec_msgs_.size(); ++k) {
    dec_nodes_[k] = receiver(dec_servers_[k], dec_msgs_[k].task.key_channel);
    dec_ptrs_[k] = &dec_msgs_[k];
  }
  decode_batch(dec_nodes_.data(), dec_ptrs_.data(), (int)dec_msgs_.size(), nullptr, &pend_dec_);
  stat_decode_ns += now_ns() - t0;
}

void PushRouter::decode_local_finish() {
  if (dec_msgs_.empty() && !pend_dec_.active) return;
  const int64_t t0 = now_ns();
  pend_dec_.finish();
  for (size_t k = 0; k < dec_msgs_.size(); ++k) results_.emplace_back(dec_servers_[k], std::move(dec_msgs_[k]));
  dec_msgs_.clear();
  dec_servers_.clear();
  stat_decode_ns += now_ns() - t0;
}

void PushRouter::decode_received(const uint8_t* recvbuf, const int64_t* sizes_in) {
  const int64_t t0 = now_ns();
  uint64_t total = 0;
  for (int r = 0; r < 2 * world_; ++r) total += (uint64_t)sizes_in[r];
  std::vector<Message> ms;
  std::vector<int> sv;
  spill_unpack(ctx_, own_copy(ctx_, recvbuf, total), world_, sizes_in, &ms, &sv);
  // a record names its server: it must be one of this rank's (the sender
  // routed it by owner(server)); anything else is a corrupt or misrouted buffer
  const int S = (int)ranges_.size();
  for (int s : sv)
    if (s < 0 || s >= S || owner(s) != rank_) throw CheckError(kErrCheck, "spill record for a server this rank does not own");
  decode_into_results(ms, sv);
  stat_decode_ns += now_ns() - t0;
}

}  // namespace psf
