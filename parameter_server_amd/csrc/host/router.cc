#include "router.h"

#include <stdlib.h>

#include <algorithm>

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
  pend_.finish();
  pend_dec_.finish();
  Exchange::unref(ex_);
  KvMapFtrl::unref(store_);
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
  auto& p = senders_[(uint64_t)(uint32_t)stream << 32 | (uint32_t)server];
  if (!p) p.reset(new RemoteNode(ctx_));
  return p.get();
}

RemoteNode* PushRouter::receiver(int server, int32_t stream) {
  auto& p = receivers_[(uint64_t)(uint32_t)server << 32 | (uint32_t)stream];
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
  slices_.clear();
  srv_.clear();
  sl_stream_.clear();
  sl_koff_.clear();
  sl_nkeys_.clear();
  std::vector<KeySigHint> sh;
  {
    PSF_HPROF(12);
    // only the slices that are sent, built where they stay (slices_)
    slice_end_flat(*job, &slices_, &sl_stream_, &srv_, &sh, &sl_koff_);
  }
  job.reset();
  std::vector<RemoteNode*> nodes(slices_.size());
  sl_nkeys_.resize(slices_.size());
  for (size_t k = 0; k < slices_.size(); ++k) {
    sl_nkeys_[k] = slices_[k].key.bytes / (uint64_t)kb;
    nodes[k] = sender(streams[sl_stream_[k]]->task.key_channel, srv_[k]);
  }
  std::vector<Message*> mp(slices_.size());
  for (size_t k = 0; k < slices_.size(); ++k) mp[k] = &slices_[k];
  {
    PSF_HPROF(13);
    encode_batch(nodes.data(), mp.data(), (int)slices_.size(), sh.data(), &pend_);
  }
  stat_encode_ns += now_ns() - t_launch_;
}

void PushRouter::encode_finish(int64_t* sizes) {
  const int64_t t0 = now_ns();
  {
    PSF_HPROF(15);
    pend_.finish();
  }
  local_.reserve(local_.size() + slices_.size());
  local_server_.reserve(local_server_.size() + slices_.size());
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
  PSF_HPROF(1);
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
  const int64_t t0 = now_ns();
  pend_.finish();  // COMPRESSING's lengths (the only device wait of the step)
  local_.reserve(local_.size() + slices_.size());
  local_server_.reserve(local_server_.size() + slices_.size());
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
  ++stat_steps;
  Inbox in;
  exchange_round(remote, dest, rsrv, [&] {
    decode_into_results(local_, local_server_);  // beside the transfer
    local_.clear();
    local_server_.clear();
  }, &in, true);
  decode_into_results(in.msgs, in.server);
  stat_decode_ns += now_ns() - t0;
}

void PushRouter::check_inbox(const Inbox& in, size_t from, bool own_servers) const {
  const int S = (int)ranges_.size();
  for (size_t k = from; k < in.server.size(); ++k) {
    const int s = in.server[k];
    if (s < 0 || s >= S) throw CheckError(kErrCheck, "spill record names no server");
    if (own_servers && owner(s) != rank_) throw CheckError(kErrCheck, "spill record for a server this rank does not own");
    if (!own_servers && owner(s) != in.src[k])
      throw CheckError(kErrCheck, "pull response from a rank that does not host its server");
  }
}

void PushRouter::exchange_round(const std::vector<Message*>& out, const std::vector<int>& dest,
                                const std::vector<int>& srv, const std::function<void()>& beside, Inbox* in,
                                bool own_servers) {
  if (!ex_) throw CheckError(kErrArg, "router: no exchange");
  if (ex_->world() != world_ || ex_->rank() != rank_) throw CheckError(kErrArg, "router: exchange of another world");
  const int W = world_;
  SpillPlan plan(ctx_, out.data(), dest.data(), srv.data(), (int)out.size(), W, /*host_meta=*/true);
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
  auto host_buffer = [](uint64_t bytes) {
    Buffer b;
    b.loc = Loc::kHost;
    b.bytes = bytes;
    uint8_t* q = new uint8_t[bytes];
    b.owner = std::shared_ptr<void>(q, [](void* v) { delete[] static_cast<uint8_t*>(v); });
    b.ptr = q;
    return b;
  };
  if (plan.total()) {
    send = ctx_->device() >= 0 ? ctx_->alloc(plan.total()) : host_buffer(plan.total());
    plan.fill(send.ptr);
  }
  ex_->post(meta.data(), pay.data(), recs.data(), send.ptr, soff.data());
  // from here until move() the step is half done on the mailbox: an error
  // marks the exchange failed (fail-fast for this rank and its peers)
  const size_t first = in->msgs.size();
  try {
    ex_->gather_meta();
    uint64_t total = 0;
    for (int s = 0; s < W; ++s) {
      roff[s] = total;
      total += (uint64_t)ex_->pay_in()[s];
    }
    Buffer recv;
    if (total) recv = ctx_->device() >= 0 ? ctx_->alloc(total) : host_buffer(total);
    for (int s = 0; s < W; ++s) {
      if (!ex_->meta_in()[s]) continue;
      spill_unpack_host(ctx_, ex_->records_in(s), (uint64_t)ex_->meta_in()[s], recv, roff[s],
                        (uint64_t)ex_->pay_in()[s], &in->msgs, &in->server);
      in->src.resize(in->server.size(), s);
    }
    check_inbox(*in, first, own_servers);
    ex_->move(send.ptr, soff.data(), recv.ptr, roff.data());
  } catch (const std::exception& e) {
    ex_->fail(e.what());
    throw;
  }
  if (beside) beside();
  ex_->join_data();
  // (released only now: the allocator orders reuse on the context's stream,
  // which has just been made to wait for the transfer that reads it)
  send.clear();
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
  results_.reserve(results_.size() + ms.size());
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
  PSF_HPROF(0);
  decode_batch(dec_nodes_.data(), dec_ptrs_.data(), (int)dec_msgs_.size(), nullptr, &pend_dec_);
  stat_decode_ns += now_ns() - t0;
}

void PushRouter::decode_local_finish() {
  if (dec_msgs_.empty() && !pend_dec_.active) return;
  PSF_HPROF(5);
  const int64_t t0 = now_ns();
  pend_dec_.finish();
  // the step's results are exactly its local decodes (the multi-step driver
  // has already queued the next step's encode_launch, which cleared results_
  // while this step's decodes were in flight: replace, never append)
  results_.clear();
  results_.reserve(dec_msgs_.size());
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

// ------------------------------------------------------------ pull leg ----
// Worker side of a pull (Executor::Submit, executor.cc:108-147): slice and
// encode every stream's request on its per-(stream, server) sender node; lay
// out the key-ordered results; split the slices into the ones this rank's
// servers answer (delivered as they are) and the ones for other ranks.
void PushRouter::pull_begin(const Message* const* reqs, int n, bool origin, Inbox* local,
                            std::vector<Message*>* remote, std::vector<int>* dest, std::vector<int>* rsrv,
                            bool prefetch_next) {
  if (!store_) throw CheckError(kErrArg, "router: a pull needs the servers' store (psf_router_set_store)");
  if (store_->context() != ctx_) throw CheckError(kErrArg, "router: the store lives on another context");
  for (int i = 0; i < n; ++i) {
    const Message& m = *reqs[i];
    if (!m.task.request || (m.task.has_param && m.task.push))
      throw CheckError(kErrArg, "router: a pull request has task.request set and param.push clear");
    if (!m.value.empty()) throw CheckError(kErrArg, "router: a pull request carries keys only (kv_vector.h:256-262)");
    if (!m.key.empty() && !(m.task.has_key_type && m.task.key_type == 8))
      throw CheckError(kErrArg, "router: KVMap keys are UINT64 (task.key_type)");
    for (int j = 0; j < i; ++j)
      if (reqs[j]->task.key_channel == m.task.key_channel)
        throw CheckError(kErrArg, "router: the streams of one pull need distinct key channels (kv_vector.h:120)");
  }
  encode_launch(reqs, n, origin);
  if (prefetch_next) prefetch(reqs, n);
  pend_.finish();  // COMPRESSING's lengths
  // the results: one HBM block, each stream's float array at a 256-aligned offset
  auto up = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
  pout_off_.assign(n, 0);
  uint64_t total = 0;
  std::vector<uint64_t> covered(n, 0);
  for (int i = 0; i < n; ++i) {
    pout_off_[i] = total;
    total += up(reqs[i]->key.bytes / 8 * 4);
  }
  for (size_t k = 0; k < slices_.size(); ++k) covered[sl_stream_[k]] += sl_nkeys_[k];
  pout_ = total ? ctx_->alloc(total) : Buffer();  // (the store's context is a device one)
  pulled_.clear();
  for (int i = 0; i < n; ++i) {
    const size_t nk = reqs[i]->key.bytes / 8;
    // keys no server range holds get no response: their values stay 0, as in
    // the zero-filled kv.value the reference matches into (kv_vector.h:177-179)
    if (covered[i] != nk && nk)
      PSF_HIP_CHECK(hipMemsetAsync(pout_.ptr + pout_off_[i], 0, nk * 4, ctx_->stream()));
    Pulled p;
    p.stream = reqs[i]->task.key_channel;
    p.msg.task = reqs[i]->task;
    p.msg.task.request = false;
    p.msg.task.filter.clear();
    p.msg.task.has_key = !reqs[i]->key.empty();
    p.msg.key = reqs[i]->key;
    Buffer v = pout_;
    v.ptr = nk ? pout_.ptr + pout_off_[i] : nullptr;
    v.bytes = nk * 4;
    if (!nk) v.clear();
    p.msg.value.push_back(v);
    p.msg.task.value_type.assign(1, kFloat);
    pulled_.push_back(std::move(p));
  }
  ppos_.clear();
  pl_koff_ = sl_koff_;
  pl_nkeys_ = sl_nkeys_;
  for (size_t k = 0; k < slices_.size(); ++k)
    ppos_[{reqs[sl_stream_[k]]->task.key_channel, srv_[k]}] = {sl_stream_[k], k};
  for (size_t k = 0; k < slices_.size(); ++k) {
    if (keep_enc_) enc_.push_back(Encoded{slices_[k].task.key_channel, srv_[k], slices_[k]});
    const int r = owner(srv_[k]);
    if (r == rank_ && !loopback_) {
      local->msgs.push_back(std::move(slices_[k]));
      local->server.push_back(srv_[k]);
      local->src.push_back(rank_);
    } else {
      remote->push_back(&slices_[k]);
      dest->push_back(r);
      rsrv->push_back(srv_[k]);
    }
  }
  ++stat_steps;
}

// Server side: decode every request on its (server, stream) node; answer it
// (Parameter::ProcessRequest, parameter.cc:5-31 -> KVMap::GetValue,
// kv_map.h:69-77) and encode the response on the same node with
// task.request = false (Executor::Reply, executor.cc:150-167); split the
// responses into this rank's own (local) and the ones going back to other
// ranks (their `remote` pointers point into *resp).
void PushRouter::pull_answer(Inbox& reqs, Inbox* local, std::vector<Message>* resp, std::vector<Message*>* remote,
                             std::vector<int>* dest, std::vector<int>* rsrv) {
  const size_t n = reqs.msgs.size();
  std::vector<RemoteNode*> nodes(n);
  std::vector<Message*> mp(n);
  for (size_t k = 0; k < n; ++k) {
    nodes[k] = receiver(reqs.server[k], reqs.msgs[k].task.key_channel);
    mp[k] = &reqs.msgs[k];
  }
  decode_batch(nodes.data(), mp.data(), (int)n);
  resp->clear();
  resp->resize(n);
  std::vector<KeySigHint> hints(n);
  for (size_t k = 0; k < n; ++k) {
    const Message& q = reqs.msgs[k];
    Message& r = (*resp)[k];  // `new Message(*request)`
    r.task = q.task;
    r.key = q.key;
    r.value = q.value;
    r.pending = q.pending;
    if (r.task.has_param && r.task.push) throw CheckError(kErrArg, "router: a push slice in a pull");
    r.task.request = false;  // executor.cc:155
    mp[k] = &r;
    // the response's KEY_CACHING signature is the request's: the decode just
    // checked (keys sent) or restored (keys cached under that signature) this
    // very key buffer, so no CRC launch and no wait for one
    const FilterConfig* kc = Filter::find(FilterConfig::KEY_CACHING, &r.task);
    if (kc && kc->has_signature && !r.key.empty()) hints[k] = KeySigHint{r.key.ptr, r.key.bytes, kc->signature};
  }
  // KVMap::GetValue of every response in one launch, grouped by server: the
  // streams' slices for one server share most of their keys, so a server's
  // lookups run back to back and find the table lines they touch on chip
  std::vector<Message*> by_server(mp.begin(), mp.end());
  {
    std::vector<size_t> ord(n);
    for (size_t k = 0; k < n; ++k) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return reqs.server[a] < reqs.server[b]; });
    for (size_t k = 0; k < n; ++k) by_server[k] = mp[ord[k]];
  }
  store_->get_values(by_server.data(), (int)n);
  PendingEncode pend;
  encode_batch(nodes.data(), mp.data(), (int)n, hints.data(), &pend);
  pend.finish();
  for (size_t k = 0; k < n; ++k) {
    const int src = reqs.src[k];
    if (keep_enc_) enc_.push_back(Encoded{(*resp)[k].task.key_channel, reqs.server[k], (*resp)[k]});
    if (src == rank_ && !loopback_) {
      local->msgs.push_back(std::move((*resp)[k]));
      local->server.push_back(reqs.server[k]);
      local->src.push_back(rank_);
    } else {
      remote->push_back(&(*resp)[k]);
      dest->push_back(src);
      rsrv->push_back(reqs.server[k]);
    }
  }
}

// Worker side: decode every response on the node that sent its request
// (keys restored from that node's cache) straight into the stream's result
// array at the slice's offset; a decode that could not write there (e.g. a
// fused COMPRESSING + FIXING_FLOAT decode) is copied there.
void PushRouter::pull_merge(Inbox& resp) {
  const size_t n = resp.msgs.size();
  std::vector<RemoteNode*> nodes(n);
  std::vector<Message*> mp(n);
  std::vector<size_t> slice(n);
  std::vector<int> stream(n);
  for (size_t k = 0; k < n; ++k) {
    Message& m = resp.msgs[k];
    auto it = ppos_.find({m.task.key_channel, resp.server[k]});
    if (it == ppos_.end()) throw CheckError(kErrCheck, "pull response for a slice this rank did not request");
    stream[k] = it->second.first;
    slice[k] = it->second.second;
    ppos_.erase(it);  // one response per slice
    nodes[k] = sender(m.task.key_channel, resp.server[k]);
    mp[k] = &m;
    const uint64_t nk = pl_nkeys_[slice[k]];
    Buffer dst = pout_;
    dst.ptr = pout_.ptr + pout_off_[stream[k]] + pl_koff_[slice[k]] * 4;
    dst.bytes = nk * 4;
    // (the batched decode writes 16-byte groups: a slice that starts inside
    // one is decoded aside and copied in with the others, one gather launch)
    if (nk && m.value.size() == 1 && (reinterpret_cast<uintptr_t>(dst.ptr) & 15) == 0) m.value_dest.assign(1, dst);
  }
  decode_batch(nodes.data(), mp.data(), (int)n);
  std::vector<DeviceCopy> copies;
  for (size_t k = 0; k < n; ++k) {
    Message& m = resp.msgs[k];
    const uint64_t nk = pl_nkeys_[slice[k]];
    // KVVector::SetValue's checks (kv_vector.h:171-183): one value array of
    // k_ = 1 value per received key, the keys the slice asked for
    if (m.key.bytes != nk * 8) throw CheckError(kErrCheck, "CHECK: the pull response's keys are not the slice's");
    if (!nk) continue;
    if (m.value.size() != 1) throw CheckError(kErrCheck, "CHECK_EQ(i, 0): can only receive one value");
    if (m.is_pending(0)) materialize(ctx_, &m);
    if (m.value[0].bytes != nk * 4) throw CheckError(kErrCheck, "CHECK_EQ(recv_data.size(), recv_key.size() * k_)");
    uint8_t* want = pout_.ptr + pout_off_[stream[k]] + pl_koff_[slice[k]] * 4;
    if (m.value[0].ptr != want) {
      if (m.value[0].loc != Loc::kDevice) m.value[0] = ctx_->to_device(m.value[0]);
      copies.push_back(DeviceCopy{m.value[0].ptr, (uint64_t)(want - pout_.ptr), nk * 4});
    }
  }
  device_copies(ctx_, copies, pout_.ptr);
  // (the copies' sources are freed stream-ordered after the launch)
  // every slice sent was answered (the reference's sent_req_tracker would
  // wait for the rest forever; here it is an error)
  if (!ppos_.empty())
    throw CheckError(kErrCheck, "pull: " + std::to_string(ppos_.size()) + " slice(s) got no response");
}

void PushRouter::pull_step(const Message* const* reqs, int n, bool origin, bool prefetch_next) {
  const int64_t t0 = now_ns();
  if (!ex_ && (world_ > 1 || loopback_))
    throw CheckError(kErrArg, "router: a pull with other ranks needs an exchange");
  Inbox reqs_in;
  std::vector<Message*> remote;
  std::vector<int> dest, rsrv;
  pull_begin(reqs, n, origin, &reqs_in, &remote, &dest, &rsrv, prefetch_next);
  stat_encode_ns += now_ns() - t0;
  const int64_t t1 = now_ns();
  if (ex_) exchange_round(remote, dest, rsrv, nullptr, &reqs_in, true);
  Inbox resp_in;
  std::vector<Message> resp;
  remote.clear();
  dest.clear();
  rsrv.clear();
  pull_answer(reqs_in, &resp_in, &resp, &remote, &dest, &rsrv);
  if (ex_) exchange_round(remote, dest, rsrv, nullptr, &resp_in, false);
  pull_merge(resp_in);
  stat_decode_ns += now_ns() - t1;
}

void PushRouter::pull_encode(const Message* const* reqs, int n, int64_t* sizes) {
  preq_local_ = Inbox();
  std::vector<Message*> remote;
  std::vector<int> dest, rsrv;
  pull_begin(reqs, n, true, &preq_local_, &remote, &dest, &rsrv);
  plan_.reset(new SpillPlan(ctx_, remote.data(), dest.data(), rsrv.data(), (int)remote.size(), world_));
  for (int r = 0; r < 2 * world_; ++r) sizes[r] = plan_->sizes()[r];
}

void PushRouter::pull_serve(const uint8_t* recvbuf, const int64_t* sizes_in, int64_t* sizes) {
  if (plan_) throw CheckError(kErrArg, "pull_serve() before fill()");
  Inbox in;
  uint64_t total = 0;
  for (int r = 0; r < 2 * world_; ++r) total += (uint64_t)sizes_in[r];
  spill_unpack(ctx_, own_copy(ctx_, recvbuf, total), world_, sizes_in, &in.msgs, &in.server, &in.src);
  check_inbox(in, 0, true);
  for (size_t k = 0; k < preq_local_.msgs.size(); ++k) {
    in.msgs.push_back(std::move(preq_local_.msgs[k]));
    in.server.push_back(preq_local_.server[k]);
    in.src.push_back(rank_);
  }
  preq_local_ = Inbox();
  presp_local_ = Inbox();
  std::vector<Message*> remote;
  std::vector<int> dest, rsrv;
  pull_answer(in, &presp_local_, &presp_, &remote, &dest, &rsrv);
  plan_.reset(new SpillPlan(ctx_, remote.data(), dest.data(), rsrv.data(), (int)remote.size(), world_));
  for (int r = 0; r < 2 * world_; ++r) sizes[r] = plan_->sizes()[r];
}

void PushRouter::pull_finish(const uint8_t* recvbuf, const int64_t* sizes_in) {
  if (plan_) throw CheckError(kErrArg, "pull_finish() before fill()");
  Inbox in;
  uint64_t total = 0;
  for (int r = 0; r < 2 * world_; ++r) total += (uint64_t)sizes_in[r];
  spill_unpack(ctx_, own_copy(ctx_, recvbuf, total), world_, sizes_in, &in.msgs, &in.server, &in.src);
  check_inbox(in, 0, false);
  for (size_t k = 0; k < presp_local_.msgs.size(); ++k) {
    in.msgs.push_back(std::move(presp_local_.msgs[k]));
    in.server.push_back(presp_local_.server[k]);
    in.src.push_back(rank_);
  }
  presp_local_ = Inbox();
  presp_.clear();
  pull_merge(in);
}

}  // namespace psf
