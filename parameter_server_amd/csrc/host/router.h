// The multi-server push path of one rank,
// native: what the reference's Executor::Submit does for a kServerGroup push
// -- slice the message at the server key ranges (SliceKOFVMessage,
// message.h:107-147), encode each slice on the sender's per-peer RemoteNode
// (executor.cc:127-146) -- and what each server's PickActiveMsg does with
// what arrives (decode on its per-peer node, executor.cc:178-219), for many
// push streams at once, with no per-slice host work outside this library.
#pragma once
#include <map>
#include <unordered_map>
#include <memory>
#include <utility>
#include <vector>

#include <functional>

#include "exchange.h"
#include "filter.h"
#include "kvstore.h"
#include "slice.h"
#include "spill.h"

namespace psf {

class PushRouter {
 public:
  // ranges: the S server key ranges (contiguous); server s lives on rank
  // s * world / S.  loopback: local slices go through the exchange too.
  PushRouter(Context* ctx, const std::vector<KeyRange>& ranges, int rank, int world, bool loopback);
  Context* context() const { return ctx_; }
  ~PushRouter();

  // Slice + encode every stream's message (templates are copied, as the
  // executor copies the Task), pack the slices for other ranks; sizes[2r],
  // sizes[2r+1] = meta / payload bytes for rank r (see SpillPlan).
  void encode(const Message* const* streams, int n, int64_t* sizes) {
    encode_launch(streams, n);
    encode_finish(sizes);
  }
  // encode() in two halves: everything up to the chains' last position,
  // whose COMPRESSING launches stay in flight, and the wait for them plus the
  // delivery split (the multi-step driver queues the next step's slicing in
  // between)
  // origin: record where the main stream stands for the next prefetch
  // (false only for the multi-step driver's steps after its first)
  void encode_launch(const Message* const* streams, int n, bool origin = true);
  void encode_finish(int64_t* sizes);
  // Launch the slicing pass of the NEXT encode() of the same streams now
  // (called once this step's encode launches are queued, so the pass runs
  // ahead of this step's decodes and the next encode waits for it alone).
  // Only valid when nothing changes the streams' keys in between -- the
  // multi-step driver (psf_router_step) -- and dropped if the inputs differ.
  void prefetch(const Message* const* streams, int n);
  // write the send buffer of the last encode()
  void fill(void* sendbuf);
  // decode the slices whose server is on this rank
  void decode_local();
  // decode_local() in two halves (the multi-step driver queues the next
  // step's encode in between, so the device goes from this step's decode to
  // the next step's min/max pass with no wait for the host): the launches --
  // a chain that ends in COMPRESSING leaves its uncompress in flight -- and
  // the wait plus the chains' remaining decodes
  void decode_local_launch();
  void decode_local_finish();
  // The native exchange (exchange.h) the multi-step driver moves slices for
  // other ranks through; then one whole step after encode_launch() is
  // exchange_step(): the delivery split, the Task records posted to the
  // node's mailbox and the data gathered into one send buffer (the computed
  // FIXING_FLOAT ranges travel on the device), this rank's records read,
  // the data moved (RCCL, on the exchange's stream) while the local slices
  // decode, then the received slices decoded where they landed.  No host
  // wait on the device except COMPRESSING's lengths.
  // (the router holds a reference: the exchange outlives it whatever the
  // order the handles are destroyed in)
  void set_exchange(Exchange* ex) {
    Exchange::ref(ex);
    Exchange::unref(ex_);
    ex_ = ex;
  }
  Exchange* exchange() const { return ex_; }
  bool loopback() const { return loopback_; }
  void exchange_step();
  // unpack a receive buffer (segments of ranks 0..world-1) and decode it
  void decode_received(const uint8_t* recvbuf, const int64_t* sizes_in);

  // ---- the pull leg (SURVEY.md §3 CS-2, §8(e) "on the pull side") ----
  // A pull of every stream's keys from the server group: each request is
  // sliced at the server ranges and encoded on the sender's per-(stream,
  // server) node (Executor::Submit, executor.cc:108-147); each server decodes
  // its slice on its per-(server, stream) node, answers it as
  // Parameter::ProcessRequest does for a pull (parameter.cc:5-31: the
  // response is a copy of the request, KVMap::GetValue appends the values,
  // kv_map.h:69-77) and encodes the response on that same node with
  // task.request = false (Executor::Reply, executor.cc:150-167) -- KEY_CACHING
  // hits and elides the keys, FIXING_FLOAT computes the slice's own min/max;
  // the response travels back to the requesting rank, which decodes it on the
  // node that sent the request (keys restored from its cache) and merges it
  // into the stream's key-ordered value array (KVVector::SetValue,
  // kv_vector.h:129-212: ParallelOrderedMatch of the slice's sorted keys into
  // the stream's zeroed array -- the slice is a contiguous run of those keys,
  // so the match is the run's offset; the FIXING_FLOAT decode writes there
  // directly).
  // store: the KVMap of this rank's servers (the router holds a reference)
  void set_store(KvMapFtrl* store) {
    KvMapFtrl::ref(store);
    KvMapFtrl::unref(store_);
    store_ = store;
  }
  KvMapFtrl* store() const { return store_; }
  // one whole pull step: through the native exchange (any world), or all
  // local (world 1 without loopback)
  // prefetch_next: queue the next pull's slicing of the same requests on the
  // side stream (the multi-step driver, as prefetch() for pushes)
  void pull_step(const Message* const* reqs, int n, bool origin = true, bool prefetch_next = false);
  // the same in three phases around a caller-driven all-to-all-v (sizes as
  // encode(); fill() writes each send buffer): the requests out, the
  // requests served and the responses out, the responses merged
  void pull_encode(const Message* const* reqs, int n, int64_t* sizes);
  void pull_serve(const uint8_t* recvbuf, const int64_t* sizes_in, int64_t* sizes);
  void pull_finish(const uint8_t* recvbuf, const int64_t* sizes_in);
  // per requesting stream: its keys and the pulled values in key order
  // (value_type FLOAT), valid until the next pull
  struct Pulled { int32_t stream; Message msg; };
  const std::vector<Pulled>& pulled() const { return pulled_; }

  // decoded messages of the last step: (server, message)
  const std::vector<std::pair<int, Message>>& results() const { return results_; }
  // encoded slices of the last step: (stream key_channel, server, message)
  struct Encoded { int32_t stream; int server; Message msg; };
  const std::vector<Encoded>& encoded() const { return enc_; }
  void keep_encoded(bool v) { keep_enc_ = v; }
  int owner(int server) const { return (int)((int64_t)server * world_ / (int64_t)ranges_.size()); }
  int world() const { return world_; }
  // host phase timers: steps, ns in encode(), ns in decode_local/received()
  int64_t stat_steps = 0, stat_encode_ns = 0, stat_decode_ns = 0;

 private:
  RemoteNode* sender(int32_t stream, int server);
  RemoteNode* receiver(int server, int32_t stream);
  void decode_into_results(std::vector<Message>& ms, const std::vector<int>& servers);
  // messages received in one exchange round: (message, server, source rank)
  struct Inbox {
    std::vector<Message> msgs;
    std::vector<int> server, src;
  };
  // One round of the native exchange: out[i] to rank dest[i] for server
  // srv[i]; `beside` is queued while the data moves; the received messages
  // are appended to *in with their data joined on the context's stream.
  // own_servers: a received server must be this rank's (requests); else it
  // must be the source rank's (pull responses).
  void exchange_round(const std::vector<Message*>& out, const std::vector<int>& dest, const std::vector<int>& srv,
                      const std::function<void()>& beside, Inbox* in, bool own_servers);
  void check_inbox(const Inbox& in, size_t from, bool own_servers) const;
  // pull phases (see pull_step)
  void pull_begin(const Message* const* reqs, int n, bool origin, Inbox* local, std::vector<Message*>* remote,
                  std::vector<int>* dest, std::vector<int>* rsrv, bool prefetch_next = false);
  void pull_answer(Inbox& reqs, Inbox* local, std::vector<Message>* resp, std::vector<Message*>* remote,
                   std::vector<int>* dest, std::vector<int>* rsrv);
  void pull_merge(Inbox& resp);

  Context* ctx_;
  Exchange* ex_ = nullptr;
  KvMapFtrl* store_ = nullptr;
  std::vector<KeyRange> ranges_;
  int rank_, world_;
  bool loopback_;
  bool keep_enc_ = false;
  // per (stream channel, server) / (server, stream channel), keyed (a << 32) | b
  std::unordered_map<uint64_t, std::unique_ptr<RemoteNode>> senders_, receivers_;
  std::vector<Message> local_;
  std::vector<int> local_server_;
  std::unique_ptr<SpillPlan> plan_;
  std::vector<std::pair<int, Message>> results_;
  std::vector<Encoded> enc_;
  std::unique_ptr<SliceJob> next_;
  hipEvent_t step_start_ = nullptr;  // the main stream at this step's encode launch (prefetch waits on it)
  // the step between encode_launch and encode_finish
  std::vector<Message> slices_;
  std::vector<int> srv_;
  // per slice: its stream (index into the step's streams), first key and
  // key count within the stream's key array
  std::vector<int> sl_stream_;
  std::vector<uint64_t> sl_koff_, sl_nkeys_;
  // the pull in progress: (stream channel, server) -> (stream index, slice)
  std::map<std::pair<int32_t, int>, std::pair<int, size_t>> ppos_;
  std::vector<uint64_t> pout_off_;  // per stream: its array's offset in pout_
  Buffer pout_;
  std::vector<Pulled> pulled_;
  std::vector<uint64_t> pl_koff_, pl_nkeys_;  // the pull's slices (copies of sl_*)
  Inbox preq_local_, presp_local_;  // the caller-driven pull's local deliveries
  std::vector<Message> presp_;      // its responses (sent from plan_)
  PendingEncode pend_;
  int64_t t_launch_ = 0;
  // the step whose decode is in flight (decode_local_launch .. _finish); its
  // messages outlive pend_dec_, which finishes them if it must
  std::vector<Message> dec_msgs_;
  std::vector<int> dec_servers_;
  std::vector<RemoteNode*> dec_nodes_;
  std::vector<Message*> dec_ptrs_;
  PendingDecode pend_dec_;
};

}  // namespace psf
