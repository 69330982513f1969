// The cross-range spill's exchange between the ranks of one node, native
// (SURVEY.md §8(e)): what replaces the reference's per-server loop of
// point-to-point ZeroMQ sends of the encoded slices (executor.cc:131-146 ->
// Van::Send, van.cc:122-191) when the servers are the ranks of one node.
//
// The message of a slice splits in two, as on the reference's wire: the Task
// frame (protobuf, host-built -- Van::Send serialises it on the host,
// van.cc:145-162) and the data frames (HBM).  Here the Task frames and the
// per-peer byte counts of a step travel through a host shared-memory mailbox
// of the node's ranks (no device read-back, no collective for the sizes),
// and the data frames through RCCL point-to-point over xGMI (one grouped
// send/recv per peer per step, on the exchange's own stream) -- or, for a
// rehearsal of several ranks on one GPU (RCCL refuses that), through the
// same mailbox (`kHost`).
//
// Mailbox (a file mapped MAP_SHARED, in /dev/shm or the temp directory):
// per rank two banks, used by alternate steps; step k of rank r writes bank
// k & 1 (per destination: Task-record bytes, data bytes, the records; kHost:
// the data), then publishes posted[r] = k + 1.  A rank reads step k of every
// source once posted[s] > k and then publishes consumed[r] = k + 1; a rank
// writes bank k & 1 only when every rank has consumed step k - 2.  Every
// wait is bounded (PSF_EXCHANGE_TIMEOUT_S, default 120 s): a rank that died
// or diverged is an error on the others, not a hang.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "context.h"

namespace psf {

class Exchange {
 public:
  enum Transport { kRccl = 0, kHost = 1 };
  // every rank of the node calls this with the same path and id; returns
  // once all `world` ranks have attached (bounded wait).  nccl_id: the
  // 128-byte ncclUniqueId rank 0 made (kRccl only).
  Exchange(Context* ctx, int rank, int world, const std::string& path, Transport t, const void* nccl_id,
           uint64_t meta_cap, uint64_t host_cap);
  ~Exchange();
  // Lifetime (as Context's): the C ABI's handle holds one reference, a router
  // using the exchange one more (psf_router_set_exchange); the last unref
  // deletes the exchange and drops its context reference.
  std::atomic<int> refs{1};
  static void ref(Exchange* e) {
    if (e) e->refs.fetch_add(1, std::memory_order_relaxed);
  }
  static void unref(Exchange* e);
  Context* context() const { return ctx_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  Transport transport() const { return transport_; }

  // one step's send side: meta[d] / pay[d] = the Task-record bytes and the
  // data bytes for rank d (the data at send + soff[d], on the device -- host
  // memory on a host-only context); records[d] = the host records.  Waits
  // until the bank is free, writes, publishes.  kHost: the context's stream
  // is synchronised first (the data must be complete before it is copied).
  void post(const int64_t* meta, const int64_t* pay, const uint8_t* const* records, const uint8_t* send,
            const uint64_t* soff);
  // waits until every source has posted this step; then meta_in[s] /
  // pay_in[s] / records_in(s) describe what rank s sent this rank
  void gather_meta();
  const std::vector<int64_t>& meta_in() const { return meta_in_; }
  const std::vector<int64_t>& pay_in() const { return pay_in_; }
  const uint8_t* records_in(int s) const;
  // move the data: send buffer (as posted) -> recv + roff[s] for every source
  // s.  The device copies run after the context stream's work queued so far
  // and the context stream waits for them (no host wait; kRccl).  kHost:
  // host copies out of the mailbox.  Then marks the step consumed.
  void move(const uint8_t* send, const uint64_t* soff, uint8_t* recv, const uint64_t* roff);
  // the context's stream waits (on the device) for move()'s data; the work
  // queued on it between move() and join_data() overlaps the transfer
  void join_data();
  // A step that failed between post() and move() leaves the mailbox
  // protocol broken for every rank: fail() marks this exchange and the
  // mailbox failed, so the next call here -- and every peer's next wait --
  // throws at once (naming the rank and the cause) instead of timing out.
  void fail(const std::string& why);
  bool failed() const { return !failed_.empty(); }

  int64_t bytes_sent = 0;  // data + Task records posted for other ranks
  int64_t steps = 0;
  int64_t wait_ns = 0;     // host time in mailbox waits
  // data-path accounting: bytes handed to ncclSend and the send calls made
  // (kRccl), bytes copied by the runtime instead (the self slice; kHost:
  // the mailbox copies in)
  int64_t rccl_bytes = 0, rccl_sends = 0, copied_bytes = 0;

  struct Shared;   // the mailbox header (exchange.cc)
  struct RankBox;  // one bank of one rank

 private:
  RankBox* box(int r, int bank) const;
  void check_failed() const;
  void wait_until(const std::atomic<uint64_t>* v, uint64_t want, const char* what, int who);

  Context* ctx_;
  int rank_, world_;
  Transport transport_;
  std::string path_;
  uint8_t* base_ = nullptr;
  size_t map_bytes_ = 0;
  uint64_t meta_cap_, host_cap_, box_bytes_;
  Shared* sh_ = nullptr;
  uint64_t step_ = 0;  // steps posted by this rank
  bool gathered_ = false;
  std::vector<int64_t> meta_in_, pay_in_;
  double timeout_s_ = 120.0;
  std::string failed_;
  // kRccl
  void* comm_ = nullptr;
  hipStream_t cstream_ = nullptr;
  hipEvent_t ev_sent_ = nullptr, ev_done_ = nullptr;
};

// The 128-byte ncclUniqueId of a new RCCL communicator (rank 0 makes it,
// every rank passes it to Exchange).  Loads librccl on first use.
void rccl_unique_id(void* out128);

// Test knob (psf_debug_exchange_self_p2p): a kRccl exchange sends the self
// slice through ncclSend / ncclRecv to its own rank inside the step's group
// instead of a device copy, so a world-1 loopback run executes the grouped
// point-to-point path the node's other ranks take.
void set_exchange_self_p2p(bool on);

}  // namespace psf
