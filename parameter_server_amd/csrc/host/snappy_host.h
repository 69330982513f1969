// COMPRESSING buffers: compress / uncompress the arrays of one message or of
// a batch of messages in batched launch chains with one wait at the end (each
// stream publishes its length / verdict to its own host-mapped slot).
#pragma once
#include <vector>

#include "context.h"

namespace psf {

uint32_t snappy_parse_header(const uint8_t* p, size_t n, uint64_t* len);
// tests: the uncompress's tail kernels run even when the fast path published
// every verdict (psf_debug_force_snappy_tail)
bool snappy_force_tail();
// header of a (device or host) buffer; 0 when malformed
uint32_t snappy_read_header(Context& c, const Buffer& in, uint64_t* len);

class SnappyBatch {
 public:
  // slot0: the first of the kSyncSlots publish slots its streams use (a
  // batch left in flight takes its own region, Context::kCompressSlot0 /
  // kDecodeSlot0)
  explicit SnappyBatch(Context& c, int slot0 = 0) : slot0_(slot0), c_(c) {}
  // *dst is assigned at flush(); src must stay alive until then
  void compress(const Buffer& src, Buffer* dst);
  // size_hint: the uncompressed length the sender recorded (COMPRESSING's
  // FilterConfig); the launch is sized from it without reading the stream's
  // header to the host, the device checks the header against it, and a
  // mismatch is redone from the header at flush()
  void uncompress(const Buffer& src, Buffer* dst, const uint64_t* size_hint = nullptr);
  // The same, with FIXING_FLOAT's decode fused (SnappyDequant; dq.values is
  // allocated here): at flush() *dst receives the values and *fused is set,
  // or -- when the stream's header disagrees with the hint, which the fused
  // launch cannot follow -- every stream of `group` is decoded again unfused
  // and *dst receives codes as uncompress() would give.
  void uncompress_dequant(const Buffer& src, Buffer* dst, uint64_t size_hint, const SnappyDequant& dq,
                          bool* fused, int group);
  // one launch chain per kSnappyBatchMax streams of a kind, then one wait
  void flush() {
    launch_all();
    finish();
  }
  // flush() in two halves: the launches, and the wait that assigns the *dst
  // (the publish slots stay taken in between)
  void launch_all();
  void finish();

 private:
  struct Job {
    bool compress = false;
    Buffer in, out;
    Buffer* dst = nullptr;
    Buffer src;      // uncompress with a size hint: redone from the header on mismatch
    bool hinted = false;
    uint32_t hdr = 0;
    int slot = 0;
    uint32_t ticket = 0;
    SnappyDequant dq;     // fused decode (dq.values: the values buffer's pointer)
    Buffer values;
    bool* fused = nullptr;
    int group = -1;       // streams decoded again together when one falls back
  };
  int slot0_;
  // an uncompress batch launched with its fast path only (SnappyTail): the
  // rest is launched at finish() unless every stream published its verdict
  struct Tail {
    SnappyTail t;
    // recorded after the fast path (a marker: polled beside the publish
    // slots; if it completes before a verdict shows, the tail kernels run and
    // find the stream decoded)
    hipEvent_t done = nullptr;
    std::vector<size_t> jobs;
    Buffer scratch;             // alive until the tail has been launched
  };
  Context& c_;
  std::vector<Job> jobs_;
  std::vector<Tail> tails_;
  size_t launched_ = 0;  // jobs_[0, launched_) are in flight
  void prepare_uncompress(Job& j, const Buffer& src, uint32_t hdr, uint64_t dsize);
  void launch(size_t b, size_t e);
};

}  // namespace psf
