// Cross-range spill: pack a rank's outgoing slices into one send buffer and
// rebuild received messages over the receive buffer (see spill.cc).
#pragma once
#include <vector>

#include "context.h"
#include "message.h"

namespace psf {

class SpillPlan {
 public:
  // message i goes to rank dest[i], addressed to server server[i].
  // host_meta: the Task records stay on the host (records(r), for the native
  // exchange's mailbox) and the send buffer holds only the data of each rank,
  // [frames][side-info block]: the FIXING_FLOAT {min, max} a batched encode
  // left on the device travel there, device to device, instead of being
  // waited for and serialised (record format 'PSSN', see spill.cc)
  SpillPlan(Context* ctx, Message* const* msgs, const int* dest, const int* server, int n, int world,
            bool host_meta = false);
  Context* context() const { return ctx_; }
  // per rank r: sizes()[2r] = meta bytes, sizes()[2r+1] = payload bytes
  const std::vector<int64_t>& sizes() const { return sizes_; }
  uint64_t total() const { return total_; }
  // host_meta: rank r's records (sizes()[2r] bytes) and the offset of its
  // data in the send buffer
  const uint8_t* records(int r) const { return blob_.data() + meta_at_[r]; }
  uint64_t send_offset(int r) const { return seg_[r]; }
  // write the send buffer (device buffer of total() bytes; host memory on a
  // host-only context), ordered on the context's stream
  void fill(void* sendbuf);

 private:
  struct Copy {
    const uint8_t* src;  // device frame, or null: blob_ + blob_off
    uint64_t blob_off;
    uint64_t dst_off;
    uint64_t len;
  };
  Context* ctx_;
  std::vector<int64_t> sizes_;
  std::vector<uint64_t> meta_at_, seg_;
  std::vector<uint8_t> blob_;
  std::vector<Copy> copies_;
  std::vector<Buffer> keep_;
  uint64_t total_ = 0;
};

// Rebuild the messages of a receive buffer laid out by SpillPlan (segments of
// sources 0..world-1 back to back, sizes as the senders reported them).  The
// messages' frames point into `recv` and share its owner (recv.owner null:
// the caller keeps the memory alive).
// srcs (optional): the source rank of each message
int spill_unpack(Context* ctx, const Buffer& recv, int world, const int64_t* sizes, std::vector<Message>* out,
                 std::vector<int>* servers, std::vector<int>* srcs = nullptr);
// a table of device copies (src, dst_off, len) into dst, in one gather launch
// on the context's stream (the sources must stay alive until it has run)
struct DeviceCopy {
  const uint8_t* src;
  uint64_t dst_off, len;
};
void device_copies(Context* ctx, const std::vector<DeviceCopy>& copies, uint8_t* dst);
// The receive side of a host_meta plan: rank s's records (host memory, mlen
// bytes) describe the data at [pay_at, pay_at + plen) of `recv`; the messages
// are appended to out / servers with their frames pointing into `recv`
// (sharing its owner, decoded where they landed) and their FIXING_FLOAT
// side-info pending on the device records that travelled with them.
void spill_unpack_host(Context* ctx, const uint8_t* records, uint64_t mlen, const Buffer& recv, uint64_t pay_at,
                       uint64_t plen, std::vector<Message>* out, std::vector<int>* servers);
// A copy of `bytes` at p that the library owns (HBM on a device context, heap
// memory on a host-only one), so received frames can outlive the caller's
// buffer (KEY_CACHING keeps received keys by reference, key_caching.h:45-47).
Buffer own_copy(Context* ctx, const void* p, size_t bytes);

}  // namespace psf
