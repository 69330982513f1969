#pragma once
#include <memory>
#include <utility>
#include <vector>

#include "context.h"
#include "filter.h"
#include "message.h"

namespace psf {

// Range<Key>::EvenDivide(n, i), src/util/range.h:100-107
KeyRange even_divide(const KeyRange& r, uint64_t n, uint64_t i);

// SliceKOFVMessage<K>, src/system/message.h:107-147 (key_bytes = sizeof(K))
void slice_message(Context* ctx, const Message& msg, const std::vector<KeyRange>& krs,
                   int key_bytes, std::vector<Message>* outs, std::vector<bool>* valid);
// the same for many messages, with one device wait in all
void slice_messages(Context* ctx, const std::vector<const Message*>& msgs, const std::vector<KeyRange>& krs,
                    int key_bytes, std::vector<std::vector<Message>>* outs,
                    std::vector<std::vector<bool>>* valid);

// slice_messages split in two: slice_begin launches the device pass (split
// positions of every device-keyed message, fused with the KEY_CACHING
// signature of every slice, results in host-mapped memory) and returns at
// once; slice_end waits for that launch's event alone -- not for the stream
// -- and builds the slices, with one signature hint per slice (a null hint
// where none was computed).  The messages must stay alive and unchanged in
// between.
struct SliceJob {
  Context* ctx = nullptr;
  std::vector<const Message*> msgs;
  std::vector<KeyRange> krs;
  int key_bytes = 8;
  std::vector<uint64_t> pos;  // M x (n + 1); host-keyed messages filled at begin
  std::vector<size_t> dev;    // device-keyed messages, in launch order
  struct KeyId {
    const uint8_t* ptr;
    size_t bytes;
    bool has_range;
    KeyRange range;
  };
  std::vector<KeyId> ids;  // what each message's slicing depended on
  Context::Pinned buf;
  hipEvent_t ev = nullptr;
  bool ended = false;
  // the same messages with the same key buffers and key ranges
  bool same_inputs(const Message* const* ms, int n) const;
  ~SliceJob();
};
// after: when non-null, the slicing runs on the context's side stream once
// the main stream has reached `after` (a prefetch that must not queue behind
// the main stream's later work); else on the main stream
std::unique_ptr<SliceJob> slice_begin(Context* ctx, const std::vector<const Message*>& msgs,
                                      const std::vector<KeyRange>& krs, int key_bytes, hipEvent_t after = nullptr);
void slice_end(SliceJob& job, std::vector<std::vector<Message>>* outs, std::vector<std::vector<bool>>* valid,
               std::vector<std::vector<KeySigHint>>* hints = nullptr);
// slice_end with the valid slices only, appended flat to *out (message by
// message, ranges in order): per slice its message's index, its range's
// index, its signature hint and the index of its first key in the message
void slice_end_flat(SliceJob& job, std::vector<Message>* out, std::vector<int>* stream, std::vector<int>* server,
                    std::vector<KeySigHint>* hints, std::vector<uint64_t>* first_key);

}  // namespace psf
