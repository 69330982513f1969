#pragma once
#include <vector>

#include "context.h"
#include "message.h"

namespace psf {

// Range<Key>::EvenDivide(n, i), src/util/range.h:100-107
KeyRange even_divide(const KeyRange& r, uint64_t n, uint64_t i);

// SliceKOFVMessage<K>, src/system/message.h:107-147 (key_bytes = sizeof(K))
void slice_message(Context* ctx, const Message& msg, const std::vector<KeyRange>& krs,
                   int key_bytes, std::vector<Message>* outs, std::vector<bool>* valid);
// the same for many messages, with one device synchronisation in all
void slice_messages(Context* ctx, const std::vector<const Message*>& msgs, const std::vector<KeyRange>& krs,
                    int key_bytes, std::vector<std::vector<Message>>* outs,
                    std::vector<std::vector<bool>>* valid);

}  // namespace psf
