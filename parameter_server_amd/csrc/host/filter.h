// The reference's filter plugin surface (src/filter/filter.h:9-24), restated for
// HBM-resident messages.  Filter::create is the registration point
// (filter.cc:9-23); each codec is a Filter subclass whose encode/decode launch
// libpsf's HIP kernels on the owning node's Context stream.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>

#include "context.h"
#include "message.h"
#include "snappy_host.h"

namespace psf {

class Filter {
 public:
  explicit Filter(Context* ctx) : ctx_(ctx) {}
  virtual ~Filter() {}

  // filter.cc:9-23; unknown types are fatal there (CHECK), an error here.
  static Filter* create(const FilterConfig& conf, Context* ctx);

  virtual void encode(Message* msg) {}
  virtual void decode(Message* msg) {}
  // FIXING_FLOAT decode may leave its codes for the consumer to dequantise
  // (see PendingDequant); set by RemoteNode::set_defer_dequant.
  void set_defer_dequant(bool v) { defer_dequant_ = v; }
  bool defer_dequant() const { return defer_dequant_; }

  // filter.cc:26-31: the first config of that type, or null.
  static FilterConfig* find(FilterConfig::Type type, Message* msg) { return find(type, &msg->task); }
  static FilterConfig* find(FilterConfig::Type type, Task* task);

 protected:
  Context* ctx_;
  bool defer_dequant_ = false;
};

// KEY_CACHING, key_caching.h:6-76
class KeyCachingFilter : public Filter {
 public:
  using Filter::Filter;
  void encode(Message* msg) override;
  void decode(Message* msg) override;
  // the same with the key signature computed by the caller (batched CRCs)
  void encode_with(Message* msg, uint32_t sig);
  void decode_with(Message* msg, uint32_t sig);
  static bool needs_signature(Message* msg, bool encode);
  size_t cache_size() const { return live_; }  // live entries (a cleared entry may be kept, reset)

 private:
  struct CacheKey {
    int32_t channel;
    KeyRange range;
    bool operator==(const CacheKey& o) const { return channel == o.channel && range == o.range; }
  };
  struct CacheKeyHash {
    size_t operator()(const CacheKey& k) const {
      uint64_t h = (uint64_t)(uint32_t)k.channel * 0x9E3779B97F4A7C15ull;
      h ^= k.range.begin + 0x7F4A7C159E3779B9ull + (h << 6) + (h >> 2);
      h ^= k.range.end + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
      return (size_t)h;
    }
  };
  struct Entry {
    uint32_t sig = 0;
    Buffer key;  // zero-copy reference, as the reference caches the SArray
  };
  static bool is_done(const Task& t) { return !t.request || (t.has_param && t.push); }  // :63-67
  uint32_t signature(const Buffer& key);
  // after entry `e` went from live `was` to its current state: count it, and
  // once reset entries outnumber live ones (and kMaxIdle), erase them all --
  // the reference erases at once (key_caching.h:31,57); keeping a reset node
  // saves an allocation per round trip, this bounds what is kept
  void account(bool was, const Entry& e);
  static constexpr size_t kMaxIdle = 4096;
  size_t live_ = 0;

  std::unordered_map<CacheKey, Entry, CacheKeyHash> cache_;
  static constexpr size_t kMaxSigLen = 2048;  // key_caching.h:74
  std::mutex mu_;
};

// FIXING_FLOAT, fixing_float.h:6-103
struct FfMessage {
  Message* msg;
  bool defer;  // the decoding node defers the dequantise (see PendingDequant)
};
class FixingFloatFilter : public Filter {
 public:
  using Filter::Filter;
  void encode(Message* msg) override { convert(msg, true); }
  void decode(Message* msg) override { convert(msg, false); }
  // the element work of many messages at once (FIXING_FLOAT is stateless)
  // lazy: computed min/max stay on the device (FixedFloatConfig::pending)
  // instead of a host wait per batch
  static void encode_messages(Context* ctx, std::vector<FfMessage>& msgs, bool lazy = false);
  static void decode_messages(Context* ctx, std::vector<FfMessage>& msgs);

 private:
  void convert(Message* msg, bool encode);
};

class RemoteNode;

// COMPRESSING, compressing.h:6-38 (snappy raw format)
class CompressingFilter : public Filter {
 public:
  using Filter::Filter;
  void encode(Message* msg) override;
  void decode(Message* msg) override;
  // the arrays of several messages on one context in batched launch chains
  // (same result as encode / decode on each message in turn)
  // defer: launch only, and hand the batch over (its finish() assigns the
  // compressed buffers)
  static void encode_messages(Context* ctx, const std::vector<Message*>& msgs,
                              std::unique_ptr<SnappyBatch>* defer = nullptr);
  // nodes (optional, one per message): where a message's next decodes are
  // KEY_CACHING then FIXING_FLOAT on that node, FIXING_FLOAT's decode runs
  // fused into the uncompress for every value array it can take
  // (Message::predecoded)
  static void decode_messages(Context* ctx, const std::vector<Message*>& msgs,
                              const std::vector<RemoteNode*>* nodes = nullptr);
  // decode_messages in two halves: the launches (the uncompress kernels in
  // flight, the publish slots taken), and the wait that assigns the arrays
  // and marks the fused ones (Message::predecoded)
  struct DecodeInFlight {
    std::unique_ptr<SnappyBatch> batch;
    std::vector<std::unique_ptr<bool[]>> fused;
    std::vector<Message*> owners;
  };
  static void decode_launch(Context* ctx, const std::vector<Message*>& msgs, const std::vector<RemoteNode*>* nodes,
                            DecodeInFlight* st, int slot0);
  static void decode_finish(DecodeInFlight* st);
};

// NOISE, add_noise.h:9-41
class AddNoiseFilter : public Filter {
 public:
  using Filter::Filter;
  void encode(Message* msg) override;
};

// RemoteNode's chain driver (remote_node.cc:7-29, remote_node.h:35-65): one
// filter instance per filter type per peer, created from the first config
// seen; encode in task.filter order, decode in reverse.
class RemoteNode {
 public:
  explicit RemoteNode(Context* ctx) : ctx_(ctx) {}
  ~RemoteNode() { for (auto& f : filters_) delete f.second; }
  void EncodeMessage(Message* msg);
  void DecodeMessage(Message* msg);
  Filter* FindFilterOrCreate(const FilterConfig& conf);
  Context* ctx() const { return ctx_; }
  // Server side: let FIXING_FLOAT's decode hand its codes to the consumer
  // (KvMapFtrl / ordered match dequantise them in-register).
  void set_defer_dequant(bool v);
  bool defer_dequant() const { return defer_dequant_; }

 private:
  Context* ctx_;
  bool defer_dequant_ = false;
  std::unordered_map<int, Filter*> filters_;
};

// A KEY_CACHING signature computed before the chain ran (the slicer's fused
// pass, slice.cc): the CRC32C of the first min(2048, bytes) bytes of the key
// buffer at `ptr`.  Used only while the message's key is still that buffer.
struct KeySigHint {
  const uint8_t* ptr = nullptr;
  size_t bytes = 0;
  uint32_t crc = 0;
  bool matches(const Buffer& key) const { return ptr && ptr == key.ptr && bytes == key.bytes; }
};

// RemoteNode::EncodeMessage / DecodeMessage of n messages at once, message i
// on nodes[i] (each message still runs its own chain, in its own order, on its
// own node's filter instances; stateful filters see their messages in array
// order).  FIXING_FLOAT's element work is batched across the messages.
// hints: null, or one per message.
// COMPRESSING launches of an encode_batch left in flight (pend argument):
// the compressed buffers are assigned by finish().  Only the last filter
// position is ever deferred, so nothing else in the batch waits on them.
struct PendingEncode {
  std::vector<std::unique_ptr<SnappyBatch>> snappy;
  void finish() {
    for (auto& b : snappy) b->finish();
    snappy.clear();
  }
};
void encode_batch(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints = nullptr,
                  PendingEncode* pend = nullptr);
// hints: as encode_batch's, for the receiver's check of keys that arrive
// (key_caching.h:43): used only while the message's key is that buffer.
// A decode_batch whose first position (the last filter of every chain) is
// COMPRESSING for every message, left in flight after its uncompress
// launches (decode_batch's `later` argument): finish() waits for them and
// runs the chains' remaining positions.  The messages, nodes and hints must
// outlive finish(); a pending decode that is never finished is finished by
// its destructor.
struct PendingDecode {
  std::vector<RemoteNode*> nodes;
  std::vector<Message*> msgs;
  std::vector<KeySigHint> hints;
  std::vector<CompressingFilter::DecodeInFlight> cz;
  bool active = false;
  void finish();
  ~PendingDecode();
};
void decode_batch(RemoteNode* const* nodes, Message* const* msgs, int n, const KeySigHint* hints = nullptr,
                  PendingDecode* later = nullptr);
// The in-process round-trip drivers (psf_node(s)_roundtrip_ex) deliver the
// sender's key buffer itself, zero-copy and unchanged, so every KEY_CACHING
// CRC of an iteration can be queued up front: per distinct device key buffer
// of msgs (chains with KEY_CACHING), one CRC job for the sender's signature
// (key_caching.h:18) and one more over the same bytes for the receiver's
// check (key_caching.h:43), all in one batch with one host wait; enc[i] /
// dec[i] receive them (left empty for host keys and key-less messages).
void presign_roundtrip(RemoteNode* const* nodes, const Message* const* msgs, int n, KeySigHint* enc,
                       KeySigHint* dec);
// The same in two halves: presign_launch queues the CRCs (ahead: into the
// context's presign slots, so the caller can queue them one iteration early,
// behind that iteration's encodes, and collect them at the start of the next
// one with no wait; falls back to waiting in presign_finish when they do not
// fit), presign_finish collects them.
struct PresignJob {
  struct Buf {
    Context* ctx;
    const uint8_t* ptr;
    size_t bytes;
    int first, last;  // the messages with this key buffer: first, next[first], ..., last
    uint32_t tk[2];
    int slot0;
  };
  std::vector<Buf> bufs;
  std::vector<int> next;  // per message: the next message of its buffer, or -1
  bool ahead = false;
};
// after_main: the side stream first waits for the main stream's current
// position (the first presign of a driver call: the keys may have been
// written there); false for the later ones of the same call
PresignJob presign_launch(RemoteNode* const* nodes, const Message* const* msgs, int n, bool ahead,
                          bool after_main);
void presign_finish(PresignJob& J, KeySigHint* enc, KeySigHint* dec);

// Run the dequantise a deferred FIXING_FLOAT decode left pending (every
// pending value array of msg becomes decoded data, as DecodeMessage would
// have produced).
void materialize(Context* ctx, Message* msg);

}  // namespace psf
