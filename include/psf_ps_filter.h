// psf_ps_filter.h -- drop-in adapter between the reference's filter plugin
// surface and libpsf (include/psf.h).
//
// Header-only C++ written against the reference's own types: PS::Filter
// (src/filter/filter.h:9-24), PS::Message (src/system/message.h:10-67),
// PS::SArray (src/util/shared_array.h:29) and the protobuf-generated
// FilterConfig / Task accessors (src/filter/proto/filter.proto:3-35,
// src/system/proto/task.proto:28-39).  A maintainer adds one line to
// Filter::create (src/filter/filter.cc:9-23), see INTEGRATION.md:
//
//     if (Filter* f = psf_hip::CreateFilter(conf)) return f;
//
// The reference's messages live in host memory (ZeroMQ frames,
// src/system/van.cc:244-255), so this adapter is the host edge: each array is
// staged into HBM, coded by libpsf's kernels, and the result comes back as a
// new SArray<char> -- exactly where the reference's filter would put its output
// (fixing_float.h:37-44) -- or, for NOISE, into the value array itself, in
// place, as add_noise.h:33-37 does.  Side-info (fixed_point min/max,
// uncompressed sizes) is written into the message's own FilterConfig as the
// reference does.  libpsf status codes map to the reference's fatal CHECK.
//
// Concurrency: RemoteNode creates one filter instance per type per peer
// (remote_node.cc:7-15), the calls of one instance are serialised by its
// Customer's Executor::node_mu_ (executor.cc:110,143,170), and different
// Customers' executor threads run their instances concurrently (SURVEY.md
// §8(b)).  So every adapter instance owns its libpsf context -- its own
// workspace and order of work, on one of the device's 4 shared HIP streams
// (PSF_STREAM_SHARED: hundreds of peers do not alias hundreds of streams onto
// the hardware queues) -- and no lock is shared between instances.  The cached
// memory of all of them is bounded once per device (psf_set_device_cache_limit).
//
// Filters adapted: all four -- KEY_CACHING, FIXING_FLOAT, COMPRESSING
// (snappy 1.1.8-identical streams) and NOISE.  (Device-resident messages go
// through psf_node_* directly, without this host edge.)
#pragma once
#include <stdint.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "psf.h"

namespace PS {
namespace psf_hip {

inline void Check(int st) { CHECK_EQ(st, PSF_OK) << "libpsf: " << psf_last_error(); }

// One filter instance's libpsf state: a context on the process's device
// (psf_default_device: PSF_DEVICE, else 0) on one of the device's shared
// streams, and a RemoteNode holding the libpsf filter instances.
class Bound {
 protected:
  Bound() {
    Check(psf_context_create(psf_default_device(), nullptr, PSF_STREAM_SHARED, &ctx_));
    Check(psf_node_create(ctx_, &node_));
  }
  ~Bound() {
    psf_node_destroy(node_);
    psf_context_destroy(ctx_);
  }
  // the Task fields the filters read (task.proto:28-39)
  psf_message* NewMessage(const Task& t) {
    psf_message* m = nullptr;
    Check(psf_msg_create(t.request(), t.has_param(), t.has_param() && t.param().push(), t.key_channel(),
                         t.has_key_range(), t.key_range().begin(), t.key_range().end(), &m));
    return m;
  }
  void Run(psf_message* m, bool encode, const char* what) {
    const int st = encode ? psf_node_encode(node_, m) : psf_node_decode(node_, m);
    if (st != PSF_OK) {
      std::string err = psf_last_error();
      psf_msg_destroy(m);
      CHECK(false) << "libpsf " << what << ": " << err;
    }
  }
  // array i (-1 = key) of the libpsf message as an SArray<char>; the input
  // array itself when libpsf left it in place
  SArray<char> Take(psf_message* m, int i, const SArray<char>& in) {
    void* p = nullptr;
    size_t bytes = 0;
    int loc = 0;
    Check(i < 0 ? psf_msg_key(m, &p, &bytes, &loc) : psf_msg_value(m, i, &p, &bytes, &loc));
    if (p == in.data() && bytes == in.size()) return in;
    SArray<char> out(bytes);
    if (bytes) Check(psf_copy_to_host(ctx_, out.data(), p, bytes));
    return out;
  }
  psf_context* ctx_ = nullptr;
  psf_node* node_ = nullptr;
};

// FixingFloatFilter (src/filter/fixing_float.h:6-103) on MI355X.
class FixingFloatFilter : public Filter, Bound {
 public:
  void encode(Message* msg) { convert(msg, true); }
  void decode(Message* msg) { convert(msg, false); }

 private:
  void convert(Message* msg, bool encode) {
    FilterConfig* conf = CHECK_NOTNULL(find(FilterConfig::FIXING_FLOAT, msg));
    if (conf->num_bytes() == 0) return;
    const Task& t = msg->task;
    CHECK_EQ(msg->value.size(), (size_t)t.value_type_size());  // fixing_float.h:28
    // Task + values as a libpsf message (host buffers, not copied)
    psf_message* m = NewMessage(t);
    for (size_t i = 0; i < msg->value.size(); ++i)
      Check(psf_msg_add_value(m, msg->value[i].data(), msg->value[i].size(), (int)t.value_type(i), PSF_LOC_HOST));
    int fi = psf_msg_add_filter(m, PSF_FIXING_FLOAT);
    Check(fi < 0 ? fi : PSF_OK);
    Check(psf_fc_set_num_bytes(m, fi, conf->num_bytes()));
    for (int k = 0; k < conf->fixed_point_size(); ++k) {
      const auto& f = conf->fixed_point(k);
      psf_fixed_point p = {f.has_min_value(), f.has_max_value(), f.min_value(), f.max_value()};
      Check(psf_fc_add_fixed_point(m, fi, &p));
    }
    Run(m, encode, "FIXING_FLOAT");
    // outputs back into the reference's message (new SArray<char>, as
    // fixing_float.h:37-44 replaces msg->value[i])
    for (size_t i = 0; i < msg->value.size(); ++i) msg->value[i] = Take(m, (int)i, msg->value[i]);
    // side-info: the fixed_point list as libpsf left it
    const int nfp = psf_fc_num_fixed_point(m, fi);
    for (int k = 0; k < nfp; ++k) {
      psf_fixed_point p;
      Check(psf_fc_fixed_point(m, fi, k, &p));
      auto* f = k < conf->fixed_point_size() ? conf->mutable_fixed_point(k) : conf->add_fixed_point();
      if (p.has_min) f->set_min_value(p.min_value);
      if (p.has_max) f->set_max_value(p.max_value);
    }
    psf_msg_destroy(m);
  }
};

// CompressingFilter (src/filter/compressing.h:8-37): key (when present) and
// values compressed / uncompressed, uncompressed_size side-info.
class CompressingFilter : public Filter, Bound {
 public:
  void encode(Message* msg) { run(msg, true); }
  void decode(Message* msg) { run(msg, false); }

 private:
  void run(Message* msg, bool encode) {
    FilterConfig* conf = find(FilterConfig::COMPRESSING, msg);
    if (!conf) return;
    const Task& t = msg->task;
    psf_message* m = NewMessage(t);
    const bool had_key = msg->has_key();
    if (had_key) Check(psf_msg_set_key(m, msg->key.data(), msg->key.size(), PSF_DT_CHAR, PSF_LOC_HOST));
    for (size_t i = 0; i < msg->value.size(); ++i) {
      const int vt = i < (size_t)t.value_type_size() ? (int)t.value_type(i) : 0;  // compressing.h reads no types
      Check(psf_msg_add_value(m, msg->value[i].data(), msg->value[i].size(), vt, PSF_LOC_HOST));
    }
    int fi = psf_msg_add_filter(m, PSF_COMPRESSING);
    Check(fi < 0 ? fi : PSF_OK);
    for (int i = 0; i < conf->uncompressed_size_size(); ++i)
      Check(psf_fc_add_uncompressed(m, fi, conf->uncompressed_size(i)));
    Run(m, encode, "COMPRESSING");
    if (had_key) msg->key = Take(m, -1, msg->key);
    for (size_t i = 0; i < msg->value.size(); ++i) msg->value[i] = Take(m, (int)i, msg->value[i]);
    conf->clear_uncompressed_size();
    const int nu = psf_fc_num_uncompressed(m, fi);
    for (int i = 0; i < nu; ++i) {
      uint64_t v = 0;
      Check(psf_fc_uncompressed(m, fi, i, &v));
      conf->add_uncompressed_size(v);
    }
    psf_msg_destroy(m);
  }
};

// AddNoiseFilter (src/filter/add_noise.h:9-41): the noise is added in place,
// on the value arrays themselves, so every SArray sharing them sees it (as
// add_noise.h:33-37 writes through its SArray<V> view).
class AddNoiseFilter : public Filter, Bound {
 public:
  void encode(Message* msg) {
    FilterConfig* conf = CHECK_NOTNULL(find(FilterConfig::NOISE, msg));  // add_noise.h:13
    const Task& t = msg->task;
    CHECK_EQ(msg->value.size(), (size_t)t.value_type_size());  // add_noise.h:14
    psf_message* m = NewMessage(t);
    for (size_t i = 0; i < msg->value.size(); ++i)
      Check(psf_msg_add_value(m, msg->value[i].data(), msg->value[i].size(), (int)t.value_type(i), PSF_LOC_HOST));
    int fi = psf_msg_add_filter(m, PSF_NOISE);
    Check(fi < 0 ? fi : PSF_OK);
    Check(psf_fc_set_noise(m, fi, conf->mean(), conf->std()));
    Run(m, true, "NOISE");
    for (size_t i = 0; i < msg->value.size(); ++i) {
      void* p = nullptr;
      size_t bytes = 0;
      int loc = 0;
      Check(psf_msg_value(m, (int)i, &p, &bytes, &loc));
      if (p != msg->value[i].data() && bytes) {
        CHECK_EQ(bytes, msg->value[i].size());
        Check(psf_copy_to_host(ctx_, msg->value[i].data(), p, bytes));
      }
    }
    psf_msg_destroy(m);
  }
};

// KeyCachingFilter (src/filter/key_caching.h:7-67) through libpsf: the
// signature (CRC32C of the first 2 KiB of the key, :18,43) and the cache per
// (key_channel, key_range) are this instance's libpsf KEY_CACHING filter.
// libpsf's cache entry refers to the key bytes of the message that filled it
// (host memory here), so the adapter keeps that message's SArray beside it:
// the cached key shares ownership as the reference's cache does (:27-28,55).
class KeyCachingFilter : public Filter, Bound {
 public:
  void encode(Message* msg) { run(msg, true); }
  void decode(Message* msg) { run(msg, false); }

 private:
  typedef std::tuple<int, uint64_t, uint64_t> CacheKey;
  static bool Done(const Task& t) { return !t.request() || (t.has_param() && t.param().push()); }  // :63-67

  void run(Message* msg, bool encode) {
    FilterConfig* conf = find(FilterConfig::KEY_CACHING, msg);
    if (!conf || (!encode && !conf->has_signature())) return;
    const Task& t = msg->task;
    psf_message* m = NewMessage(t);
    const bool had_key = msg->has_key();
    if (had_key) Check(psf_msg_set_key(m, msg->key.data(), msg->key.size(), PSF_DT_CHAR, PSF_LOC_HOST));
    const int fi = psf_msg_add_filter(m, PSF_KEY_CACHING);
    Check(fi < 0 ? fi : PSF_OK);
    if (conf->clear_cache_if_done()) Check(psf_fc_set_clear_cache(m, fi, 1));
    if (!encode) Check(psf_fc_set_signature(m, fi, 1, conf->signature()));
    const CacheKey ck(t.key_channel(), t.key_range().begin(), t.key_range().end());
    std::lock_guard<std::mutex> l(mu_);  // "thread safe" (:8), as the reference's mu_
    Run(m, encode, "KEY_CACHING");
    int has = 0;
    uint32_t sig = 0;
    Check(psf_fc_signature(m, fi, &has, &sig));
    if (has)
      conf->set_signature(sig);
    else
      conf->clear_signature();
    void* kp = nullptr;
    size_t kb = 0;
    int loc = 0;
    Check(psf_msg_key(m, &kp, &kb, &loc));
    if (had_key) {
      if (encode && kb == 0)
        msg->clear_key();  // a hit: the receiver restores the key from its cache
      else
        keep_[ck] = msg->key;
    } else if (!encode) {  // restored from the cache (:53-55)
      auto it = keep_.find(ck);
      SArray<char> k = it == keep_.end() ? SArray<char>() : it->second;
      CHECK(k.size() == kb && (kb == 0 || k.data() == kp)) << "KEY_CACHING: adapter cache out of step";
      msg->set_key(k);
    }
    if (conf->clear_cache_if_done() && Done(t)) keep_.erase(ck);
    psf_msg_destroy(m);
  }

  std::map<CacheKey, SArray<char>> keep_;
  std::mutex mu_;
};

// The whole chain of one RemoteNode on one libpsf node: what
// RemoteNode::EncodeMessage / DecodeMessage (remote_node.cc:17-29) do with the
// per-type instances FindFilterOrCreate keeps (remote_node.cc:7-15), in one
// call.  One Chain per RemoteNode (a member the RemoteNode patch adds,
// INTEGRATION.md), so one libpsf context -- device psf_default_device(), one
// of the device's shared streams, its own workspace -- serves all of that peer's
// filters, and the arrays stay in HBM from the first filter to the last:
// encode stages each host array in once (the first filter that touches it)
// and only the chain's result comes back as new SArray<char>s; decode stages
// the received frames in once and brings the decoded arrays back.  The
// batched entry points run it (psf_nodes_encode / _decode with one message),
// so a [.., FIXING_FLOAT, COMPRESSING] decode takes the fused uncompress +
// dequantise.  Chains with NOISE (in place on the caller's buffer,
// add_noise.h:33-37) or an unknown type are left to the per-filter path
// (Encode/Decode return false); so is a message without filters.
class Chain {
 public:
  Chain() {}
  ~Chain() {
    if (node_) psf_node_destroy(node_);
    if (ctx_) psf_context_destroy(ctx_);
  }
  Chain(const Chain&) = delete;
  Chain& operator=(const Chain&) = delete;
  bool Encode(Message* msg) { return Run(msg, true); }
  bool Decode(Message* msg) { return Run(msg, false); }

 private:
  typedef std::tuple<int, uint64_t, uint64_t> CacheKey;
  static bool Done(const Task& t) { return !t.request() || (t.has_param() && t.param().push()); }  // key_caching.h:63-67
  static bool Handles(const Task& t) {
    if (t.filter_size() == 0) return false;
    for (int i = 0; i < t.filter_size(); ++i) {
      const int ty = t.filter(i).type();
      if (ty != FilterConfig::KEY_CACHING && ty != FilterConfig::FIXING_FLOAT && ty != FilterConfig::COMPRESSING)
        return false;
    }
    return true;
  }
  bool Run(Message* msg, bool encode) {
    Task& t = msg->task;
    if (!Handles(t)) return false;
    std::lock_guard<std::mutex> l(mu_);
    if (!ctx_) {
      Check(psf_context_create(psf_default_device(), nullptr, PSF_STREAM_SHARED, &ctx_));
      Check(psf_node_create(ctx_, &node_));
    }
    psf_message* m = nullptr;
    Check(psf_msg_create(t.request(), t.has_param(), t.has_param() && t.param().push(), t.key_channel(),
                         t.has_key_range(), t.key_range().begin(), t.key_range().end(), &m));
    const bool had_key = msg->has_key();
    // the inputs stay referenced until the chain's one sync: their H2D copies
    // run in flight on the stream, and a received zero-copy frame or a pinned
    // SArray from a pool must not be freed or reused under them
    const SArray<char> key_in = msg->key;
    const std::vector<SArray<char>> values_in = msg->value;
    if (had_key) Check(psf_msg_set_key(m, msg->key.data(), msg->key.size(), PSF_DT_CHAR, PSF_LOC_HOST));
    for (size_t i = 0; i < msg->value.size(); ++i) {
      const int vt = i < (size_t)t.value_type_size() ? (int)t.value_type(i) : 0;
      Check(psf_msg_add_value(m, msg->value[i].data(), msg->value[i].size(), vt, PSF_LOC_HOST));
    }
    int kc = -1;
    for (int i = 0; i < t.filter_size(); ++i) {
      const FilterConfig& c = t.filter(i);
      const int fi = psf_msg_add_filter(m, (int)c.type());
      Check(fi < 0 ? fi : PSF_OK);
      switch (c.type()) {
        case FilterConfig::FIXING_FLOAT:
          Check(psf_fc_set_num_bytes(m, fi, c.num_bytes()));
          for (int k = 0; k < c.fixed_point_size(); ++k) {
            const auto& f = c.fixed_point(k);
            psf_fixed_point p = {f.has_min_value(), f.has_max_value(), f.min_value(), f.max_value()};
            Check(psf_fc_add_fixed_point(m, fi, &p));
          }
          break;
        case FilterConfig::KEY_CACHING:
          if (kc < 0) kc = i;
          if (c.clear_cache_if_done()) Check(psf_fc_set_clear_cache(m, fi, 1));
          if (c.has_signature()) Check(psf_fc_set_signature(m, fi, 1, c.signature()));
          break;
        default:  // COMPRESSING
          for (int k = 0; k < c.uncompressed_size_size(); ++k) Check(psf_fc_add_uncompressed(m, fi, c.uncompressed_size(k)));
          break;
      }
    }
    const int st = encode ? psf_nodes_encode(&node_, &m, 1) : psf_nodes_decode(&node_, &m, 1);
    if (st != PSF_OK) {
      std::string err = psf_last_error();
      psf_msg_destroy(m);
      CHECK(false) << "libpsf chain " << (encode ? "encode" : "decode") << ": " << err;
    }
    // side-info into the message's own FilterConfigs
    for (int i = 0; i < t.filter_size(); ++i) {
      FilterConfig* c = t.mutable_filter(i);
      switch (c->type()) {
        case FilterConfig::FIXING_FLOAT: {
          const int nfp = psf_fc_num_fixed_point(m, i);
          for (int k = 0; k < nfp; ++k) {
            psf_fixed_point p;
            Check(psf_fc_fixed_point(m, i, k, &p));
            auto* f = k < c->fixed_point_size() ? c->mutable_fixed_point(k) : c->add_fixed_point();
            if (p.has_min) f->set_min_value(p.min_value);
            if (p.has_max) f->set_max_value(p.max_value);
          }
          break;
        }
        case FilterConfig::KEY_CACHING: {
          int has = 0;
          uint32_t sig = 0;
          Check(psf_fc_signature(m, i, &has, &sig));
          if (has) c->set_signature(sig);
          else c->clear_signature();
          break;
        }
        default: {
          c->clear_uncompressed_size();
          const int nu = psf_fc_num_uncompressed(m, i);
          for (int k = 0; k < nu; ++k) {
            uint64_t v = 0;
            Check(psf_fc_uncompressed(m, i, k, &v));
            c->add_uncompressed_size(v);
          }
        }
      }
    }
    // the key: elided (a KEY_CACHING hit), restored (from the cache), or
    // the chain's output
    void* kp = nullptr;
    size_t kb = 0;
    int kloc = 0;
    Check(psf_msg_key(m, &kp, &kb, &kloc));
    CacheKey ck(t.key_channel(), t.key_range().begin(), t.key_range().end());
    if (had_key && kb == 0) {
      msg->clear_key();
    } else if (kb && !(kloc == PSF_LOC_HOST && kp == key_in.data() && kb == key_in.size())) {
      SArray<char> k;
      auto it = keep_.find(ck);
      if (kloc == PSF_LOC_HOST && it != keep_.end() && it->second.data() == kp && it->second.size() == kb) {
        k = it->second;  // a host key the cache refers to: shared, as key_caching.h:55 shares it
      } else {
        CHECK_EQ(kloc, PSF_LOC_DEVICE) << "libpsf chain: host key of unknown owner";
        k = HostArray(kp, kb);
      }
      if (had_key) msg->key = k;  // a codec's output replaces the key (compressing.h:14,30)
      else msg->set_key(k);       // restored (key_caching.h:55, set_key<char>)
    }
    // libpsf's KEY_CACHING cache may refer to the host key bytes it was
    // given: keep that SArray while the entry lives (the cache is replaced
    // on a miss and on a decode with keys, key_caching.h:27-28,47)
    if (kc >= 0) {
      if (had_key && !(encode && kb == 0)) keep_[ck] = key_in;
      if (t.filter(kc).clear_cache_if_done() && Done(t)) keep_.erase(ck);
    }
    for (size_t i = 0; i < msg->value.size(); ++i) {
      void* p = nullptr;
      size_t bytes = 0;
      int loc = 0;
      Check(psf_msg_value(m, (int)i, &p, &bytes, &loc));
      if (p == msg->value[i].data() && bytes == msg->value[i].size()) continue;
      msg->value[i] = HostArray(p, bytes);
    }
    // one wait for every copy; the device buffers go back to the pool
    // (stream-ordered) with the message
    const int synced = psf_context_sync(ctx_);
    psf_msg_destroy(m);
    Check(synced);
    return true;
  }

  // a chain output as a new SArray<char> in pinned host memory (the copy's
  // fast target), filled by a copy left in flight until the chain's one
  // sync; the SArray's last owner returns it to the context's pool, as the
  // reference's zero-copy receive frees a frame (van.cc:244-255)
  SArray<char> HostArray(const void* src, size_t bytes) {
    if (bytes == 0) return SArray<char>();
    void* p = nullptr;
    void* h = nullptr;
    Check(psf_host_buffer_alloc(ctx_, bytes, &p, &h));
    SArray<char> out(static_cast<char*>(p), bytes, false);
    out.pointer().reset(static_cast<char*>(p), [h](char*) { psf_host_buffer_release(h); });
    Check(psf_copy_to_host_async(ctx_, p, src, bytes));
    return out;
  }

  psf_context* ctx_ = nullptr;
  psf_node* node_ = nullptr;
  std::map<CacheKey, SArray<char>> keep_;
  std::mutex mu_;
};

// Registration hook for Filter::create (filter.cc:9-23): a libpsf filter, or
// nullptr to fall through to the reference's own switch.
inline Filter* CreateFilter(const FilterConfig& conf) {
  switch (conf.type()) {
    case FilterConfig::KEY_CACHING: return new KeyCachingFilter();
    case FilterConfig::FIXING_FLOAT: return new FixingFloatFilter();
    case FilterConfig::COMPRESSING: return new CompressingFilter();
    case FilterConfig::NOISE: return new AddNoiseFilter();
    default: return nullptr;
  }
}

}  // namespace psf_hip
}  // namespace PS
