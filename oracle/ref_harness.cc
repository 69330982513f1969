// ORACLE TEST INFRASTRUCTURE -- not product code; never linked into libpsf.
//
// ctypes-callable harness around the reference's UNMODIFIED codec headers
// (/root/reference/src/filter/{fixing_float,key_caching,compressing,add_noise}.h
// + filter.cc + util/crc32c.cc), compiled against oracle/ref_stub.  Built by
// oracle/Makefile into oracle/_ref/libpsref.so (git-ignored).
//
// The chain driver below restates RemoteNode::EncodeMessage / DecodeMessage /
// FindFilterOrCreate (remote_node.cc:7-29): encode in task.filter order, decode
// in reverse, one filter instance per filter type per peer.
//
// FIXING_FLOAT seeds its LCG with time(NULL) (fixing_float.h:78); the library is
// linked with -Wl,--wrap=time so psref_set_time() pins it.
#include "filter/filter.h"
#include "filter/fixing_float.h"
#include "filter/key_caching.h"
#include "filter/compressing.h"
#include "filter/add_noise.h"
#include "util/crc32c.h"

#include <map>
#include <string>

using namespace PS;

static time_t g_time = 0;
extern "C" time_t __wrap_time(time_t* t) {
  if (t) *t = g_time;
  return g_time;
}

#include "snappy_glue.h"

namespace {
thread_local std::string g_err;

struct RefNode {
  std::map<int, Filter*> filters;
  ~RefNode() { for (auto& f : filters) delete f.second; }
  Filter* find_or_create(const FilterConfig& c) {
    auto it = filters.find(c.type());
    if (it == filters.end()) it = filters.emplace(c.type(), Filter::create(c)).first;
    return it->second;
  }
};

template <typename F> int guarded(F&& f) {
  try { f(); return 0; }
  catch (const std::exception& e) { g_err = e.what(); return -1; }
}
}  // namespace

extern "C" {

const char* psref_last_error() { return g_err.c_str(); }
void psref_set_time(int64_t t) { g_time = (time_t)t; }

uint32_t psref_crc32c(const void* p, size_t n) {
  return crc32c::Value(reinterpret_cast<const char*>(p), n);
}

void* psref_node_new() { return new RefNode(); }
void psref_node_free(void* n) { delete static_cast<RefNode*>(n); }

void* psref_msg_new(int request, int has_param, int push, int key_channel,
                    int has_key_range, uint64_t kr_begin, uint64_t kr_end) {
  auto* m = new Message();
  m->task.request_ = request != 0;
  m->task.has_param_ = has_param != 0;
  m->task.param_.push_ = push != 0;
  m->task.key_channel_ = key_channel;
  if (has_key_range) {
    m->task.mutable_key_range()->set_begin(kr_begin);
    m->task.mutable_key_range()->set_end(kr_end);
  }
  return m;
}
void psref_msg_free(void* m) { delete static_cast<Message*>(m); }

// Simulates the wire: the receiver gets a copy of the Task (with all filter
// side-info) and the same buffers (zero-copy, as ZeroMQ frames, van.cc:244-255).
void* psref_msg_clone(void* src) {
  auto* s = static_cast<Message*>(src);
  auto* m = new Message();
  m->task = s->task;
  m->key = s->key;
  m->value = s->value;
  return m;
}

void psref_msg_set_key(void* mp, const void* data, size_t bytes, int key_type) {
  auto* m = static_cast<Message*>(mp);
  SArray<char> k(bytes);
  if (bytes) memcpy(k.data(), data, bytes);
  m->key = k;
  m->task.set_has_key(bytes > 0);
  m->task.set_key_type((DataType)key_type);
  if (!m->task.has_key_range()) Range<Key>::All().To(m->task.mutable_key_range());
}
void psref_msg_add_value(void* mp, const void* data, size_t bytes, int value_type) {
  auto* m = static_cast<Message*>(mp);
  SArray<char> v(bytes);
  if (bytes) memcpy(v.data(), data, bytes);
  m->task.value_type_.push_back((DataType)value_type);
  m->value.push_back(v);
}
size_t psref_msg_key_bytes(void* mp) { return static_cast<Message*>(mp)->key.size(); }
int psref_msg_has_key_flag(void* mp) { return static_cast<Message*>(mp)->task.has_key_ ? 1 : 0; }
int psref_msg_key_type(void* mp) { return static_cast<Message*>(mp)->task.key_type_; }
void psref_msg_copy_key(void* mp, void* dst) {
  auto* m = static_cast<Message*>(mp);
  if (m->key.size()) memcpy(dst, m->key.data(), m->key.size());
}
int psref_msg_num_values(void* mp) { return (int)static_cast<Message*>(mp)->value.size(); }
size_t psref_msg_value_bytes(void* mp, int i) { return static_cast<Message*>(mp)->value.at(i).size(); }
void psref_msg_copy_value(void* mp, int i, void* dst) {
  auto& v = static_cast<Message*>(mp)->value.at(i);
  if (v.size()) memcpy(dst, v.data(), v.size());
}

int psref_msg_add_filter(void* mp, int type) {
  auto* m = static_cast<Message*>(mp);
  m->task.add_filter()->set_type((FilterConfig::Type)type);
  return m->task.filter_size() - 1;
}
static FilterConfig* fc(void* mp, int idx) {
  return static_cast<Message*>(mp)->task.mutable_filter(idx);
}
void psref_fc_set_num_bytes(void* mp, int idx, int nb) { fc(mp, idx)->num_bytes_ = nb; }
void psref_fc_set_clear_cache(void* mp, int idx, int v) { fc(mp, idx)->clear_cache_if_done_ = v != 0; }
void psref_fc_set_noise(void* mp, int idx, float mean, float sd) {
  fc(mp, idx)->mean_ = mean; fc(mp, idx)->std_ = sd;
}
void psref_fc_add_fixed_point(void* mp, int idx, int has_min, float mn, int has_max, float mx) {
  auto* f = fc(mp, idx)->add_fixed_point();
  if (has_min) f->set_min_value(mn);
  if (has_max) f->set_max_value(mx);
}
int psref_fc_num_fixed_point(void* mp, int idx) { return fc(mp, idx)->fixed_point_size(); }
void psref_fc_get_fixed_point(void* mp, int idx, int k, int* has_min, float* mn, int* has_max, float* mx) {
  const auto& f = fc(mp, idx)->fixed_point(k);
  *has_min = f.has_min_value(); *mn = f.min_value();
  *has_max = f.has_max_value(); *mx = f.max_value();
}
int psref_fc_get_signature(void* mp, int idx, uint32_t* sig) {
  *sig = fc(mp, idx)->signature();
  return fc(mp, idx)->has_signature() ? 1 : 0;
}
int psref_fc_num_uncompressed(void* mp, int idx) { return fc(mp, idx)->uncompressed_size_size(); }
uint64_t psref_fc_uncompressed(void* mp, int idx, int i) { return fc(mp, idx)->uncompressed_size(i); }

int psref_node_encode(void* np, void* mp) {
  auto* n = static_cast<RefNode*>(np);
  auto* m = static_cast<Message*>(mp);
  return guarded([&] {
    for (int i = 0; i < m->task.filter_size(); ++i) n->find_or_create(m->task.filter(i))->encode(m);
  });
}
int psref_node_decode(void* np, void* mp) {
  auto* n = static_cast<RefNode*>(np);
  auto* m = static_cast<Message*>(mp);
  return guarded([&] {
    for (int i = m->task.filter_size() - 1; i >= 0; --i) n->find_or_create(m->task.filter(i))->decode(m);
  });
}

// Direct snappy (1.1.8) entry points for fixture generation.
size_t psref_snappy_max(size_t n) { return snappy::MaxCompressedLength(n); }
size_t psref_snappy_compress(const void* src, size_t n, void* dst) {
  size_t out = 0;
  snappy::RawCompress(static_cast<const char*>(src), n, static_cast<char*>(dst), &out);
  return out;
}
// -1: GetUncompressedLength fails; -2: length > cap; -3: RawUncompress fails.
int psref_snappy_uncompress(const void* src, size_t n, void* dst, size_t cap, size_t* out_len) {
  size_t d = 0;
  if (!snappy::GetUncompressedLength(static_cast<const char*>(src), n, &d)) return -1;
  *out_len = d;
  if (d > cap) return -2;
  return snappy::RawUncompress(static_cast<const char*>(src), n, static_cast<char*>(dst)) ? 0 : -3;
}

}  // extern "C"
