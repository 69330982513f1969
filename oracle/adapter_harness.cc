// ORACLE TEST INFRASTRUCTURE -- drop-in check for include/psf_ps_filter.h.
//
// Compiles the adapter against the PS types of oracle/ref_stub (the same
// accessor names as the reference's generated protobuf classes) next to the
// reference's UNMODIFIED src/filter/fixing_float.h, and runs both on the same
// PS::Message: the reference filter and the libpsf-backed filter must produce
// identical codes, identical FilterConfig side-info and identical decoded
// values, and each must decode the other's wire output identically.
// Built by `make -C oracle adapter` into oracle/_ref/libpsadapter.so.
#include "filter/filter.h"
#include "filter/fixing_float.h"
#include "filter/compressing.h"
#include "filter/add_noise.h"
#include "psf_ps_filter.h"
#include "snappy_glue.h"

#include <string>
#include <vector>

using namespace PS;

static time_t g_time = 0;
extern "C" time_t __wrap_time(time_t* t) {
  if (t) *t = g_time;
  return g_time;
}

namespace PS {
FilterConfig* Filter::find(FilterConfig::Type type, Task* task) {  // filter.cc:26-31
  for (int i = 0; i < task->filter_size(); ++i)
    if (task->filter(i).type() == type) return task->mutable_filter(i);
  return nullptr;
}
}  // namespace PS

namespace {
thread_local std::string g_err;

Message* make_msg(const void* x, size_t bytes, int vt, int nb, int has_min, float mn, int has_max,
                  float mx) {
  auto* m = new Message();
  SArray<char> v(bytes);
  memcpy(v.data(), x, bytes);
  m->task.value_type_.push_back((DataType)vt);
  m->value.push_back(v);
  auto* f = m->task.add_filter();
  f->set_type(FilterConfig::FIXING_FLOAT);
  f->num_bytes_ = nb;
  if (has_min || has_max) {
    auto* p = f->add_fixed_point();
    if (has_min) p->set_min_value(mn);
    if (has_max) p->set_max_value(mx);
  }
  return m;
}

bool same_bytes(const SArray<char>& a, const SArray<char>& b) {
  return a.size() == b.size() && (a.size() == 0 || memcmp(a.data(), b.data(), a.size()) == 0);
}
bool same_fp(const FilterConfig& a, const FilterConfig& b) {
  if (a.fixed_point_size() != b.fixed_point_size()) return false;
  for (int k = 0; k < a.fixed_point_size(); ++k) {
    const auto &p = a.fixed_point(k), &q = b.fixed_point(k);
    if (p.has_min_value() != q.has_min_value() || p.has_max_value() != q.has_max_value()) return false;
    if (memcmp(&p.min_, &q.min_, 4) || memcmp(&p.max_, &q.max_, 4)) return false;
  }
  return true;
}
}  // namespace

extern "C" {

const char* psadapter_last_error() { return g_err.c_str(); }

// 0 = identical; >0 = which comparison failed; <0 = both rejected identically
int psadapter_compare_ff(const void* x, size_t bytes, int value_type, int nb, int64_t seed,
                         int has_min, float mn, int has_max, float mx) {
  g_time = (time_t)seed;
  psf_set_clock(1, seed);
  Message* a = make_msg(x, bytes, value_type, nb, has_min, mn, has_max, mx);
  Message* b = make_msg(x, bytes, value_type, nb, has_min, mn, has_max, mx);
  PS::FixingFloatFilter ref;
  psf_hip::FixingFloatFilter hip;
  int rc = 0;
  bool ra = true, rb = true;
  try { ref.encode(a); } catch (const std::exception& e) { ra = false; g_err = e.what(); }
  try { hip.encode(b); } catch (const std::exception& e) { rb = false; g_err += std::string(" | ") + e.what(); }
  if (!ra || !rb) {
    rc = (ra == rb) ? -1 : 1;
  } else if (!same_bytes(a->value[0], b->value[0])) {
    rc = 2;
  } else if (!same_fp(a->task.filter(0), b->task.filter(0))) {
    rc = 3;
  } else {
    // cross decode: reference decodes the adapter's wire output and vice versa
    Message a2 = *b, b2 = *a;
    try {
      ref.decode(&a2);
      hip.decode(&b2);
      if (!same_bytes(a2.value[0], b2.value[0])) rc = 4;
    } catch (const std::exception& e) {
      g_err = e.what();
      rc = 5;
    }
  }
  delete a;
  delete b;
  return rc;
}

// COMPRESSING: reference CompressingFilter vs the adapter on one message with
// keys (if kbytes) and one value array.  0 = identical wire bytes, identical
// uncompressed_size and both cross decodes restore the input.
int psadapter_compare_compress(const void* key, size_t kbytes, const void* val, size_t vbytes, int vt) {
  auto mk = [&] {
    auto* m = new Message();
    if (kbytes) {
      SArray<char> k(kbytes);
      memcpy(k.data(), key, kbytes);
      m->set_key(k);
    }
    SArray<char> v(vbytes);
    if (vbytes) memcpy(v.data(), val, vbytes);
    m->task.value_type_.push_back((DataType)vt);
    m->value.push_back(v);
    m->task.add_filter()->set_type(FilterConfig::COMPRESSING);
    return m;
  };
  Message *a = mk(), *b = mk(), *orig = mk();
  PS::CompressingFilter ref;
  psf_hip::MessageFilter hip(FilterConfig::COMPRESSING);
  int rc = 0;
  try {
    ref.encode(a);
    hip.encode(b);
    const auto &fa = a->task.filter(0), &fb = b->task.filter(0);
    if (!same_bytes(a->key, b->key) || !same_bytes(a->value[0], b->value[0])) rc = 2;
    else if (fa.uncompressed_size_size() != fb.uncompressed_size_size()) rc = 3;
    for (int i = 0; rc == 0 && i < fa.uncompressed_size_size(); ++i)
      if (fa.uncompressed_size(i) != fb.uncompressed_size(i)) rc = 3;
    if (rc == 0) {
      Message a2 = *b, b2 = *a;
      ref.decode(&a2);
      hip.decode(&b2);
      if (!same_bytes(a2.key, orig->key) || !same_bytes(b2.key, orig->key) ||
          !same_bytes(a2.value[0], orig->value[0]) || !same_bytes(b2.value[0], orig->value[0]))
        rc = 4;
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    rc = 5;
  }
  delete a;
  delete b;
  delete orig;
  return rc;
}

// NOISE: reference AddNoiseFilter vs the adapter (in place); 0 = identical bytes
int psadapter_compare_noise(const void* val, size_t vbytes, int vt, float mean, float sd) {
  auto mk = [&] {
    auto* m = new Message();
    SArray<char> v(vbytes);
    memcpy(v.data(), val, vbytes);
    m->task.value_type_.push_back((DataType)vt);
    m->value.push_back(v);
    auto* f = m->task.add_filter();
    f->set_type(FilterConfig::NOISE);
    f->mean_ = mean;
    f->std_ = sd;
    return m;
  };
  Message *a = mk(), *b = mk();
  PS::AddNoiseFilter ref;
  psf_hip::MessageFilter hip(FilterConfig::NOISE);
  int rc = 0;
  try {
    ref.encode(a);
    hip.encode(b);
    if (!same_bytes(a->value[0], b->value[0])) rc = 2;
  } catch (const std::exception& e) {
    g_err = e.what();
    rc = 5;
  }
  delete a;
  delete b;
  return rc;
}

}  // extern "C"
