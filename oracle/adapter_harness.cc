// ORACLE TEST INFRASTRUCTURE -- exercises include/psf_ps_filter.h, the
// reference-side drop-in, compiled against oracle/ps_mock (a test double of
// the PS types it calls; no reference source is compiled here).  Each entry
// point runs one PS::Message through an adapter filter and hands back what
// the reference's message would hold afterwards (wire bytes, FilterConfig
// side-info, decoded arrays); tests/test_gpu_adapter.py compares them with
// the C restatement (oracle/psf_port.c, snappy_port.c).
// Built by `make -C oracle adapter` into oracle/_port/libpsadapter.so.
#include "filter/filter.h"
#include "psf_ps_filter.h"

#include <chrono>
#include <string>
#include <thread>
#include <vector>

using namespace PS;

namespace PS {
FilterConfig* Filter::find(FilterConfig::Type type, Task* task) {  // filter.cc:26-31
  for (int i = 0; i < task->filter_size(); ++i)
    if (task->filter(i).type() == type) return task->mutable_filter(i);
  return nullptr;
}
}  // namespace PS

namespace {
thread_local std::string g_err;

Message* ff_msg(const void* x, size_t bytes, int vt, int nb, int has_min, float mn, int has_max, float mx) {
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

// encode + decode of one FIXING_FLOAT array through the adapter; 0 ok,
// -1 encode CHECK, -2 decode CHECK
int ff_roundtrip(psf_hip::FixingFloatFilter& f, const void* x, size_t bytes, int vt, int nb, int has_min, float mn,
                 int has_max, float mx, void* codes, float* range, void* dec) {
  Message* a = ff_msg(x, bytes, vt, nb, has_min, mn, has_max, mx);
  int rc = 0;
  try {
    f.encode(a);
  } catch (const std::exception& e) {
    g_err = e.what();
    rc = -1;
  }
  if (rc == 0) {
    memcpy(codes, a->value[0].data(), a->value[0].size());
    const auto& fp = a->task.filter(0).fixed_point(0);
    range[0] = fp.min_value();
    range[1] = fp.max_value();
    Message w = *a;  // what the receiver's executor decodes
    try {
      f.decode(&w);
      memcpy(dec, w.value[0].data(), w.value[0].size());
    } catch (const std::exception& e) {
      g_err = e.what();
      rc = -2;
    }
  }
  delete a;
  return rc;
}
}  // namespace

extern "C" {

const char* psadapter_last_error() { return g_err.c_str(); }

int psadapter_ff(const void* x, size_t bytes, int vt, int nb, int64_t seed, int has_min, float mn, int has_max,
                 float mx, void* codes, float* range, void* dec) {
  psf_set_clock(1, seed);
  psf_hip::FixingFloatFilter f;
  return ff_roundtrip(f, x, bytes, vt, nb, has_min, mn, has_max, mx, codes, range, dec);
}

// `nthreads` adapter instances (one per executor thread, as RemoteNode creates
// one per peer) each encoding + decoding the same array `reps` times
// concurrently; outputs of thread t land at codes + t * n * nb etc.  Returns
// the wall time in seconds (negative: a CHECK failed).
double psadapter_ff_threads(int nthreads, int reps, const void* x, size_t bytes, int vt, int nb, int64_t seed,
                            void* codes, float* range, void* dec) {
  psf_set_clock(1, seed);
  const size_t vsz = vt == 9 ? 4 : 8, n = bytes / vsz;
  std::vector<int> rc(nthreads, 0);
  std::vector<std::thread> th;
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      psf_hip::FixingFloatFilter f;
      for (int r = 0; r < reps && rc[t] == 0; ++r)
        rc[t] = ff_roundtrip(f, x, bytes, vt, nb, 0, 0.f, 0, 0.f, static_cast<uint8_t*>(codes) + t * n * nb,
                             range + 2 * t, static_cast<uint8_t*>(dec) + t * bytes);
    });
  for (auto& t : th) t.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (int r : rc)
    if (r) return -1.0;
  return s;
}

// COMPRESSING: one message with keys (if kbytes) and one value array.
// Wire bytes -> key_out / val_out (lengths *klen / *vlen), uncompressed_size
// side-info -> sizes (*nsizes), decoded key / value -> key_dec / val_dec.
int psadapter_compress(const void* key, size_t kbytes, const void* val, size_t vbytes, int vt, void* key_out,
                       size_t* klen, void* val_out, size_t* vlen, uint64_t* sizes, int* nsizes, void* key_dec,
                       void* val_dec) {
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
  psf_hip::CompressingFilter f;
  int rc = 0;
  try {
    f.encode(m);
    *klen = m->key.size();
    *vlen = m->value[0].size();
    if (*klen) memcpy(key_out, m->key.data(), *klen);
    if (*vlen) memcpy(val_out, m->value[0].data(), *vlen);
    const auto& fc = m->task.filter(0);
    *nsizes = fc.uncompressed_size_size();
    for (int i = 0; i < *nsizes && i < 2; ++i) sizes[i] = fc.uncompressed_size(i);
    Message w = *m;
    f.decode(&w);
    if (w.key.size()) memcpy(key_dec, w.key.data(), w.key.size());
    if (w.value[0].size()) memcpy(val_dec, w.value[0].data(), w.value[0].size());
    if (w.key.size() != kbytes || w.value[0].size() != vbytes) rc = 4;
  } catch (const std::exception& e) {
    g_err = e.what();
    rc = 5;
  }
  delete m;
  return rc;
}

// KEY_CACHING over a sequence of n messages between one sender and one
// receiver instance.  Message i: key bytes kbuf[koff[i], koff[i+1]) (none when
// empty), key_channel ch[i], key_range [rb[i], re[i]); flags fl[i]: 1 request,
// 2 has_param + push, 4 clear_cache_if_done, 8 the receiver restarts (a fresh
// instance) before it.  The receiver decodes a copy of what the sender's
// encode left (Task by value, SArrays shared).  Per message: sent[i] = key
// bytes left on the wire, has_sig/sig = the FilterConfig side-info, got[i] =
// 1 when the decoded key equals the input's, rc[i] = 0, 1 (encode CHECK) or
// 2 (decode CHECK; the sequence stops there).
void psadapter_kc(int n, const uint8_t* kbuf, const uint64_t* koff, const int* ch, const uint64_t* rb,
                  const uint64_t* re, const int* fl, uint64_t* sent, int* has_sig, uint32_t* sig, int* got,
                  int* rc) {
  psf_hip::KeyCachingFilter snd;
  std::unique_ptr<psf_hip::KeyCachingFilter> rcv(new psf_hip::KeyCachingFilter());
  for (int i = 0; i < n; ++i) rc[i] = -1;
  for (int i = 0; i < n; ++i) {
    if (fl[i] & 8) rcv.reset(new psf_hip::KeyCachingFilter());
    Message a;
    a.task.request_ = fl[i] & 1;
    a.task.has_param_ = (fl[i] & 2) != 0;
    a.task.param_.push_ = (fl[i] & 2) != 0;
    a.task.key_channel_ = ch[i];
    a.task.mutable_key_range()->set_begin(rb[i]);
    a.task.mutable_key_range()->set_end(re[i]);
    const size_t kb = koff[i + 1] - koff[i];
    if (kb) {
      SArray<char> k(kb);
      memcpy(k.data(), kbuf + koff[i], kb);
      a.set_key(k);
    }
    auto* f = a.task.add_filter();
    f->set_type(FilterConfig::KEY_CACHING);
    f->clear_cache_if_done_ = (fl[i] & 4) != 0;
    try {
      snd.encode(&a);
    } catch (const std::exception& e) {
      g_err = e.what();
      rc[i] = 1;
      return;
    }
    sent[i] = a.key.size();
    has_sig[i] = a.task.filter(0).has_signature();
    sig[i] = a.task.filter(0).signature();
    Message w = a;
    try {
      rcv->decode(&w);
    } catch (const std::exception& e) {
      g_err = e.what();
      rc[i] = 2;
      return;
    }
    got[i] = w.key.size() == kb && (kb == 0 || memcmp(w.key.data(), kbuf + koff[i], kb) == 0);
    rc[i] = 0;
  }
}

// NOISE on one value array, in place; `alias` receives the array's bytes as
// seen through a second SArray sharing the buffer (the sender's own copy).
int psadapter_noise(const void* val, size_t vbytes, int vt, float mean, float sd, void* out, void* alias) {
  auto* m = new Message();
  SArray<char> v(vbytes);
  memcpy(v.data(), val, vbytes);
  SArray<char> keep = v;  // another reference to the same buffer
  m->task.value_type_.push_back((DataType)vt);
  m->value.push_back(v);
  auto* f = m->task.add_filter();
  f->set_type(FilterConfig::NOISE);
  f->mean_ = mean;
  f->std_ = sd;
  psf_hip::AddNoiseFilter a;
  int rc = 0;
  try {
    a.encode(m);
    memcpy(out, m->value[0].data(), vbytes);
    memcpy(alias, keep.data(), vbytes);
  } catch (const std::exception& e) {
    g_err = e.what();
    rc = 5;
  }
  delete m;
  return rc;
}

}  // extern "C"
