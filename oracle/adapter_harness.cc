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

#include <hip/hip_runtime_api.h>

#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
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

// `n` per-filter FIXING_FLOAT adapter instances on one device (a server with
// n worker peers: RemoteNode keeps one instance per type per peer,
// remote_node.cc:7-15), `rounds` passes over them, instance i's message
// length cycling through distinct sizes in [min_values, max_values].  After
// every message the device-wide allocator stats are read; out[0] = the peak
// of the device's cached HBM, out[1] = the device cap, out[2] = the peak of
// the device's live streams, out[3] = shared streams, out[4] = evictions,
// out[5] = the largest allocated HBM seen.  Returns 0, or -1 when a round
// trip's decoded values differ from the first pass's for the same size (the
// decode is deterministic given the seed) or a CHECK failed.
int psadapter_many_instances(int n, int rounds, const float* x, size_t min_values, size_t max_values,
                             uint64_t* out) {
  psf_set_clock(1, 4242);
  std::vector<std::unique_ptr<psf_hip::FixingFloatFilter>> fs;
  for (int i = 0; i < n; ++i) fs.emplace_back(new psf_hip::FixingFloatFilter());
  const size_t span = max_values - min_values + 1;
  std::vector<uint8_t> codes(max_values);
  std::vector<float> dec(max_values);
  float range[2];
  for (int k = 0; k < 6; ++k) out[k] = 0;
  for (int r = 0; r < rounds; ++r)
    for (int i = 0; i < n; ++i) {
      const size_t m = min_values + ((size_t)(i + 1) * 7919u + (size_t)r * 104729u) % span;
      if (ff_roundtrip(*fs[i], x, m * 4, 9, 1, 0, 0.f, 0, 0.f, codes.data(), range, dec.data()) != 0) return -1;
      for (size_t j = 0; j < m; j += 997)  // decoded values lie in the range
        if (!(dec[j] >= range[0] && dec[j] <= range[1])) {
          g_err = "decoded value outside [min, max]";
          return -1;
        }
      uint64_t st[10];
      if (psf_device_memory_stats(psf_default_device(), st) != PSF_OK) return -1;
      out[0] = std::max(out[0], st[0]);
      out[1] = st[1];
      out[2] = std::max(out[2], st[8]);
      out[3] = st[9];
      out[4] = st[3];
      out[5] = std::max(out[5], st[2]);
    }
  return 0;
}

// a FIXING_FLOAT instance created (its context lazily made on first use) on
// one thread and used from another: the reference's Submit encodes on the
// app thread and PickActiveMsg decodes on the executor thread
// (executor.cc:143, 219); the second thread's current device is set to
// `other_device` first, so a libpsf entry that did not make its context's
// device current would allocate on the wrong GPU.
int psadapter_ff_cross_thread(const void* x, size_t bytes, int nb, int64_t seed, int other_device, void* codes,
                              float* range, void* dec) {
  psf_set_clock(1, seed);
  std::unique_ptr<psf_hip::FixingFloatFilter> f(new psf_hip::FixingFloatFilter());
  int rc = 0;
  std::thread t([&] {
    if (hipSetDevice(other_device) != hipSuccess) {
      rc = -3;
      return;
    }
    rc = ff_roundtrip(*f, x, bytes, 9, nb, 0, 0.f, 0, 0.f, codes, range, dec);
    int cur = -1;
    if (rc == 0 && (hipGetDevice(&cur) != hipSuccess || cur != other_device)) rc = -4;  // restored
  });
  t.join();
  return rc;
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

// ---- the per-RemoteNode chain (psf_hip::Chain) and, for comparison, the
// reference's own RemoteNode loop (remote_node.cc:7-29) over per-filter
// adapter instances from the Filter::create hook
struct RefNode {  // RemoteNode::FindFilterOrCreate / EncodeMessage / DecodeMessage
  std::map<int, Filter*> filters;
  ~RefNode() {
    for (auto& f : filters) delete f.second;
  }
  Filter* find_or_create(const FilterConfig& c) {
    auto it = filters.find((int)c.type());
    if (it == filters.end()) it = filters.emplace((int)c.type(), psf_hip::CreateFilter(c)).first;
    return it->second;
  }
  void encode(Message* m) {
    for (int i = 0; i < m->task.filter_size(); ++i) find_or_create(m->task.filter(i))->encode(m);
  }
  void decode(Message* m) {
    for (int i = m->task.filter_size() - 1; i >= 0; --i) find_or_create(m->task.filter(i))->decode(m);
  }
};
struct Peer {  // one side's RemoteNode: the patched one (Chain) or the reference loop
  bool chain;
  psf_hip::Chain c;
  RefNode r;
  void encode(Message* m) {
    if (!(chain && c.Encode(m))) r.encode(m);
  }
  void decode(Message* m) {
    if (!(chain && c.Decode(m))) r.decode(m);
  }
};

// flags: 1 request, 2 has_param + push; filters: type per entry, param = nb
// (FIXING_FLOAT) or clear_cache_if_done (KEY_CACHING)
Message* chain_msg(int flags, int ch, uint64_t rb, uint64_t re, const void* key, size_t kbytes, const void* val,
                   size_t vbytes, int vt, int nf, const int* ftype, const int* fparam) {
  auto* m = new Message();
  m->task.request_ = flags & 1;
  m->task.has_param_ = (flags & 2) != 0;
  m->task.param_.push_ = (flags & 2) != 0;
  m->task.key_channel_ = ch;
  m->task.mutable_key_range()->set_begin(rb);
  m->task.mutable_key_range()->set_end(re);
  if (kbytes) {
    SArray<char> k(kbytes);
    memcpy(k.data(), key, kbytes);
    m->set_key(k);
  }
  if (val) {
    SArray<char> v(vbytes);
    if (vbytes) memcpy(v.data(), val, vbytes);
    m->task.value_type_.push_back((DataType)vt);
    m->value.push_back(v);
  }
  for (int i = 0; i < nf; ++i) {
    auto* f = m->task.add_filter();
    f->set_type((FilterConfig::Type)ftype[i]);
    if (ftype[i] == FilterConfig::FIXING_FLOAT) f->num_bytes_ = fparam[i];
    if (ftype[i] == FilterConfig::KEY_CACHING) f->clear_cache_if_done_ = fparam[i] != 0;
  }
  return m;
}
}  // extern "C"

extern "C" {
void* psadapter_peer_new(int chain) {
  auto* p = new Peer();
  p->chain = chain != 0;
  return p;
}
void psadapter_peer_free(void* p) { delete static_cast<Peer*>(p); }

// One message: encode on snd, the receiver decodes a copy (Task by value,
// SArrays shared).  Out: the wire key / value (wk, *wkl; wv, *wvl), per filter
// 8 words of side-info {has_sig, sig, has_fp, min bits, max bits, n_unc,
// unc0, unc1}, the decoded key / value (dk, *dkl; dv, *dvl).  0 ok, 1 encode
// CHECK, 2 decode CHECK.
int psadapter_chain_msg(void* snd, void* rcv, int flags, int ch, uint64_t rb, uint64_t re, const void* key,
                        size_t kbytes, const void* val, size_t vbytes, int vt, int nf, const int* ftype,
                        const int* fparam, uint8_t* wk, size_t* wkl, uint8_t* wv, size_t* wvl, int64_t* side,
                        uint8_t* dk, size_t* dkl, uint8_t* dv, size_t* dvl) {
  std::unique_ptr<Message> m(chain_msg(flags, ch, rb, re, key, kbytes, val, vbytes, vt, nf, ftype, fparam));
  try {
    static_cast<Peer*>(snd)->encode(m.get());
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
  *wkl = m->key.size();
  if (*wkl) memcpy(wk, m->key.data(), *wkl);
  *wvl = m->value.empty() ? 0 : m->value[0].size();
  if (*wvl) memcpy(wv, m->value[0].data(), *wvl);
  for (int i = 0; i < nf; ++i) {
    const FilterConfig& c = m->task.filter(i);
    int64_t* o = side + 8 * i;
    o[0] = c.has_signature();
    o[1] = c.signature();
    o[2] = c.fixed_point_size() > 0;
    float mn = 0.f, mx = 0.f;
    if (o[2]) {
      mn = c.fixed_point(0).min_value();
      mx = c.fixed_point(0).max_value();
    }
    uint32_t a, b;
    memcpy(&a, &mn, 4);
    memcpy(&b, &mx, 4);
    o[3] = a;
    o[4] = b;
    o[5] = c.uncompressed_size_size();
    o[6] = o[5] > 0 ? (int64_t)c.uncompressed_size(0) : 0;
    o[7] = o[5] > 1 ? (int64_t)c.uncompressed_size(1) : 0;
  }
  Message w = *m;
  try {
    static_cast<Peer*>(rcv)->decode(&w);
  } catch (const std::exception& e) {
    g_err = e.what();
    return 2;
  }
  *dkl = w.key.size();
  if (*dkl) memcpy(dk, w.key.data(), *dkl);
  *dvl = w.value.empty() ? 0 : w.value[0].size();
  if (*dvl) memcpy(dv, w.value[0].data(), *dvl);
  return 0;
}

// The host edge: `iters` rounds of `nmsg` messages (message j: key bytes
// key[koff[j], koff[j+1]), value bytes val[voff[j], voff[j+1]) -- none when
// empty --, flags fl[j]) encoded on snd and decoded (a copy) on rcv (the
// other way round when dir[j]), messages already built in host
// memory.  Returns seconds per round (negative: a CHECK); *enc_s / *dec_s =
// the encode / decode share.
double psadapter_chain_bench(void* snd, void* rcv, int iters, int nmsg, const uint8_t* key, const uint64_t* koff,
                             const uint8_t* val, const uint64_t* voff, const int* fl, const int* dir, int ch, int vt,
                             int nf, const int* ftype, const int* fparam, double* enc_s, double* dec_s) {
  std::vector<std::unique_ptr<Message>> tm;
  for (int j = 0; j < nmsg; ++j)
    tm.emplace_back(chain_msg(fl[j], ch, 0, ~0ull, key + koff[j], koff[j + 1] - koff[j],
                              voff[j + 1] > voff[j] ? val + voff[j] : nullptr, voff[j + 1] - voff[j], vt, nf, ftype,
                              fparam));
  double te = 0, td = 0;
  // PSAD_FRESH=1: every round's messages in freshly allocated arrays (built
  // outside the timed region), as an application that allocates a new
  // gradient array per minibatch produces them; else the same arrays each round
  const char* fe = getenv("PSAD_FRESH");
  const bool fresh = fe && *fe == '1';
  try {
    for (int it = 0; it < iters; ++it)
      for (int j = 0; j < nmsg; ++j) {
        if (fresh && it)
          tm[j].reset(chain_msg(fl[j], ch, 0, ~0ull, key + koff[j], koff[j + 1] - koff[j],
                                voff[j + 1] > voff[j] ? val + voff[j] : nullptr, voff[j + 1] - voff[j], vt, nf,
                                ftype, fparam));
        Message a = *tm[j];  // the application's message (buffers shared, as KVVector::Push passes them)
        Peer* s = static_cast<Peer*>(dir[j] ? rcv : snd);
        Peer* r = static_cast<Peer*>(dir[j] ? snd : rcv);
        auto t0 = std::chrono::steady_clock::now();
        s->encode(&a);
        auto t1 = std::chrono::steady_clock::now();
        Message w = a;
        r->decode(&w);
        auto t2 = std::chrono::steady_clock::now();
        te += std::chrono::duration<double>(t1 - t0).count();
        td += std::chrono::duration<double>(t2 - t1).count();
      }
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1.0;
  }
  *enc_s = te / iters;
  *dec_s = td / iters;
  return (te + td) / iters;
}

// The same rounds with the sender's encodes and the receiver's decodes on two
// threads, as the reference runs them (EncodeMessage on the application
// thread under Executor::Submit, DecodeMessage on the receiving executor's
// thread, executor.cc:143,219): message k+1 is encoded while message k is
// decoded, so H2D-heavy and D2H-heavy copies share the link in both
// directions.  One direction only (every dir[j] == 0): a queue of at most
// two encoded messages between the threads.  Returns seconds per round.
double psadapter_chain_bench_pipelined(void* snd, void* rcv, int iters, int nmsg, const uint8_t* key,
                                       const uint64_t* koff, const uint8_t* val, const uint64_t* voff, const int* fl,
                                       int ch, int vt, int nf, const int* ftype, const int* fparam) {
  std::vector<std::unique_ptr<Message>> tm;
  for (int j = 0; j < nmsg; ++j)
    tm.emplace_back(chain_msg(fl[j], ch, 0, ~0ull, key + koff[j], koff[j + 1] - koff[j],
                              voff[j + 1] > voff[j] ? val + voff[j] : nullptr, voff[j + 1] - voff[j], vt, nf, ftype,
                              fparam));
  std::deque<Message> q;
  std::mutex mu;
  std::condition_variable cv;
  bool failed = false;
  const int total = iters * nmsg;
  auto t0 = std::chrono::steady_clock::now();
  std::thread enc([&] {
    try {
      for (int k = 0; k < total; ++k) {
        Message a = *tm[k % nmsg];
        static_cast<Peer*>(snd)->encode(&a);
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return q.size() < 2 || failed; });
        if (failed) return;
        q.push_back(a);
        cv.notify_all();
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> l(mu);
      g_err = e.what();
      failed = true;
      cv.notify_all();
    }
  });
  try {
    for (int k = 0; k < total; ++k) {
      Message w;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return !q.empty() || failed; });
        if (failed) break;
        w = q.front();
        q.pop_front();
        cv.notify_all();
      }
      static_cast<Peer*>(rcv)->decode(&w);
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> l(mu);
    g_err = e.what();
    failed = true;
    cv.notify_all();
  }
  enc.join();
  if (failed) return -1.0;
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
}
}  // extern "C"
