// extern "C" boundary of libpsf (include/psf.h).
#include "../../../include/psf.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <set>
#include <string>

#include "exchange.h"
#include "filter.h"
#include "kvstore.h"
#include "router.h"
#include "slice.h"
#include "snappy_host.h"
#include "spill.h"
#include "wire.h"

struct psf_context { psf::Context* impl; };
struct psf_node { psf::RemoteNode* impl; };
struct psf_message { psf::Message m; };
struct psf_kvmap { psf::KvMapFtrl* impl; psf::Context* ctx; };

namespace {
thread_local std::string g_last_error;

template <typename F> int guarded(F&& f) {
  try {
    return f();
  } catch (const psf::CheckError& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return PSF_ERR_CHECK;
  }
}

// the same, with the context's device current on the calling thread for the
// call (hipMalloc, hipEventCreate and the per-device kernel tables follow the
// thread's current device, not the stream's): a context on device k may be
// used from any thread -- the reference encodes on the app thread and decodes
// on the executor thread (executor.cc:143, 219)
template <typename F> int guarded(psf::Context* c, F&& f) {
  return guarded([&] {
    psf::DeviceScope ds(c ? c->device() : -1);
    return f();
  });
}

psf::FilterConfig* fc_at(psf_message* msg, int idx) {
  if (!msg || idx < 0 || idx >= (int)msg->m.task.filter.size())
    throw psf::CheckError(PSF_ERR_ARG, "filter index out of range");
  return &msg->m.task.filter[idx];
}
const psf::FilterConfig* fc_at(const psf_message* msg, int idx) {
  return fc_at(const_cast<psf_message*>(msg), idx);
}
psf::Buffer wrap(void* ptr, size_t bytes, int loc) {
  psf::Buffer b;
  b.ptr = static_cast<uint8_t*>(ptr);
  b.bytes = ptr ? bytes : 0;
  b.loc = loc == PSF_LOC_HOST ? psf::Loc::kHost : psf::Loc::kDevice;
  return b;
}
}  // namespace

extern "C" {

const char* psf_last_error(void) { return g_last_error.c_str(); }
const char* psf_version(void) { return "psf 0.1 gfx950"; }
void psf_set_clock(int enable, int64_t t) { psf::set_clock_override(enable != 0, t); }

static std::atomic<int> g_default_device{-1};
int psf_set_default_device(int device) {
  if (device < 0) {
    g_last_error = "psf_set_default_device: negative device";
    return PSF_ERR_ARG;
  }
  g_default_device.store(device);
  return PSF_OK;
}
int psf_default_device(void) {
  int d = g_default_device.load();
  if (d >= 0) return d;
  const char* e = getenv("PSF_DEVICE");
  d = 0;
  if (e && *e) {
    char* end = nullptr;
    const long v = strtol(e, &end, 10);
    if (end && *end == 0 && v >= 0 && v < 1024) {
      d = (int)v;
    } else {  // a typo would send every server process to GPU 0 silently: say so
      g_last_error = std::string("PSF_DEVICE='") + e + "' is not a device index; using device 0";
      fprintf(stderr, "libpsf: warning: %s\n", g_last_error.c_str());
    }
  }
  int expect = -1;
  g_default_device.compare_exchange_strong(expect, d);
  return g_default_device.load();
}

int psf_context_create(int device, void* stream, int own_stream, psf_context** out) {
  return guarded([&] {
    if (!out || own_stream < 0 || own_stream > PSF_STREAM_SHARED) return PSF_ERR_ARG;
    if (own_stream == PSF_STREAM_SHARED && stream) return PSF_ERR_ARG;
    *out = new psf_context{new psf::Context(device, static_cast<hipStream_t>(stream), own_stream)};
    return PSF_OK;
  });
}
int psf_context_destroy(psf_context* ctx) {
  if (!ctx) return PSF_OK;
  psf::Context::unref(ctx->impl);  // deleted now, or when its last node / router / exchange / map goes
  delete ctx;
  return PSF_OK;
}
int psf_context_sync(psf_context* ctx) {
  return guarded(ctx ? ctx->impl : nullptr, [&] { ctx->impl->sync_checked(); return PSF_OK; });
}
int psf_copy_to_host(psf_context* ctx, void* dst, const void* src, size_t bytes) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || (bytes && (!dst || !src))) return PSF_ERR_ARG;
    if (bytes == 0) return PSF_OK;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) { memcpy(dst, src, bytes); return PSF_OK; }
    PSF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, c.stream()));
    c.sync();
    return PSF_OK;
  });
}

int psf_copy_to_host_async(psf_context* ctx, void* dst, const void* src, size_t bytes) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || (bytes && (!dst || !src))) return PSF_ERR_ARG;
    if (bytes == 0) return PSF_OK;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) { memcpy(dst, src, bytes); return PSF_OK; }
    PSF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, c.stream()));
    return PSF_OK;
  });
}

// a pinned host buffer from the context's pool; the handle owns it (and keeps
// the pool alive after the context is gone)
int psf_host_buffer_alloc(psf_context* ctx, size_t bytes, void** ptr, void** handle) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !ptr || !handle) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) return PSF_ERR_ARG;
    psf::Context::Pinned p = c.pinned(bytes ? bytes : 1);
    *ptr = p.host;
    *handle = new std::shared_ptr<void>(p.owner);
    return PSF_OK;
  });
}
int psf_host_buffer_release(void* handle) {
  delete static_cast<std::shared_ptr<void>*>(handle);
  return PSF_OK;
}

// ---------------------------------------------------------------- kernels
int psf_ff_encode(psf_context* ctx, const void* d_values, size_t n, int value_type,
                  int num_bytes, psf_fixed_point* fp, int32_t seed, void* d_code) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !fp) return PSF_ERR_ARG;
    if (num_bytes <= 0 || num_bytes >= 8) return PSF_ERR_NBYTES;
    if (value_type != PSF_DT_FLOAT && value_type != PSF_DT_DOUBLE) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    psf::FixedPoint pre{fp->has_min, fp->has_max, fp->min_value, fp->max_value};
    if (pre.has_min && pre.has_max) {
      if (!((double)pre.max_value - (double)pre.min_value > 0)) return PSF_ERR_BIN;
      return psf::ff_encode_launch(d_values, n, value_type, num_bytes, pre, (uint32_t)seed, d_code,
                                   c.partials(), nullptr, nullptr, c.stream(), c.prof());
    }
    if (n == 0) return PSF_ERR_ARG;  // min/max of an empty array
    const uint32_t ticket = c.next_ticket();
    int st = psf::ff_encode_launch(d_values, n, value_type, num_bytes, pre, (uint32_t)seed, d_code,
                                   c.partials(), nullptr, nullptr, c.stream(), c.prof(),
                                   c.pub_dev(0), ticket);
    if (st != PSF_OK) return st;
    c.wait_ticket(0, ticket);
    const psf::Slot& h = *c.pub_host(0);
    if (!fp->has_min) { fp->min_value = h.range[0]; fp->has_min = 1; }
    if (!fp->has_max) { fp->max_value = h.range[1]; fp->has_max = 1; }
    return h.status;
  });
}

int psf_ff_encode_async(psf_context* ctx, const void* d_values, size_t n, int value_type,
                        int num_bytes, const psf_fixed_point* preset, int32_t seed,
                        void* d_code, float* d_range, int32_t* d_status) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx) return PSF_ERR_ARG;
    psf::FixedPoint pre{0, 0, 0.f, 0.f};
    if (preset) pre = psf::FixedPoint{preset->has_min, preset->has_max, preset->min_value, preset->max_value};
    psf::Context& c = *ctx->impl;
    return psf::ff_encode_launch(d_values, n, value_type, num_bytes, pre, (uint32_t)seed, d_code,
                                 c.partials(), d_range, d_status, c.stream(), c.prof());
  });
}

int psf_ff_decode(psf_context* ctx, const void* d_code, size_t n, int value_type,
                  int num_bytes, float min_value, float max_value, void* d_values) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx) return PSF_ERR_ARG;
    if (!((double)max_value - (double)min_value > 0)) return PSF_ERR_BIN;
    return psf::ff_decode_launch(d_code, n, value_type, num_bytes, nullptr, min_value, max_value,
                                 d_values, ctx->impl->stream(), ctx->impl->prof());
  });
}

int psf_ff_decode_async(psf_context* ctx, const void* d_code, size_t n, int value_type,
                        int num_bytes, const float* d_range, void* d_values) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !d_range) return PSF_ERR_ARG;
    return psf::ff_decode_launch(d_code, n, value_type, num_bytes, d_range, 0.f, 0.f, d_values,
                                 ctx->impl->stream(), ctx->impl->prof());
  });
}

int psf_crc32c(psf_context* ctx, const void* d_data, size_t bytes, uint32_t* crc) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !crc) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (bytes == 0) { *crc = 0; return PSF_OK; }  // crc32c("") == 0
    uint32_t* d_out = &c.d_slots()[0].crc;
    int st = psf::crc32c_launch(d_data, bytes, d_out, c.stream(), c.prof());
    if (st != PSF_OK) return st;
    PSF_HIP_CHECK(hipMemcpyAsync(crc, d_out, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream()));
    c.sync();
    return PSF_OK;
  });
}

int psf_key_signature(psf_context* ctx, const void* d_keys, size_t bytes, uint32_t* sig) {
  return psf_crc32c(ctx, d_keys, bytes < 2048 ? bytes : 2048, sig);
}

// ---------------------------------------------------------------- chain
size_t psf_snappy_max_compressed_length(size_t n) { return psf::snappy_max_compressed(n); }

int psf_snappy_compress(psf_context* ctx, const void* d_in, size_t n, void* d_out, size_t* out_len) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !d_out || !out_len || (n && !d_in) || n > 0xffffffffull) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) return PSF_ERR_ARG;
    if (n == 0) {  // RawCompress of nothing: the one-byte header
      PSF_HIP_CHECK(hipMemsetAsync(d_out, 0, 1, c.stream()));
      PSF_HIP_CHECK(hipStreamSynchronize(c.stream()));
      *out_len = 1;
      return PSF_OK;
    }
    psf::Buffer scratch = c.alloc(psf::snappy_compress_scratch(n));
    const uint32_t ticket = c.next_ticket();
    int st = psf::snappy_compress_launch(d_in, n, d_out, scratch.ptr, c.stream(), c.prof(), c.pub_dev(0), ticket);
    if (st != PSF_OK) return st;
    c.wait_ticket(0, ticket);
    if (c.pub_host(0)->status != PSF_OK) {
      c.sync();
      return (int)c.pub_host(0)->status;
    }
    *out_len = c.pub_host(0)->size;
    // the size is published before every fragment has placed its bytes:
    // "synchronous" means the stream in d_out is complete on return
    c.sync();
    return PSF_OK;
  });
}

// A stored-layout stream (psf_internal.h StoredLayout: what FIXING_FLOAT
// writes when COMPRESSING follows) compressed: left where it is when every
// fragment comes out stored, else placed by the compressor and copied back.
static size_t stored_capacity(size_t n) {
  const size_t st = (size_t)psf::stored_alloc_bytes(psf::stored_layout((uint32_t)n));
  const size_t mx = psf::snappy_max_compressed(n);
  return st > mx ? st : mx;
}
int psf_snappy_compress_stored(psf_context* ctx, void* d_buf, size_t n, size_t cap, size_t* out_len) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !d_buf || !out_len || n == 0 || n > 0xffffffffull) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0 || cap < stored_capacity(n)) return PSF_ERR_ARG;
    psf::Buffer src;
    src.ptr = static_cast<uint8_t*>(d_buf);
    src.bytes = n;
    src.loc = psf::Loc::kDevice;
    src.layout = psf::kLayoutStored1;
    psf::Buffer out;
    psf::SnappyBatch b(c);
    b.compress(src, &out);
    b.flush();
    if (out.ptr != src.ptr && out.bytes)
      PSF_HIP_CHECK(hipMemcpyAsync(d_buf, out.ptr, out.bytes, hipMemcpyDeviceToDevice, c.stream()));
    c.sync();
    *out_len = out.bytes;
    return PSF_OK;
  });
}

size_t psf_snappy_stored_capacity(size_t n) { return n && n <= 0xffffffffull ? stored_capacity(n) : 0; }

static psf::Buffer device_view(const void* p, size_t n) {
  psf::Buffer b;
  b.ptr = static_cast<uint8_t*>(const_cast<void*>(p));
  b.bytes = n;
  b.loc = psf::Loc::kDevice;
  return b;
}

int psf_snappy_uncompressed_length(psf_context* ctx, const void* d_in, size_t n, size_t* out_len) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !out_len || (n && !d_in)) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) return PSF_ERR_ARG;
    uint64_t d = 0;
    if (!psf::snappy_read_header(c, device_view(d_in, n), &d)) return PSF_ERR_CHECK;
    *out_len = d;
    return PSF_OK;
  });
}

int psf_snappy_uncompress(psf_context* ctx, const void* d_in, size_t n, void* d_out, size_t out_cap,
                          size_t* out_len) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !out_len || (n && !d_in)) return PSF_ERR_ARG;
    psf::Context& c = *ctx->impl;
    if (c.device() < 0) return PSF_ERR_ARG;
    uint64_t d = 0;
    const uint32_t hdr = psf::snappy_read_header(c, device_view(d_in, n), &d);
    if (!hdr) return PSF_ERR_CHECK;
    *out_len = d;
    if (d > out_cap || (d && !d_out)) return PSF_ERR_ARG;
    psf::Buffer scratch = c.alloc(psf::snappy_uncompress_scratch(n, d));
    const uint32_t ticket = c.next_ticket();
    // the fast path (K-spec) first; the scan / link / index / fragment
    // kernels only if it did not publish the verdict -- a stream of stored
    // fragments needs none of them (as SnappyBatch::finish does for batches)
    const psf::SnappyDJob job{d_in, n, hdr, d, d_out, 0, ticket};
    psf::SnappyTail tail;
    int st = psf::snappy_uncompress_batch_launch(&job, 1, scratch.ptr, c.stream(), c.prof(), c.pub_dev(0),
                                                 psf::ZeroPair{}, &tail);
    if (st != PSF_OK) return st;
    hipEvent_t done = c.take_marker();
    PSF_HIP_CHECK(hipEventRecord(done, c.stream()));
    bool published = false;
    const bool force = psf::snappy_force_tail();
    for (uint64_t spin = 0;; ++spin) {
      if (!force && (published = __atomic_load_n(&c.pub_host(0)->ticket, __ATOMIC_ACQUIRE) == ticket)) break;
      const hipError_t q = hipEventQuery(done);
      if (q == hipSuccess) {
        published = !force && __atomic_load_n(&c.pub_host(0)->ticket, __ATOMIC_ACQUIRE) == ticket;
        break;
      }
      if (q != hipErrorNotReady) {
        c.give_marker(done);
        throw psf::CheckError(PSF_ERR_HIP, std::string("stream failed: ") + hipGetErrorString(q));
      }
      if (spin > 4096) sched_yield();
    }
    c.give_marker(done);
    if (!published) {
      st = psf::snappy_uncompress_tail_launch(&tail, c.stream());
      if (st != PSF_OK) return st;
    }
    c.wait_ticket(0, ticket);
    return c.pub_host(0)->status;
  });
}

int psf_node_create(psf_context* ctx, psf_node** out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !out) return PSF_ERR_ARG;
    *out = new psf_node{new psf::RemoteNode(ctx->impl)};
    psf::Context::ref(ctx->impl);
    return PSF_OK;
  });
}
int psf_node_destroy(psf_node* node) {
  if (!node) return PSF_OK;
  psf::Context* c = node->impl->ctx();
  delete node->impl;
  delete node;
  psf::Context::unref(c);
  return PSF_OK;
}
int psf_node_encode(psf_node* node, psf_message* msg) {
  return guarded(node ? node->impl->ctx() : nullptr, [&] {
    if (!node || !msg) return PSF_ERR_ARG;
    node->impl->EncodeMessage(&msg->m);
    return PSF_OK;
  });
}
int psf_node_decode(psf_node* node, psf_message* msg) {
  return guarded(node ? node->impl->ctx() : nullptr, [&] {
    if (!node || !msg) return PSF_ERR_ARG;
    node->impl->DecodeMessage(&msg->m);
    return PSF_OK;
  });
}

int psf_msg_create(int request, int has_param, int push, int32_t key_channel,
                   int has_key_range, uint64_t kr_begin, uint64_t kr_end, psf_message** out) {
  return guarded([&] {
    if (!out) return PSF_ERR_ARG;
    auto* m = new psf_message();
    m->m.task.request = request != 0;
    m->m.task.has_param = has_param != 0;
    m->m.task.push = push != 0;
    m->m.task.key_channel = key_channel;
    if (has_key_range) {
      m->m.task.has_key_range = true;
      m->m.task.key_range = psf::KeyRange{kr_begin, kr_end};
    }
    *out = m;
    return PSF_OK;
  });
}
int psf_msg_destroy(psf_message* msg) {
  delete msg;
  return PSF_OK;
}
int psf_msg_clone(const psf_message* msg, psf_message** out) {
  return guarded([&] {
    if (!msg || !out) return PSF_ERR_ARG;
    *out = new psf_message(*msg);
    return PSF_OK;
  });
}

int psf_msg_set_key(psf_message* msg, void* ptr, size_t bytes, int key_type, int loc) {
  return guarded([&] {
    if (!msg) return PSF_ERR_ARG;
    auto& t = msg->m.task;
    msg->m.key = wrap(ptr, bytes, loc);
    t.has_key = msg->m.key.bytes > 0;
    t.key_type = key_type;
    t.has_key_type = true;
    if (!t.has_key_range) { t.has_key_range = true; t.key_range = psf::KeyRange::All(); }
    return PSF_OK;
  });
}
int psf_msg_add_value(psf_message* msg, void* ptr, size_t bytes, int value_type, int loc) {
  return guarded([&] {
    if (!msg) return PSF_ERR_ARG;
    msg->m.task.value_type.push_back(value_type);
    msg->m.value.push_back(wrap(ptr, bytes, loc));
    return PSF_OK;
  });
}
int psf_msg_recv_frame(psf_message* msg, void* ptr, size_t bytes, int loc) {
  return guarded([&] {
    if (!msg || (bytes && !ptr)) return PSF_ERR_ARG;
    psf::Message& m = msg->m;
    if (m.task.has_key && m.key.empty() && m.value.empty() && !m.key_frame_seen) {
      m.key = wrap(ptr, bytes, loc);
      m.key_frame_seen = true;
    } else {
      m.value.push_back(wrap(ptr, bytes, loc));
      if (!m.pending.empty()) m.pending.resize(m.value.size());
    }
    return PSF_OK;
  });
}
int psf_msg_set_value(psf_message* msg, int i, void* ptr, size_t bytes, int loc) {
  return guarded([&] {
    if (!msg || i < 0 || i >= (int)msg->m.value.size()) return PSF_ERR_ARG;
    msg->m.value[i] = wrap(ptr, bytes, loc);
    return PSF_OK;
  });
}
int psf_task_serialize(const psf_message* msg, void* buf, size_t cap, size_t* len) {
  return guarded([&] {
    if (!msg || !len) return PSF_ERR_ARG;
    psf::Task t = msg->m.task;
    t.has_key = !msg->m.key.empty();  // van.cc:131-137 double check
    const std::string s = psf::serialize_task(t);
    *len = s.size();
    if (!buf || cap < s.size()) return buf ? PSF_ERR_ARG : PSF_OK;
    memcpy(buf, s.data(), s.size());
    return PSF_OK;
  });
}
int psf_task_parse(const void* buf, size_t len, psf_message** out) {
  return guarded([&] {
    if (!out || (len && !buf)) return PSF_ERR_ARG;
    auto* m = new psf_message();
    try {
      psf::parse_task(static_cast<const uint8_t*>(buf), len, &m->m.task);
    } catch (...) {
      delete m;
      throw;
    }
    *out = m;
    return PSF_OK;
  });
}
int psf_msg_key(const psf_message* msg, void** ptr, size_t* bytes, int* loc) {
  if (!msg) return PSF_ERR_ARG;
  if (ptr) *ptr = msg->m.key.ptr;
  if (bytes) *bytes = msg->m.key.bytes;
  if (loc) *loc = (int)msg->m.key.loc;
  return PSF_OK;
}
int psf_msg_key_channel(const psf_message* msg, int32_t* key_channel) {
  if (!msg || !key_channel) return PSF_ERR_ARG;
  *key_channel = msg->m.task.key_channel;
  return PSF_OK;
}
int psf_task_value_count(const psf_message* msg, int* n) {
  if (!msg || !n) return PSF_ERR_ARG;
  *n = (int)msg->m.task.value_type.size();
  return PSF_OK;
}
int psf_msg_key_info(const psf_message* msg, int* has_key_flag, int* key_type) {
  if (!msg) return PSF_ERR_ARG;
  if (has_key_flag) *has_key_flag = msg->m.task.has_key ? 1 : 0;
  if (key_type) *key_type = msg->m.task.key_type;
  return PSF_OK;
}
int psf_msg_num_values(const psf_message* msg) { return msg ? (int)msg->m.value.size() : PSF_ERR_ARG; }
int psf_msg_value(const psf_message* msg, int i, void** ptr, size_t* bytes, int* loc) {
  if (!msg || i < 0 || i >= (int)msg->m.value.size()) return PSF_ERR_ARG;
  const auto& b = msg->m.value[i];
  if (ptr) *ptr = b.ptr;
  if (bytes) *bytes = b.bytes;
  if (loc) *loc = (int)b.loc;
  return PSF_OK;
}

int psf_msg_add_filter(psf_message* msg, int type) {
  return guarded([&] {
    if (!msg) return PSF_ERR_ARG;
    if (type < 1 || type > 4) return PSF_ERR_ARG;
    msg->m.task.filter.emplace_back();
    msg->m.task.filter.back().type = (psf::FilterConfig::Type)type;
    return (int)msg->m.task.filter.size() - 1;
  });
}
int psf_fc_set_num_bytes(psf_message* msg, int idx, int nb) {
  return guarded([&] {
    auto* f = fc_at(msg, idx);
    f->num_bytes = nb;
    f->has_num_bytes = true;
    return PSF_OK;
  });
}
int psf_fc_set_clear_cache(psf_message* msg, int idx, int v) {
  return guarded([&] {
    auto* f = fc_at(msg, idx);
    f->clear_cache_if_done = v != 0;
    f->has_clear_cache_if_done = true;
    return PSF_OK;
  });
}
int psf_fc_set_noise(psf_message* msg, int idx, float mean, float sd) {
  return guarded([&] {
    auto* f = fc_at(msg, idx);
    f->mean = mean;
    f->std = sd;
    f->has_mean = f->has_std = true;
    return PSF_OK;
  });
}
int psf_fc_add_fixed_point(psf_message* msg, int idx, const psf_fixed_point* fp) {
  return guarded([&] {
    auto* f = fc_at(msg, idx);
    f->fixed_point.emplace_back();
    auto& x = f->fixed_point.back();
    if (fp && fp->has_min) x.set_min(fp->min_value);
    if (fp && fp->has_max) x.set_max(fp->max_value);
    return PSF_OK;
  });
}
int psf_fc_num_fixed_point(const psf_message* msg, int idx) {
  return guarded([&] { return (int)fc_at(msg, idx)->fixed_point.size(); });
}
int psf_fc_fixed_point(const psf_message* msg, int idx, int k, psf_fixed_point* fp) {
  return guarded([&] {
    const auto* f = fc_at(msg, idx);
    if (!fp || k < 0 || k >= (int)f->fixed_point.size()) return PSF_ERR_ARG;
    auto& x = const_cast<psf::FixedFloatConfig&>(f->fixed_point[k]);
    x.settle();  // computed min/max a batched encode left on the device
    fp->has_min = x.has_min;
    fp->has_max = x.has_max;
    fp->min_value = x.min_value;
    fp->max_value = x.max_value;
    return PSF_OK;
  });
}
int psf_fc_signature(const psf_message* msg, int idx, int* has_signature, uint32_t* sig) {
  return guarded([&] {
    const auto* f = fc_at(msg, idx);
    if (has_signature) *has_signature = f->has_signature ? 1 : 0;
    if (sig) *sig = f->signature;
    return PSF_OK;
  });
}
int psf_fc_set_signature(psf_message* msg, int idx, int has_signature, uint32_t sig) {
  return guarded([&] {
    auto* f = fc_at(msg, idx);
    f->has_signature = has_signature != 0;
    f->signature = has_signature ? sig : 0u;
    return PSF_OK;
  });
}
int psf_fc_num_uncompressed(const psf_message* msg, int idx) {
  return guarded([&] { return (int)fc_at(msg, idx)->uncompressed_size.size(); });
}
int psf_range_even_divide(uint64_t begin, uint64_t end, uint64_t n, uint64_t i,
                          uint64_t* out_begin, uint64_t* out_end) {
  return guarded([&] {
    psf::KeyRange r = psf::even_divide(psf::KeyRange{begin, end}, n, i);
    if (out_begin) *out_begin = r.begin;
    if (out_end) *out_end = r.end;
    return PSF_OK;
  });
}

int psf_msg_slice(psf_context* ctx, const psf_message* msg, const uint64_t* bounds, int nranges,
                  int key_bytes, psf_message** outs, int* valid) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !msg || nranges < 0 || (nranges && (!bounds || !outs || !valid))) return PSF_ERR_ARG;
    std::vector<psf::KeyRange> krs(nranges);
    for (int i = 0; i < nranges; ++i) krs[i] = psf::KeyRange{bounds[i], bounds[i + 1]};
    std::vector<psf::Message> parts;
    std::vector<bool> ok;
    psf::slice_message(ctx->impl, msg->m, krs, key_bytes, &parts, &ok);
    for (int i = 0; i < nranges; ++i) {
      outs[i] = new psf_message{parts[i]};
      valid[i] = ok[i] ? 1 : 0;
    }
    return PSF_OK;
  });
}

int psf_msgs_slice(psf_context* ctx, const psf_message* const* msgs, int nmsgs, const uint64_t* bounds,
                   int nranges, int key_bytes, psf_message** outs, int* valid) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || nmsgs < 0 || nranges < 0 || (nmsgs && !msgs) || (nranges && (!bounds || !outs || !valid)))
      return PSF_ERR_ARG;
    std::vector<psf::KeyRange> krs(nranges);
    for (int i = 0; i < nranges; ++i) krs[i] = psf::KeyRange{bounds[i], bounds[i + 1]};
    std::vector<const psf::Message*> ms(nmsgs);
    for (int m = 0; m < nmsgs; ++m) {
      if (!msgs[m]) return PSF_ERR_ARG;
      ms[m] = &msgs[m]->m;
    }
    std::vector<std::vector<psf::Message>> parts;
    std::vector<std::vector<bool>> ok;
    psf::slice_messages(ctx->impl, ms, krs, key_bytes, &parts, &ok);
    for (int m = 0; m < nmsgs; ++m)
      for (int i = 0; i < nranges; ++i) {
        outs[(size_t)m * nranges + i] = new psf_message{parts[m][i]};
        valid[(size_t)m * nranges + i] = ok[m][i] ? 1 : 0;
      }
    return PSF_OK;
  });
}

int psf_node_roundtrip_ex(psf_node* snd, psf_node* rcv, const psf_message* const* tmpls, int ntmpl,
                          int iters, psf_message** enc_out, psf_message** dec_out) {
  return guarded(snd ? snd->impl->ctx() : nullptr, [&] {
    if (!snd || !rcv || !tmpls || ntmpl <= 0 || iters < 0) return PSF_ERR_ARG;
    psf_message* last_enc = nullptr;
    psf_message* last_dec = nullptr;
    psf::RemoteNode* s = snd->impl;
    psf::RemoteNode* r = rcv->impl;
    // each iteration's KEY_CACHING CRCs run on the side stream while the
    // previous iteration runs, and are collected when the iteration starts
    const psf::Message* t0 = iters ? &tmpls[0]->m : nullptr;
    psf::PresignJob next = psf::presign_launch(&s, &t0, iters ? 1 : 0, true, true);
    for (int i = 0; i < iters; ++i) {
      psf::Message m = tmpls[i % ntmpl]->m;  // fresh Task + zero-copy buffers
      psf::Message* mp = &m;
      psf::KeySigHint eh, dh;
      psf::presign_finish(next, &eh, &dh);
      if (i + 1 < iters) {  // the next iteration's CRCs, beside this one (side stream)
        const psf::Message* tn = &tmpls[(i + 1) % ntmpl]->m;
        next = psf::presign_launch(&s, &tn, 1, true, false);
      }
      psf::encode_batch(&s, &mp, 1, &eh);  // = EncodeMessage, side-info left on the device
      psf::Message w = m;                  // delivered copy (van: Task frame + data frames)
      psf::Message* wp = &w;
      psf::decode_batch(&r, &wp, 1, &dh);  // = DecodeMessage
      if (i == iters - 1) {
        if (enc_out) last_enc = new psf_message{m};
        if (dec_out) last_dec = new psf_message{w};
      }
    }
    s->ctx()->check_ranges();  // CHECK_GT(bin, 0) of the computed ranges
    if (enc_out) *enc_out = last_enc;
    if (dec_out) *dec_out = last_dec;
    return PSF_OK;
  });
}
int psf_node_roundtrip(psf_node* snd, psf_node* rcv, const psf_message* const* tmpls, int ntmpl,
                       int iters, psf_message** out) {
  return psf_node_roundtrip_ex(snd, rcv, tmpls, ntmpl, iters, nullptr, out);
}

int psf_nodes_encode(psf_node* const* nodes, psf_message* const* msgs, int n) {
  return guarded((nodes && n > 0 && nodes[0]) ? nodes[0]->impl->ctx() : nullptr, [&] {
    if (n < 0 || (n && (!nodes || !msgs))) return PSF_ERR_ARG;
    std::vector<psf::RemoteNode*> nd(n);
    std::vector<psf::Message*> ms(n);
    for (int i = 0; i < n; ++i) {
      if (!nodes[i] || !msgs[i]) return PSF_ERR_ARG;
      nd[i] = nodes[i]->impl;
      ms[i] = &msgs[i]->m;
    }
    psf::encode_batch(nd.data(), ms.data(), n);
    return PSF_OK;
  });
}
int psf_nodes_decode(psf_node* const* nodes, psf_message* const* msgs, int n) {
  return guarded((nodes && n > 0 && nodes[0]) ? nodes[0]->impl->ctx() : nullptr, [&] {
    if (n < 0 || (n && (!nodes || !msgs))) return PSF_ERR_ARG;
    std::vector<psf::RemoteNode*> nd(n);
    std::vector<psf::Message*> ms(n);
    for (int i = 0; i < n; ++i) {
      if (!nodes[i] || !msgs[i]) return PSF_ERR_ARG;
      nd[i] = nodes[i]->impl;
      ms[i] = &msgs[i]->m;
    }
    psf::decode_batch(nd.data(), ms.data(), n);
    return PSF_OK;
  });
}
int psf_nodes_roundtrip_ex(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                           const int* phase_end, int nphases, int iters, psf_message** enc_out,
                           psf_message** dec_out) {
  return psf_nodes_roundtrip_opts(snd, rcv, tmpls, n, phase_end, nphases, iters, 0, enc_out, dec_out);
}
int psf_nodes_roundtrip_opts(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                             const int* phase_end, int nphases, int iters, int flags, psf_message** enc_out,
                             psf_message** dec_out) {
  return guarded((snd && n > 0 && snd[0]) ? snd[0]->impl->ctx() : nullptr, [&] {
    if (flags & ~PSF_RT_WIRE) return PSF_ERR_ARG;
    const bool wire = (flags & PSF_RT_WIRE) != 0;
    if (n <= 0 || iters < 0 || !snd || !rcv || !tmpls) return PSF_ERR_ARG;
    std::vector<int> ends;
    if (phase_end && nphases > 0) {
      for (int p = 0; p < nphases; ++p) {
        if (phase_end[p] <= (p ? phase_end[p - 1] : 0) || phase_end[p] > n) return PSF_ERR_ARG;
        ends.push_back(phase_end[p]);
      }
      if (ends.back() != n) return PSF_ERR_ARG;
    } else {
      ends.push_back(n);
    }
    std::vector<psf::RemoteNode*> s(n), r(n);
    for (int i = 0; i < n; ++i) {
      if (!snd[i] || !rcv[i] || !tmpls[i]) return PSF_ERR_ARG;
      s[i] = snd[i]->impl;
      r[i] = rcv[i]->impl;
    }
    // a phase's FIXING_FLOAT decode is held back until the next phase's
    // first encode launch (one launch instead of two); whatever is still held
    // is launched before returning, also on an error
    std::set<psf::Context*> dctx;
    for (int i = 0; i < n; ++i) {
      dctx.insert(s[i]->ctx());
      dctx.insert(r[i]->ctx());
    }
    struct DeferScope {
      std::set<psf::Context*>& cs;
      explicit DeferScope(std::set<psf::Context*>& c) : cs(c) {
        for (psf::Context* x : cs) x->set_defer_decodes(true);
      }
      void finish() {
        for (psf::Context* x : cs) {
          x->set_defer_decodes(false);
          x->flush_deferred();
        }
      }
      ~DeferScope() {
        for (psf::Context* x : cs) {
          x->set_defer_decodes(false);
          try {
            x->flush_deferred();
          } catch (...) {
          }
        }
      }
    } defer(dctx);
    std::vector<psf::Message> m(n), w(n);
    std::vector<psf::Message*> mp(n), wp(n);
    std::vector<const psf::Message*> tp(n);
    for (int i = 0; i < n; ++i) tp[i] = &tmpls[i]->m;
    std::vector<psf::KeySigHint> eh(n), dh(n);
    // every KEY_CACHING CRC of an iteration (all phases): launched on the
    // context's side stream when the previous iteration starts, collected
    // when this one starts
    psf::PresignJob next = psf::presign_launch(s.data(), tp.data(), iters ? n : 0, true, true);
    for (int it = 0; it < iters; ++it) {
      PSF_HPROF(14);
      {
        PSF_HPROF(12);
        std::fill(eh.begin(), eh.end(), psf::KeySigHint{});
        std::fill(dh.begin(), dh.end(), psf::KeySigHint{});
        psf::presign_finish(next, eh.data(), dh.data());
      }
      if (it + 1 < iters) {  // the next iteration's CRCs, beside this one (side stream)
        PSF_HPROF(13);
        next = psf::presign_launch(s.data(), tp.data(), n, true, false);
      }
      int b = 0;
      for (int e : ends) {  // phase [b, e): encode all, deliver, decode all
        {
          PSF_HPROF(0);
          for (int i = b; i < e; ++i) {
            m[i] = tmpls[i]->m;  // fresh Task + zero-copy buffers
            mp[i] = &m[i];
          }
        }
        {
          PSF_HPROF(1);
          psf::encode_batch(s.data() + b, mp.data() + b, e - b, eh.data() + b);
        }
        {
          PSF_HPROF(5);
          for (int i = b; i < e; ++i) {
            if (wire) {
              // Van::Send / Van::Recv (van.cc:122-191, 244-269): the Task
              // serialised after EncodeMessage (its computed min/max settled
              // to the host first), parsed by the receiver, the data frames
              // delivered as they are (zero copy)
              psf::Task t = m[i].task;
              t.has_key = !m[i].key.empty();
              const std::string frame = psf::serialize_task(t);
              w[i] = psf::Message();
              psf::parse_task(reinterpret_cast<const uint8_t*>(frame.data()), frame.size(), &w[i].task);
              w[i].key = m[i].key;
              w[i].value = m[i].value;
            } else {
              w[i] = m[i];  // delivered copy
            }
            wp[i] = &w[i];
          }
        }
        {
          PSF_HPROF(6);
          psf::decode_batch(r.data() + b, wp.data() + b, e - b, dh.data() + b);
        }
        b = e;
      }
    }
    defer.finish();
    std::set<psf::Context*> ctxs;  // CHECK_GT(bin, 0) of the lazily encoded ranges
    for (int i = 0; i < n; ++i) ctxs.insert(s[i]->ctx());
    for (psf::Context* c : ctxs) c->check_ranges();
    for (int i = 0; i < n; ++i) {
      if (enc_out) enc_out[i] = iters ? new psf_message{m[i]} : nullptr;
      if (dec_out) dec_out[i] = iters ? new psf_message{w[i]} : nullptr;
    }
    return PSF_OK;
  });
}
int psf_nodes_roundtrip(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                        int iters) {
  return psf_nodes_roundtrip_ex(snd, rcv, tmpls, n, nullptr, 0, iters, nullptr, nullptr);
}

int psf_spill_pack(psf_context* ctx, psf_message* const* msgs, const int* dest, const int* server, int n,
                   int world, int64_t* sizes, psf_spill** out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !sizes || !out || n < 0 || world <= 0 || (n && (!msgs || !dest || !server))) return PSF_ERR_ARG;
    std::vector<psf::Message*> ms(n);
    for (int i = 0; i < n; ++i) {
      if (!msgs[i]) return PSF_ERR_ARG;
      ms[i] = &msgs[i]->m;
    }
    auto* p = new psf::SpillPlan(ctx->impl, ms.data(), dest, server, n, world);
    for (int r = 0; r < 2 * world; ++r) sizes[r] = p->sizes()[r];
    *out = reinterpret_cast<psf_spill*>(p);
    return PSF_OK;
  });
}
int psf_spill_fill(psf_spill* plan, void* sendbuf) {
  return guarded(plan ? reinterpret_cast<psf::SpillPlan*>(plan)->context() : nullptr, [&] {
    if (!plan) return PSF_ERR_ARG;
    reinterpret_cast<psf::SpillPlan*>(plan)->fill(sendbuf);
    return PSF_OK;
  });
}
int psf_spill_destroy(psf_spill* plan) {
  delete reinterpret_cast<psf::SpillPlan*>(plan);
  return PSF_OK;
}
int psf_spill_unpack(psf_context* ctx, const void* recvbuf, int world, const int64_t* sizes, psf_message** outs,
                     int* servers, int cap, int* n) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !sizes || !n || world <= 0 || cap < 0 || (cap && (!outs || !servers))) return PSF_ERR_ARG;
    int64_t total = 0;
    for (int r = 0; r < 2 * world; ++r) total += sizes[r];
    if (total && !recvbuf) return PSF_ERR_ARG;
    std::vector<psf::Message> ms;
    std::vector<int> sv;
    psf::spill_unpack(ctx->impl, psf::own_copy(ctx->impl, recvbuf, (size_t)total), world, sizes, &ms, &sv);
    *n = (int)ms.size();
    if ((int)ms.size() > cap) {
      g_last_error = "psf_spill_unpack: more messages than cap";
      return PSF_ERR_ARG;
    }
    for (size_t i = 0; i < ms.size(); ++i) {
      outs[i] = new psf_message{std::move(ms[i])};
      servers[i] = sv[i];
    }
    return PSF_OK;
  });
}

int psf_router_create(psf_context* ctx, const uint64_t* bounds, int nservers, int rank, int world, int loopback,
                      psf_router** out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !bounds || !out || nservers <= 0) return PSF_ERR_ARG;
    std::vector<psf::KeyRange> krs(nservers);
    for (int i = 0; i < nservers; ++i) krs[i] = psf::KeyRange{bounds[i], bounds[i + 1]};
    *out = reinterpret_cast<psf_router*>(new psf::PushRouter(ctx->impl, krs, rank, world, loopback != 0));
    psf::Context::ref(ctx->impl);
    return PSF_OK;
  });
}
int psf_router_destroy(psf_router* r) {
  if (!r) return PSF_OK;
  psf::Context* c = reinterpret_cast<psf::PushRouter*>(r)->context();
  delete reinterpret_cast<psf::PushRouter*>(r);
  psf::Context::unref(c);
  return PSF_OK;
}
static psf::PushRouter* R(psf_router* r) {
  if (!r) throw psf::CheckError(PSF_ERR_ARG, "null router");
  return reinterpret_cast<psf::PushRouter*>(r);
}
int psf_router_keep_encoded(psf_router* r, int on) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { R(r)->keep_encoded(on != 0); return PSF_OK; });
}
int psf_router_encode(psf_router* r, psf_message* const* streams, int n, int64_t* sizes) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (n < 0 || (n && !streams) || !sizes) return PSF_ERR_ARG;
    std::vector<const psf::Message*> ms(n);
    for (int i = 0; i < n; ++i) {
      if (!streams[i]) return PSF_ERR_ARG;
      ms[i] = &streams[i]->m;
    }
    R(r)->encode(ms.data(), n, sizes);
    return PSF_OK;
  });
}
int psf_router_fill(psf_router* r, void* sendbuf) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { R(r)->fill(sendbuf); return PSF_OK; });
}
int psf_router_decode_local(psf_router* r) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { R(r)->decode_local(); return PSF_OK; });
}
int psf_router_decode_received(psf_router* r, const void* recvbuf, const int64_t* sizes_in) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (!sizes_in) return PSF_ERR_ARG;
    R(r)->decode_received(static_cast<const uint8_t*>(recvbuf), sizes_in);
    return PSF_OK;
  });
}
int psf_router_step(psf_router* r, psf_message* const* streams, int n, int iters) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (n < 0 || (n && !streams) || iters < 0) return PSF_ERR_ARG;
    psf::PushRouter* pr = R(r);
    std::vector<const psf::Message*> ms(n);
    for (int i = 0; i < n; ++i) {
      if (!streams[i]) return PSF_ERR_ARG;
      ms[i] = &streams[i]->m;
    }
    if (pr->exchange()) {  // any world: the native exchange
      for (int it = 0; it < iters; ++it) {
        pr->encode_launch(ms.data(), n, it == 0);
        if (it + 1 < iters) pr->prefetch(ms.data(), n);
        pr->exchange_step();
      }
      return PSF_OK;
    }
    if (pr->world() > 1 || pr->loopback())
      throw psf::CheckError(PSF_ERR_ARG, "psf_router_step: a router with other ranks needs an exchange");
    std::vector<int64_t> sizes(2 * (size_t)pr->world());
    if (iters > 0) pr->encode_launch(ms.data(), n);
    for (int it = 0; it < iters; ++it) {
      // the next step's slicing pass goes ahead of this step's decodes (and
      // of the wait for its COMPRESSING lengths)
      if (it + 1 < iters) pr->prefetch(ms.data(), n);
      pr->encode_finish(sizes.data());
      for (int64_t s : sizes)
        if (s) throw psf::CheckError(PSF_ERR_ARG, "psf_router_step: slices for other ranks need an exchange");
      pr->fill(nullptr);
      // this step's decodes in flight, the next step's encode queued behind
      // them, then the wait for the decodes: the device runs on from one
      // step into the next while the host waits
      pr->decode_local_launch();
      if (it + 1 < iters) pr->encode_launch(ms.data(), n, false);
      pr->decode_local_finish();
    }
    return PSF_OK;
  });
}
int psf_exchange_unique_id(void* out, size_t bytes) {
  return guarded([&] {
    if (!out || bytes < 128) return PSF_ERR_ARG;
    psf::rccl_unique_id(out);
    return PSF_OK;
  });
}
int psf_exchange_create(psf_context* ctx, int rank, int world, const char* name, int transport, const void* nccl_id,
                        uint64_t meta_cap, uint64_t host_cap, psf_exchange** out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !name || !out || (transport != PSF_EXCHANGE_RCCL && transport != PSF_EXCHANGE_HOST)) return PSF_ERR_ARG;
    *out = reinterpret_cast<psf_exchange*>(new psf::Exchange(
        ctx->impl, rank, world, name, transport == PSF_EXCHANGE_RCCL ? psf::Exchange::kRccl : psf::Exchange::kHost,
        nccl_id, meta_cap, host_cap));
    psf::Context::ref(ctx->impl);
    return PSF_OK;
  });
}
int psf_exchange_destroy(psf_exchange* ex) {
  if (!ex) return PSF_OK;
  // deleted now, or when the last router using it goes
  psf::Exchange::unref(reinterpret_cast<psf::Exchange*>(ex));
  return PSF_OK;
}
int psf_exchange_stats(psf_exchange* ex, int64_t* out) {
  if (!ex || !out) return PSF_ERR_ARG;
  const psf::Exchange* e = reinterpret_cast<psf::Exchange*>(ex);
  out[0] = e->bytes_sent;
  out[1] = e->steps;
  out[2] = e->wait_ns;
  return PSF_OK;
}
int psf_exchange_data_stats(psf_exchange* ex, int64_t* out) {
  if (!ex || !out) return PSF_ERR_ARG;
  const psf::Exchange* e = reinterpret_cast<psf::Exchange*>(ex);
  out[0] = e->rccl_bytes;
  out[1] = e->rccl_sends;
  out[2] = e->copied_bytes;
  out[3] = e->failed() ? 1 : 0;
  return PSF_OK;
}
int psf_router_set_exchange(psf_router* r, psf_exchange* ex) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    psf::PushRouter* pr = R(r);
    psf::Exchange* e = reinterpret_cast<psf::Exchange*>(ex);
    if (e && (e->context() != pr->context() || e->world() != pr->world())) return PSF_ERR_ARG;
    pr->set_exchange(e);
    return PSF_OK;
  });
}
int psf_router_set_store(psf_router* r, psf_kvmap* store) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    psf::PushRouter* pr = R(r);
    if (store && store->impl->context() != pr->context()) return PSF_ERR_ARG;
    pr->set_store(store ? store->impl : nullptr);
    return PSF_OK;
  });
}
static std::vector<const psf::Message*> msg_ptrs(psf_message* const* ms, int n) {
  if (n < 0 || (n && !ms)) throw psf::CheckError(PSF_ERR_ARG, "bad message array");
  std::vector<const psf::Message*> v(n);
  for (int i = 0; i < n; ++i) {
    if (!ms[i]) throw psf::CheckError(PSF_ERR_ARG, "null message");
    v[i] = &ms[i]->m;
  }
  return v;
}
int psf_router_pull(psf_router* r, psf_message* const* requests, int n, int iters) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (iters < 0) return PSF_ERR_ARG;
    psf::PushRouter* pr = R(r);
    const std::vector<const psf::Message*> ms = msg_ptrs(requests, n);
    for (int it = 0; it < iters; ++it) pr->pull_step(ms.data(), n, it == 0, it + 1 < iters);
    return PSF_OK;
  });
}
int psf_router_pull_encode(psf_router* r, psf_message* const* requests, int n, int64_t* sizes) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (!sizes) return PSF_ERR_ARG;
    const std::vector<const psf::Message*> ms = msg_ptrs(requests, n);
    R(r)->pull_encode(ms.data(), n, sizes);
    return PSF_OK;
  });
}
int psf_router_pull_serve(psf_router* r, const void* recvbuf, const int64_t* sizes_in, int64_t* sizes) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (!sizes_in || !sizes) return PSF_ERR_ARG;
    R(r)->pull_serve(static_cast<const uint8_t*>(recvbuf), sizes_in, sizes);
    return PSF_OK;
  });
}
int psf_router_pull_finish(psf_router* r, const void* recvbuf, const int64_t* sizes_in) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (!sizes_in) return PSF_ERR_ARG;
    R(r)->pull_finish(static_cast<const uint8_t*>(recvbuf), sizes_in);
    return PSF_OK;
  });
}
int psf_router_num_pulled(psf_router* r) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { return (int)R(r)->pulled().size(); });
}
int psf_router_pulled(psf_router* r, int i, int32_t* stream, psf_message** out) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    const auto& p = R(r)->pulled();
    if (i < 0 || i >= (int)p.size() || !out) return PSF_ERR_ARG;
    if (stream) *stream = p[i].stream;
    *out = new psf_message{p[i].msg};
    return PSF_OK;
  });
}
int psf_router_host_stats(psf_router* r, int64_t* out) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    if (!out) return PSF_ERR_ARG;
    psf::PushRouter* pr = R(r);
    out[0] = pr->stat_steps;
    out[1] = pr->stat_encode_ns;
    out[2] = pr->stat_decode_ns;
    return PSF_OK;
  });
}
int psf_router_host_stats_reset(psf_router* r) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    psf::PushRouter* pr = R(r);
    pr->stat_steps = pr->stat_encode_ns = pr->stat_decode_ns = 0;
    return PSF_OK;
  });
}
int psf_router_num_results(psf_router* r) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { return (int)R(r)->results().size(); });
}
int psf_router_result(psf_router* r, int i, int* server, psf_message** out) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    const auto& res = R(r)->results();
    if (i < 0 || i >= (int)res.size() || !out) return PSF_ERR_ARG;
    if (server) *server = res[i].first;
    *out = new psf_message{res[i].second};
    return PSF_OK;
  });
}
int psf_router_num_encoded(psf_router* r) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] { return (int)R(r)->encoded().size(); });
}
int psf_router_encoded(psf_router* r, int i, int32_t* stream, int* server, psf_message** out) {
  return guarded(r ? reinterpret_cast<psf::PushRouter*>(r)->context() : nullptr, [&] {
    const auto& e = R(r)->encoded();
    if (i < 0 || i >= (int)e.size() || !out) return PSF_ERR_ARG;
    if (stream) *stream = e[i].stream;
    if (server) *server = e[i].server;
    *out = new psf_message{e[i].msg};
    return PSF_OK;
  });
}

int psf_context_host_stats(psf_context* ctx, int64_t* wait_ns, int64_t* waits) {
  if (!ctx || !wait_ns || !waits) return PSF_ERR_ARG;
  for (int w = 0; w < psf::Context::kWaitNum; ++w) {
    wait_ns[w] = ctx->impl->wait_ns(w);
    waits[w] = ctx->impl->wait_count(w);
  }
  return PSF_OK;
}
int psf_context_host_stats_reset(psf_context* ctx) {
  if (!ctx) return PSF_ERR_ARG;
  ctx->impl->reset_waits();
  return PSF_OK;
}
int psf_context_set_cache_limit(psf_context* ctx, uint64_t hbm_bytes, uint64_t pinned_bytes) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx) return PSF_ERR_ARG;
    ctx->impl->set_cache_limit(hbm_bytes, pinned_bytes);
    return PSF_OK;
  });
}
int psf_context_memory_stats(psf_context* ctx, uint64_t* out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !out) return PSF_ERR_ARG;
    const psf::Context::MemoryStats m = ctx->impl->memory_stats();
    const uint64_t v[8] = {m.dev_cached, m.dev_cap, m.dev_allocated, m.dev_evictions,
                           m.host_cached, m.host_cap, m.host_allocated, m.host_evictions};
    for (int i = 0; i < 8; ++i) out[i] = v[i];
    return PSF_OK;
  });
}
int psf_set_device_cache_limit(int device, uint64_t hbm_bytes, uint64_t pinned_bytes) {
  return guarded([&] {
    if (device < 0) return PSF_ERR_ARG;
    psf::set_device_cache_limit(device, hbm_bytes, pinned_bytes);
    return PSF_OK;
  });
}
int psf_device_memory_stats(int device, uint64_t* out) {
  return guarded([&] {
    if (device < 0 || !out) return PSF_ERR_ARG;
    const psf::DeviceMemoryStats d = psf::device_memory_stats(device);
    const psf::Context::MemoryStats& m = d.m;
    const uint64_t v[10] = {m.dev_cached, m.dev_cap, m.dev_allocated, m.dev_evictions,
                            m.host_cached, m.host_cap, m.host_allocated, m.host_evictions,
                            d.holders, d.shared_streams};
    for (int i = 0; i < 10; ++i) out[i] = v[i];
    return PSF_OK;
  });
}
int psf_profile_enable(psf_context* ctx, int kernel_mask) {
  if (!ctx) return PSF_ERR_ARG;
  ctx->impl->prof()->enable((uint32_t)kernel_mask);
  return PSF_OK;
}
int psf_profile_stride(psf_context* ctx, int stride) {
  if (!ctx || stride < 1) return PSF_ERR_ARG;
  ctx->impl->prof()->set_stride((uint32_t)stride);
  return PSF_OK;
}
int psf_profile_reset(psf_context* ctx) {
  if (!ctx) return PSF_ERR_ARG;
  ctx->impl->prof()->reset();
  return PSF_OK;
}
int psf_profile_read(psf_context* ctx, int k, int64_t* launches, double* total_ms,
                     double* alg_bytes) {
  if (!ctx || k < 0 || k >= psf::kKNum) return PSF_ERR_ARG;
  psf::Profiler* p = ctx->impl->prof();
  p->collect();
  if (launches) *launches = p->launches[k];
  if (total_ms) *total_ms = p->total_ms[k];
  if (alg_bytes) *alg_bytes = p->bytes[k];
  return PSF_OK;
}
const char* psf_profile_kernel_name(int k) {
  static const char* names[] = {"ff_minmax_partials", "ff_encode", "ff_decode", "crc32c_chunks",
                                "noise_add", "snappy_compress", "snappy_decompress", "ordered_match",
                                "kvmap_push", "kvmap_get", "ff_decode_minmax", "ff_minmax_encode"};
  static_assert(sizeof(names) / sizeof(names[0]) == psf::kKNum, "one name per kernel id");
  return (k >= 0 && k < psf::kKNum) ? names[k] : "?";
}

int psf_fc_add_uncompressed(psf_message* msg, int idx, uint64_t size) {
  return guarded([&] {
    fc_at(msg, idx)->uncompressed_size.push_back(size);
    return PSF_OK;
  });
}

int psf_fc_uncompressed(const psf_message* msg, int idx, int i, uint64_t* size) {
  return guarded([&] {
    const auto* f = fc_at(msg, idx);
    if (!size || i < 0 || i >= (int)f->uncompressed_size.size()) return PSF_ERR_ARG;
    *size = f->uncompressed_size[i];
    return PSF_OK;
  });
}

// ------------------------------------------------- server-side consumers
int psf_node_set_defer_dequant(psf_node* node, int enable) {
  return guarded(node ? node->impl->ctx() : nullptr, [&] {
    if (!node) return PSF_ERR_ARG;
    node->impl->set_defer_dequant(enable != 0);
    return PSF_OK;
  });
}
int psf_msg_pending(const psf_message* msg, int i, int* num_bytes, float* min_value, float* max_value) {
  if (!msg || i < 0 || i >= (int)msg->m.value.size()) return PSF_ERR_ARG;
  const psf::PendingDequant pd = msg->m.is_pending(i) ? msg->m.pending[i] : psf::PendingDequant{};
  if (num_bytes) *num_bytes = pd.nb;
  if (min_value) *min_value = pd.min_value;
  if (max_value) *max_value = pd.max_value;
  return PSF_OK;
}
int psf_msg_materialize(psf_context* ctx, psf_message* msg) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !msg) return PSF_ERR_ARG;
    psf::materialize(ctx->impl, &msg->m);
    return PSF_OK;
  });
}
int psf_ordered_match(psf_context* ctx, const uint64_t* d_src_key, size_t nsrc, const void* d_src_val,
                      const uint64_t* d_dst_key, size_t ndst, void* d_dst_val, int k, int value_type,
                      int op, size_t* n) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !n || k <= 0 || op < 0 || op > 4) return PSF_ERR_ARG;
    if (value_type != PSF_DT_FLOAT && value_type != PSF_DT_DOUBLE) return PSF_ERR_ARG;
    *n = psf::ordered_match_raw(ctx->impl, d_src_key, nsrc, d_src_val, psf::PendingDequant{}, d_dst_key,
                                ndst, d_dst_val, value_type, k, op);
    return PSF_OK;
  });
}
int psf_ff_decode_match(psf_context* ctx, const uint64_t* d_src_key, size_t nsrc, const void* d_code,
                        int num_bytes, float min_value, float max_value, const uint64_t* d_dst_key,
                        size_t ndst, void* d_dst_val, int k, int op, size_t* n) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !n || k <= 0 || op < 0 || op > 4) return PSF_ERR_ARG;
    if (num_bytes <= 0 || num_bytes >= 8) return PSF_ERR_NBYTES;
    if (!((double)max_value - (double)min_value > 0)) return PSF_ERR_BIN;
    psf::PendingDequant pd{num_bytes, min_value, max_value};
    *n = psf::ordered_match_raw(ctx->impl, d_src_key, nsrc, d_code, pd, d_dst_key, ndst, d_dst_val,
                                PSF_DT_FLOAT, k, op);
    return PSF_OK;
  });
}
int psf_msg_ordered_match(psf_context* ctx, const psf_message* msg, int i, const uint64_t* d_dst_key,
                          size_t ndst, void* d_dst_val, int k, int value_type, int op, size_t* n) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !msg || !n || op < 0 || op > 4) return PSF_ERR_ARG;
    if (value_type != PSF_DT_FLOAT && value_type != PSF_DT_DOUBLE) return PSF_ERR_ARG;
    *n = psf::ordered_match(ctx->impl, msg->m, i, d_dst_key, ndst, d_dst_val, value_type, k, op);
    return PSF_OK;
  });
}
int psf_kvmap_create(psf_context* ctx, size_t capacity, int lr_type, double alpha, double beta,
                     double lambda1, double lambda2, psf_kvmap** out) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    if (!ctx || !out || (lr_type != 1 && lr_type != 2)) return PSF_ERR_ARG;
    psf::FtrlConfig c;
    c.lr_type = lr_type;
    c.alpha = alpha;
    c.beta = beta;
    c.lambda1 = lambda1;
    c.lambda2 = lambda2;
    *out = new psf_kvmap{new psf::KvMapFtrl(ctx->impl, capacity, c), ctx->impl};
    psf::Context::ref(ctx->impl);
    return PSF_OK;
  });
}
int psf_kvmap_destroy(psf_kvmap* map) {
  if (!map) return PSF_OK;
  psf::KvMapFtrl::unref(map->impl);  // (drops the context reference with the map)
  delete map;
  return PSF_OK;
}
int psf_kvmap_set_value(psf_kvmap* map, const psf_message* msg) {
  return guarded(map ? map->ctx : nullptr, [&] {
    if (!map || !msg) return PSF_ERR_ARG;
    map->impl->set_value(msg->m);
    return PSF_OK;
  });
}
int psf_kvmap_get_value(psf_kvmap* map, psf_message* msg) {
  return guarded(map ? map->ctx : nullptr, [&] {
    if (!map || !msg) return PSF_ERR_ARG;
    map->impl->get_value(&msg->m);
    return PSF_OK;
  });
}
int psf_kvmap_push(psf_kvmap* map, const uint64_t* d_keys, size_t n, const float* d_grad) {
  return guarded(map ? map->ctx : nullptr, [&] {
    if (!map || (n && (!d_keys || !d_grad))) return PSF_ERR_ARG;
    map->impl->push(d_keys, n, d_grad, psf::PendingDequant{});
    return PSF_OK;
  });
}
int psf_kvmap_pull(psf_kvmap* map, const uint64_t* d_keys, size_t n, float* d_w) {
  return guarded(map ? map->ctx : nullptr, [&] {
    if (!map || (n && (!d_keys || !d_w))) return PSF_ERR_ARG;
    map->impl->pull(d_keys, n, d_w);
    return PSF_OK;
  });
}
int psf_kvmap_stats(psf_kvmap* map, int64_t* nnz, double* weight_sum, double* delta_sum, uint64_t* size) {
  return guarded(map ? map->ctx : nullptr, [&] {
    if (!map) return PSF_ERR_ARG;
    const psf::KvMapFtrl::Stats s = map->impl->stats();
    if (nnz) *nnz = s.nnz;
    if (weight_sum) *weight_sum = s.weight_sum;
    if (delta_sum) *delta_sum = s.delta_sum;
    if (size) *size = s.size;
    return PSF_OK;
  });
}

}  // extern "C"

// test knob: the RCCL exchange's self slice through ncclSend / ncclRecv to self
extern "C" int psf_debug_exchange_self_p2p(int on) {
  psf::set_exchange_self_p2p(on != 0);
  return PSF_OK;
}

// diagnostic: the context's ff_fused_batch counter words (after a sync)
extern "C" int psf_debug_fused_ctl(psf_context* ctx, uint32_t* out, int n) {
  return guarded(ctx ? ctx->impl : nullptr, [&] {
    psf::FfFusedCtl* f = ctx->impl->fused();
    if (!f || n < 0 || (size_t)n * 4 > psf::kFusedCtlBytes) return PSF_ERR_ARG;
    ctx->impl->sync();
    PSF_HIP_CHECK(hipMemcpy(out, f->ctl, (size_t)n * 4, hipMemcpyDeviceToHost));
    return PSF_OK;
  });
}
