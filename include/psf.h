/*
 * libpsf -- MI355X-native (HIP/gfx950) parameter_server filter codec chain.
 *
 * C ABI of the drop-in boundary.  Plain pointers and sizes only; `stream` is a
 * hipStream_t passed as void* (see psf_context_create).  Every entry
 * point returns PSF_OK (0) or a negative PSF_ERR_* code; psf_last_error()
 * describes the last failure on the calling thread.  The reference aborts the
 * process through glog CHECK at the same points; the C++ shim in
 * include/psf_ps_filter.h maps a non-zero status back to that fatal CHECK.
 *
 * Two layers:
 *
 *  1. Codec kernels -- what a reference Filter subclass binds
 *     (replaces the element loops of the reference headers):
 *       psf_ff_encode / psf_ff_decode   <- FixingFloatFilter::convert<V>
 *                                          src/filter/fixing_float.h:50-101
 *       psf_key_signature / psf_crc32c  <- KeyCachingFilter signature
 *                                          src/filter/key_caching.h:18,43
 *                                          (crc32c::Value, src/util/crc32c.h:19-21)
 *       psf_snappy_*                    <- CompressingFilter's SArray::CompressTo /
 *                                          UncompressFrom, src/util/shared_array_inl.h:
 *                                          232-255 (snappy::RawCompress /
 *                                          GetUncompressedLength / RawUncompress, 1.1.8)
 *
 *  2. Filter plugin surface -- the reference's message path in one library:
 *       psf_node_encode / psf_node_decode  <- RemoteNode::EncodeMessage / DecodeMessage
 *                                             src/system/remote_node.cc:17-29, running
 *                                             Filter::create (src/filter/filter.cc:9-23)
 *                                             instances of KEY_CACHING, FIXING_FLOAT,
 *                                             COMPRESSING, NOISE on HBM buffers
 *       psf_msg_* / psf_fc_*               <- Message / Task / FilterConfig fields
 *                                             (src/system/message.h:10-76,
 *                                             src/system/proto/task.proto:28-39,
 *                                             src/filter/proto/filter.proto:3-35)
 */
#ifndef PSF_H_
#define PSF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define PSF_OK 0
#define PSF_ERR_ARG (-1)         /* bad argument / unknown filter type            */
#define PSF_ERR_NBYTES (-2)      /* CHECK_GT(nbytes,0), CHECK_LT(nbytes,8)        */
#define PSF_ERR_BIN (-3)         /* CHECK_GT(bin,0): max <= min after +1e-6        */
#define PSF_ERR_HIP (-4)         /* HIP runtime failure                           */
#define PSF_ERR_CHECK (-5)       /* other reference CHECK (signature mismatch ...) */
#define PSF_ERR_UNSUPPORTED (-6)
#define PSF_ERR_TIMEOUT (-7)     /* reserved: no entry point returns it (libpsf has no device-side waits) */

/* ---- task.proto DataType / filter.proto Type values -------------------- */
#define PSF_DT_UINT64 8
#define PSF_DT_FLOAT 9
#define PSF_DT_DOUBLE 10
#define PSF_DT_CHAR 11
#define PSF_KEY_CACHING 1
#define PSF_COMPRESSING 2
#define PSF_FIXING_FLOAT 3
#define PSF_NOISE 4

/* buffer location */
#define PSF_LOC_HOST 0
#define PSF_LOC_DEVICE 1

const char* psf_last_error(void);
const char* psf_version(void);

/* time(NULL) is FIXING_FLOAT's LCG seed in the reference (fixing_float.h:78);
 * enable=1 pins it to `t` process-wide (parity testing), enable=0 restores it. */
void psf_set_clock(int enable, int64_t t);


/* The device the reference-side adapter (include/psf_ps_filter.h) creates
 * its contexts on: the last psf_set_default_device(d), else the PSF_DEVICE
 * environment variable (a device ordinal), else 0.  One server process per
 * GPU (src/system/assigner.h:17-28 gives each server its key range) sets
 * PSF_DEVICE=<gpu> at launch.  psf_set_default_device returns PSF_ERR_ARG for
 * a negative device; psf_default_device reads the environment once. */
int psf_set_default_device(int device);
int psf_default_device(void);

/* ---- execution context (device + stream + workspace) ------------------- */
/* A context (and the nodes and messages that use it) is not thread-safe:
 * callers serialise its use, as the reference serialises one Customer's
 * filter calls under Executor::node_mu_ (executor.cc:110,143,170). */
typedef struct psf_context psf_context;
/* own_stream=1: a private non-blocking stream; own_stream=0: kernels go on
 * `stream` as given (NULL = the legacy default stream); own_stream=2
 * (PSF_STREAM_SHARED, stream NULL): one of the device's 4 process-wide
 * streams, round robin -- what the reference-side adapter uses, so hundreds of
 * per-peer contexts do not alias hundreds of streams onto the hardware queues
 * (each context still keeps its own order on its stream).  device < 0 gives a
 * host-only context (host-resident buffers; codecs needing HBM fail).  A
 * context may be used from any thread (one at a time): every entry point
 * makes the context's device current for the call and restores the
 * caller's. */
#define PSF_STREAM_GIVEN 0
#define PSF_STREAM_OWN 1
#define PSF_STREAM_SHARED 2
int psf_context_create(int device, void* stream, int own_stream, psf_context** out);
int psf_context_destroy(psf_context* ctx);
/* Waits for the context's stream; also resolves the min/max a batched encode
 * left on the device (psf_nodes_encode) and returns PSF_ERR_BIN if any of
 * them failed CHECK_GT(bin, 0) (fixing_float.h:71) since the last check. */
int psf_context_sync(psf_context* ctx);
/* Ordered on the context's stream, then synchronous: copy `bytes` from a
 * buffer the library returned (device or host) into host memory. */
int psf_copy_to_host(psf_context* ctx, void* dst, const void* src, size_t bytes);
/* The same, left in flight on the context's stream (complete after
 * psf_context_sync). */
int psf_copy_to_host_async(psf_context* ctx, void* dst, const void* src, size_t bytes);
/* A pinned host buffer of `bytes` from the context's pool (the fast target of
 * the copies above); released with psf_host_buffer_release(*handle), which
 * may outlive the context.  The adapter hands these out as the reference's
 * zero-copy SArrays with a custom deleter (van.cc:244-255's pattern). */
int psf_host_buffer_alloc(psf_context* ctx, size_t bytes, void** ptr, void** handle);
int psf_host_buffer_release(void* handle);

/* ---- layer 1: codec kernels (device pointers, async unless noted) ------ */
typedef struct {
  int32_t has_min, has_max; /* FixedFloatConfig has-bits                      */
  float min_value, max_value;
} psf_fixed_point;

/* FIXING_FLOAT encode of n values (value_type FLOAT/DOUBLE) into n*num_bytes
 * bytes at d_code.  fp is in/out: preset min/max are honoured, computed ones
 * are written back (this call then synchronises the stream once).  `seed` is
 * the LCG seed the reference takes from time(NULL). */
int psf_ff_encode(psf_context* ctx, const void* d_values, size_t n, int value_type,
                  int num_bytes, psf_fixed_point* fp, int32_t seed, void* d_code);

/* Fully asynchronous encode: side-info {min,max} goes to d_range (device
 * float[2]) and the CHECK_GT(bin,0) outcome to d_status (device int32,
 * PSF_OK or PSF_ERR_BIN); either may be NULL. */
int psf_ff_encode_async(psf_context* ctx, const void* d_values, size_t n, int value_type,
                        int num_bytes, const psf_fixed_point* preset, int32_t seed,
                        void* d_code, float* d_range, int32_t* d_status);

/* FIXING_FLOAT decode of n codes into n values, min/max from the received
 * FilterConfig (psf_ff_decode) or from device memory (psf_ff_decode_async). */
int psf_ff_decode(psf_context* ctx, const void* d_code, size_t n, int value_type,
                  int num_bytes, float min_value, float max_value, void* d_values);
int psf_ff_decode_async(psf_context* ctx, const void* d_code, size_t n, int value_type,
                        int num_bytes, const float* d_range, void* d_values);

/* CRC32C of d_data[0:bytes) -> *crc (host); synchronous. */
int psf_crc32c(psf_context* ctx, const void* d_data, size_t bytes, uint32_t* crc);
/* KEY_CACHING signature: CRC32C of the first min(bytes, 2048) key bytes. */
int psf_key_signature(psf_context* ctx, const void* d_keys, size_t bytes, uint32_t* sig);

/* COMPRESSING codec: the snappy raw format, byte-identical to snappy 1.1.8.
 * snappy::MaxCompressedLength(n) = 32 + n + n/6. */
size_t psf_snappy_max_compressed_length(size_t n);
/* snappy::RawCompress: d_out holds >= psf_snappy_max_compressed_length(n)
 * bytes; *out_len = stream length.  Synchronous.  n < 2^32. */
int psf_snappy_compress(psf_context* ctx, const void* d_in, size_t n, void* d_out, size_t* out_len);
/* snappy::GetUncompressedLength: PSF_ERR_CHECK when the header is malformed. */
/* COMPRESSING of a stream already in the stored layout -- varint32(n), then
 * per 64 KiB fragment snappy's literal tag and the fragment's bytes, what
 * 1.1.8 writes for data without matches (FIXING_FLOAT writes its codes so
 * when COMPRESSING follows it): on return d_buf holds RawCompress of the n
 * payload bytes (left in place when every fragment comes out stored,
 * rewritten in place when each fragment's start moves by at most 64 bytes,
 * else placed and copied back), *out_len its length.  The buffer holds cap >=
 * psf_snappy_stored_capacity(n) bytes (the stream can grow: a short match may
 * cost more than the literal it replaces).  Synchronous. */
int psf_snappy_compress_stored(psf_context* ctx, void* d_buf, size_t n, size_t cap, size_t* out_len);
size_t psf_snappy_stored_capacity(size_t n);
int psf_snappy_uncompressed_length(psf_context* ctx, const void* d_in, size_t n, size_t* out_len);
/* snappy::RawUncompress into d_out (out_cap >= the declared length, else
 * PSF_ERR_ARG); PSF_ERR_CHECK when RawUncompress would return false. */
int psf_snappy_uncompress(psf_context* ctx, const void* d_in, size_t n, void* d_out, size_t out_cap,
                          size_t* out_len);

/* ---- layer 2: messages and the filter chain ---------------------------- */
typedef struct psf_message psf_message;
typedef struct psf_node psf_node;

/* A RemoteNode: one filter instance per type, created on first use. */
int psf_node_create(psf_context* ctx, psf_node** out);
int psf_node_destroy(psf_node* node);
int psf_node_encode(psf_node* node, psf_message* msg);
int psf_node_decode(psf_node* node, psf_message* msg);

/* Task fields the filters read (task.proto:28-39; param.push = ParamCall). */
int psf_msg_create(int request, int has_param, int push, int32_t key_channel,
                   int has_key_range, uint64_t key_range_begin, uint64_t key_range_end,
                   psf_message** out);
int psf_msg_destroy(psf_message* msg);
/* Receiver-side copy: same Task (incl. all filter side-info) and the same
 * buffers (zero-copy), as the wire delivers it. */
int psf_msg_clone(const psf_message* msg, psf_message** out);

/* Attach caller memory (not copied, not freed; keep it alive while any
 * message or key cache refers to it).  loc = PSF_LOC_DEVICE / PSF_LOC_HOST. */
int psf_msg_set_key(psf_message* msg, void* ptr, size_t bytes, int key_type, int loc);
int psf_msg_add_value(psf_message* msg, void* ptr, size_t bytes, int value_type, int loc);
/* The Task frame of the wire (van.cc:122-191: [Task][key][value...]): the
 * fields the filter path reads and writes, protobuf wire format with the
 * reference's field numbers (task.proto, filter.proto).  serialize: buf = NULL
 * asks for the length; has_key is set from the key as Van::Send does.  parse:
 * a new message with that Task and no buffers (attach the key / value frames
 * with psf_msg_set_key / psf_msg_add_value); PSF_ERR_CHECK where protobuf's
 * ParseFromArray fails. */
int psf_task_serialize(const psf_message* msg, void* buf, size_t cap, size_t* len);
int psf_task_parse(const void* buf, size_t len, psf_message** out);
/* Van::Recv's data frames (van.cc:240-255): the first data frame of a message
 * whose Task has has_key becomes the key, every other frame is appended as a
 * value array; the Task (key_type, value_type, filters) is left as parsed. */
int psf_msg_recv_frame(psf_message* msg, void* ptr, size_t bytes, int loc);
/* Replace value array i by a caller buffer (e.g. a received frame, van.cc:244-255). */
int psf_msg_set_value(psf_message* msg, int i, void* ptr, size_t bytes, int loc);
int psf_msg_key(const psf_message* msg, void** ptr, size_t* bytes, int* loc);
/* task.key_channel and the number of task.value_type entries (a parsed Task's
 * value frames) */
int psf_msg_key_channel(const psf_message* msg, int32_t* key_channel);
int psf_task_value_count(const psf_message* msg, int* n);
int psf_msg_key_info(const psf_message* msg, int* has_key_flag, int* key_type);
int psf_msg_num_values(const psf_message* msg);
int psf_msg_value(const psf_message* msg, int i, void** ptr, size_t* bytes, int* loc);

/* FilterConfig access; `idx` is the position in task.filter. */
int psf_msg_add_filter(psf_message* msg, int type);  /* returns idx >= 0 or error */
int psf_fc_set_num_bytes(psf_message* msg, int idx, int num_bytes);
int psf_fc_set_clear_cache(psf_message* msg, int idx, int enable);
int psf_fc_set_noise(psf_message* msg, int idx, float mean, float std);
int psf_fc_add_fixed_point(psf_message* msg, int idx, const psf_fixed_point* fp);
int psf_fc_num_fixed_point(const psf_message* msg, int idx);
int psf_fc_fixed_point(const psf_message* msg, int idx, int k, psf_fixed_point* fp);
int psf_fc_signature(const psf_message* msg, int idx, int* has_signature, uint32_t* sig);
/* the signature a received FilterConfig carries (filter.proto:33), for a
 * decode fed from another wire format than psf_task_deserialize */
int psf_fc_set_signature(psf_message* msg, int idx, int has_signature, uint32_t sig);
int psf_fc_num_uncompressed(const psf_message* msg, int idx);
int psf_fc_uncompressed(const psf_message* msg, int idx, int i, uint64_t* size);
int psf_fc_add_uncompressed(psf_message* msg, int idx, uint64_t size);

/* ---- key-range partition and slicing (multi-server / multi-GPU split) --
 * Range<Key>::EvenDivide(n, i) (src/util/range.h:100-107): the i-th of n
 * server ranges of [begin, end), computed in long double as the reference. */
int psf_range_even_divide(uint64_t begin, uint64_t end, uint64_t n, uint64_t i,
                          uint64_t* out_begin, uint64_t* out_end);
/* SliceKOFVMessage<K> (src/system/message.h:107-147): split `msg` (sorted keys
 * of key_bytes = sizeof(K), 8 or 4) at the contiguous ranges
 * [bounds[i], bounds[i+1]), i < nranges.  outs[i] receives a new message
 * (the original Task, zero-copy key/value segments; free with
 * psf_msg_destroy) and valid[i] = 0 when range i misses the message's key
 * range (the reference does not send those).  Device keys: lower_bound runs
 * on the GPU. */
int psf_msg_slice(psf_context* ctx, const psf_message* msg, const uint64_t* bounds, int nranges,
                  int key_bytes, psf_message** outs, int* valid);

/* psf_msg_slice for nmsgs messages (outs / valid: nmsgs x nranges, row-major),
 * with one device synchronisation for all of them. */
int psf_msgs_slice(psf_context* ctx, const psf_message* const* msgs, int nmsgs, const uint64_t* bounds,
                   int nranges, int key_bytes, psf_message** outs, int* valid);

/* Message path driver (what Executor::Submit -> remote peer -> PickActiveMsg
 * does per message, executor.cc:131-146,178-219): for i in [0, iters), encode
 * a fresh copy of tmpls[i % ntmpl] on `snd`, deliver it (Task copy + zero-copy
 * buffers) and decode it on `rcv`.  The last decoded message is returned in
 * *out (may be NULL).  Used by bench.py so no Python runs per message. */
int psf_node_roundtrip(psf_node* snd, psf_node* rcv, const psf_message* const* tmpls, int ntmpl,
                       int iters, psf_message** out);
/* The same, also returning the last encoded message as it went on the wire
 * (*enc_out) next to the decoded one (*dec_out); either may be NULL. */
int psf_node_roundtrip_ex(psf_node* snd, psf_node* rcv, const psf_message* const* tmpls, int ntmpl,
                          int iters, psf_message** enc_out, psf_message** dec_out);

/* ---- server-side consumers ------------------------
 * What the receiving server does with a decoded message, fused with the
 * FIXING_FLOAT dequantise: psf_node_set_defer_dequant(server, 1) makes
 * FIXING_FLOAT's decode leave its codes pending (only where every filter
 * listed before it is KEY_CACHING, so nothing decoded later reads values);
 * the consumers below then dequantise in-register with ff_decode's exact
 * arithmetic (fixing_float.h:89-101) and never materialise the float array. */
int psf_node_set_defer_dequant(psf_node* node, int enable);
/* value i still holds FIXING_FLOAT codes: *num_bytes > 0 and the range, else 0 */
int psf_msg_pending(const psf_message* msg, int i, int* num_bytes, float* min_value, float* max_value);
/* run the pending dequantise(s) now (what DecodeMessage would have produced) */
int psf_msg_materialize(psf_context* ctx, psf_message* msg);

/* AssignOpType (src/util/proto/assign_op.proto:4-13), the float subset
 * AssignOp handles (src/util/assign_op.h:10-26) */
#define PSF_OP_ASSIGN 0
#define PSF_OP_PLUS 1
#define PSF_OP_MINUS 2
#define PSF_OP_TIMES 3
#define PSF_OP_DIVIDE 4

/* ParallelOrderedMatch (src/util/parallel_ordered_match.h:7-83): for every key
 * of the sorted d_src_key also in the sorted d_dst_key,
 * d_dst_val[j*k + i] op= d_src_val[s*k + i] (value_type FLOAT / DOUBLE); the
 * r-th copy of a repeated key pairs with the r-th copy in dst, as the
 * reference's two cursors do.  *n = matched keys * k (the reference's return
 * value).  d_dst_val must hold ndst*k values (the reference zero-fills an
 * empty one first, parallel_ordered_match.h:69-72).  Synchronous. */
int psf_ordered_match(psf_context* ctx, const uint64_t* d_src_key, size_t nsrc, const void* d_src_val,
                      const uint64_t* d_dst_key, size_t ndst, void* d_dst_val, int k, int value_type,
                      int op, size_t* n);
/* The same with the src values given as FIXING_FLOAT codes (num_bytes per
 * value, range [min_value, max_value]); value_type FLOAT. */
int psf_ff_decode_match(psf_context* ctx, const uint64_t* d_src_key, size_t nsrc, const void* d_code,
                        int num_bytes, float min_value, float max_value, const uint64_t* d_dst_key,
                        size_t ndst, void* d_dst_val, int k, int op, size_t* n);
/* KVVector::SetValue's merge of value array i of a received message
 * (src/parameter/kv_vector.h:182-183 / 205-207): src keys = the message's key;
 * a pending FIXING_FLOAT array is dequantised in-register. */
int psf_msg_ordered_match(psf_context* ctx, const psf_message* msg, int i, const uint64_t* d_dst_key,
                          size_t ndst, void* d_dst_val, int k, int value_type, int op, size_t* n);

/* KVMap<Key, float, FTRLEntry, SGDState> (src/parameter/kv_map.h:32-91,
 * src/app/linear_method/async_sgd.h:42-154): the async-SGD server's model as a
 * hash table in HBM (grows 2x on the device at load 1/2).  lr_type 1 CONSTANT /
 * 2 DECAY with alpha, beta (LearningRateConfig, linear.proto:93-101); penalty
 * ElasticNet(lambda1, lambda2) (penalty.h:41-91: L1 = (lambda[0], lambda[1] or
 * 0), L2 = (0, lambda[0])).  CHECKs of LearningRate / ElasticNet ->
 * PSF_ERR_CHECK.  `capacity` = expected number of keys (a hint). */
typedef struct psf_kvmap psf_kvmap;
int psf_kvmap_create(psf_context* ctx, size_t capacity, int lr_type, double alpha, double beta,
                     double lambda1, double lambda2, psf_kvmap** out);
int psf_kvmap_destroy(psf_kvmap* map);
/* KVMap::SetValue on a push message: FTRLEntry::Set for every key (pending
 * FIXING_FLOAT codes dequantised in-register).  Asynchronous; a failed
 * CHECK_GT(eta, 0) is reported by the next psf_kvmap_stats. */
int psf_kvmap_set_value(psf_kvmap* map, const psf_message* msg);
/* KVMap::GetValue on a pull message: appends the FLOAT array of w. */
int psf_kvmap_get_value(psf_kvmap* map, psf_message* msg);
/* raw device arrays */
int psf_kvmap_push(psf_kvmap* map, const uint64_t* d_keys, size_t n, const float* d_grad);
int psf_kvmap_pull(psf_kvmap* map, const uint64_t* d_keys, size_t n, float* d_w);
/* SGDState counters (async_sgd.h:106-125): nnz exactly; weight_sum and
 * delta_sum accumulated in double (the reference sums the same float terms
 * serially in float); size = stored keys.  Synchronous. */
int psf_kvmap_stats(psf_kvmap* map, int64_t* nnz, double* weight_sum, double* delta_sum,
                    uint64_t* size);

/* ---- many messages at once --------------------------------------------
 * RemoteNode::EncodeMessage / DecodeMessage of n messages, message i on
 * nodes[i]: every message runs its own chain in its own order on its own
 * node's filter instances (stateful filters see their messages in array
 * order), with FIXING_FLOAT's element work batched into one launch per kernel
 * for up to 64 arrays (the async-SGD minibatch messages and the per-server
 * slices of SURVEY.md §8(d) C1/C4 are latency-bound one at a time).
 * Computed FIXING_FLOAT min/max are not waited for: a decode of the message
 * on the same context reads them on the device, and any host reader
 * (psf_fc_fixed_point, psf_task_serialize, a decode elsewhere) resolves them
 * first -- CHECK_GT(bin, 0) is reported there, by psf_context_sync, or at the
 * end of psf_nodes_roundtrip, instead of at encode time. */
int psf_nodes_encode(psf_node* const* nodes, psf_message* const* msgs, int n);
int psf_nodes_decode(psf_node* const* nodes, psf_message* const* msgs, int n);
/* psf_node_roundtrip for n streams at once: for i in [0, iters), encode fresh
 * copies of tmpls[0..n) on snd[0..n), deliver, decode on rcv[0..n). */
int psf_nodes_roundtrip(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                        int iters);
/* ... in phases: messages [phase_end[p-1], phase_end[p]) are encoded, delivered
 * and decoded before phase p+1 starts (phase_end ascending, last = n; NULL =
 * one phase), so a request / response / push sequence runs in the
 * reference's order (the ctr example's pull request, pull response and push
 * of a minibatch, async_sgd.h:229-296); returning the last iteration's
 * encoded and decoded messages, message i in enc_out[i] / dec_out[i] (arrays
 * of n, or NULL). */
int psf_nodes_roundtrip_ex(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                           const int* phase_end, int nphases, int iters, psf_message** enc_out,
                           psf_message** dec_out);
/* The same with options: PSF_RT_WIRE serialises each encoded message's Task
 * frame (psf_task_serialize: the computed min/max settled to the host first,
 * as Van::Send does after EncodeMessage, van.cc:122-191) and decodes a
 * message parsed from it (psf_task_parse) with the data frames as they are
 * (Van::Recv's zero-copy frames, van.cc:244-269). */
#define PSF_RT_WIRE 1
int psf_nodes_roundtrip_opts(psf_node* const* snd, psf_node* const* rcv, const psf_message* const* tmpls, int n,
                             const int* phase_end, int nphases, int iters, int flags, psf_message** enc_out,
                             psf_message** dec_out);

/* ---- cross-range spill (multi-GPU split, one all-to-all-v per step) -----
 * Replaces the reference's per-server send loop (src/system/executor.cc:
 * 135-146), each slice one ZeroMQ multipart message [Task][key][value...]
 * (Van::Send src/system/van.cc:122-191, Van::Recv :193-269): every slice a rank
 * sends in a step is laid out in ONE send buffer, one segment per destination
 * rank, for a single all-to-all-v (RCCL over xGMI).  Segment = [meta][payload],
 * both multiples of 256 bytes: meta holds one record per message (server id,
 * the Task frame, frame lengths), payload the key / value frames at 256-byte
 * aligned offsets.
 *
 * psf_spill_pack: message i goes to rank dest[i], addressed to server
 * server[i]; sizes[2r] / sizes[2r+1] = meta / payload bytes of rank r's
 * segment (serialises the Tasks: resolves side-info a batched encode left on
 * the device).  psf_spill_fill writes the send buffer (sum of sizes bytes; HBM
 * on a device context) with one gather launch on the context's stream.
 * psf_spill_unpack rebuilds the received messages (segments of sources
 * 0..world-1 back to back, sizes_in as their senders reported them) over
 * recvbuf without copying the frames (keep recvbuf alive); servers[i] is the
 * server message i is addressed to; *n = message count (PSF_ERR_ARG when it
 * exceeds cap). */
typedef struct psf_spill psf_spill;
int psf_spill_pack(psf_context* ctx, psf_message* const* msgs, const int* dest, const int* server, int n,
                   int world, int64_t* sizes, psf_spill** out);
int psf_spill_fill(psf_spill* plan, void* sendbuf);
int psf_spill_destroy(psf_spill* plan);
int psf_spill_unpack(psf_context* ctx, const void* recvbuf, int world, const int64_t* sizes_in,
                     psf_message** outs, int* servers, int cap, int* n);

/* ---- the multi-server push path of one rank -----------------------------
 * What Executor::Submit does for a push to the server group
 * (src/system/executor.cc:127-146: SliceKOFVMessage at the server key ranges,
 * src/system/message.h:107-147, then EncodeMessage on the per-peer
 * RemoteNode) and what each server's executor does with what arrives
 * (DecodeMessage, executor.cc:178-219), for many push streams at once:
 * S servers with the contiguous key ranges [bounds[s], bounds[s+1]), server s
 * hosted by rank s * world / S; one sender node per (stream key_channel,
 * server), one receiver node per (server, stream).  loopback = 1 sends the
 * local slices through the exchange as well.
 *
 * A step: psf_router_encode (slice + encode every stream's template, copied
 * as the executor copies the Task; pack the slices for other ranks: sizes as
 * psf_spill_pack), psf_router_fill (the send buffer), the caller's
 * all-to-all-v, psf_router_decode_local / psf_router_decode_received (the
 * receive buffer is copied into library-owned memory: KEY_CACHING keeps
 * received keys by reference).  psf_router_step runs `iters` whole steps of a
 * world-1 router, or of any router with a native exchange
 * (psf_router_set_exchange, below).  Results of the last step: the decoded
 * messages with their server (psf_router_result), and with
 * psf_router_keep_encoded(1) the encoded slices (psf_router_encoded); both
 * return new message handles. */
typedef struct psf_router psf_router;
int psf_router_create(psf_context* ctx, const uint64_t* bounds, int nservers, int rank, int world, int loopback,
                      psf_router** out);
int psf_router_destroy(psf_router* r);
int psf_router_keep_encoded(psf_router* r, int enable);
int psf_router_encode(psf_router* r, psf_message* const* streams, int n, int64_t* sizes);
int psf_router_fill(psf_router* r, void* sendbuf);
int psf_router_decode_local(psf_router* r);
int psf_router_decode_received(psf_router* r, const void* recvbuf, const int64_t* sizes_in);
int psf_router_step(psf_router* r, psf_message* const* streams, int n, int iters);
int psf_router_num_results(psf_router* r);
int psf_router_result(psf_router* r, int i, int* server, psf_message** out);
int psf_router_num_encoded(psf_router* r);
int psf_router_encoded(psf_router* r, int i, int32_t* stream, int* server, psf_message** out);

/* ---- the native exchange of the ranks of one node ------------------------
 * Replaces the reference's per-server send loop (executor.cc:131-146 ->
 * Van::Send / Recv, van.cc:122-269) between the servers of one node: each
 * slice's Task frame (serialised on the host, as Van::Send does) travels
 * through a host shared-memory mailbox of the node's ranks, its data frames
 * device to device -- PSF_EXCHANGE_RCCL: RCCL point-to-point over xGMI, one
 * grouped send/recv per peer per step on the exchange's stream (librccl is
 * loaded on first use); PSF_EXCHANGE_HOST: through the mailbox (several ranks
 * on one GPU, or host-only contexts).  FIXING_FLOAT ranges computed on the
 * device travel on the device too, so a step needs no device->host wait
 * except COMPRESSING's output lengths.
 *
 * psf_exchange_unique_id: rank 0's RCCL id (bytes >= 128), handed to every
 * rank by the caller.  psf_exchange_create: every rank of the node, same
 * `name` (a file name; the mailbox lives in PSF_EXCHANGE_DIR, /dev/shm or
 * TMPDIR), same caps (meta_cap: Task-record bytes a rank posts per step, 0 =
 * 1 MiB; host_cap: data bytes per step for PSF_EXCHANGE_HOST, 0 = 64 MiB);
 * returns when every rank has attached.  Waits are bounded by
 * PSF_EXCHANGE_TIMEOUT_S (default 120 s).  psf_router_set_exchange: the
 * router's psf_router_step then runs at any world size (and with loopback),
 * one call for `iters` whole steps.  psf_exchange_stats: out[3] = {bytes
 * posted for other ranks (records + data), steps, host ns waiting on the
 * mailbox}. */
#define PSF_EXCHANGE_RCCL 0
#define PSF_EXCHANGE_HOST 1
typedef struct psf_exchange psf_exchange;
int psf_exchange_unique_id(void* out, size_t bytes);
int psf_exchange_create(psf_context* ctx, int rank, int world, const char* name, int transport, const void* nccl_id,
                        uint64_t meta_cap, uint64_t host_cap, psf_exchange** out);
int psf_exchange_destroy(psf_exchange* ex);
int psf_exchange_stats(psf_exchange* ex, int64_t* out);
/* out[4] = {data bytes handed to ncclSend, ncclSend calls, data bytes copied
 * by the runtime instead (the self slice; PSF_EXCHANGE_HOST: the mailbox
 * copies), 1 if a step failed on this rank (every later call fails at once,
 * and so do the peers' waits)} */
int psf_exchange_data_stats(psf_exchange* ex, int64_t* out);
/* the router keeps a reference: the exchange may be destroyed first */
int psf_router_set_exchange(psf_router* r, psf_exchange* ex);

/* ---- the pull leg of the partition (CS-2) --------------------------------
 * A pull of every stream's keys from the server group, answered per server
 * range and merged back into key order -- Executor::Submit of the request
 * (executor.cc:108-147), Parameter::ProcessRequest on each server
 * (parameter.cc:5-31: the response is a copy of the request and
 * KVMap::GetValue appends the values, kv_map.h:69-77), Executor::Reply
 * (executor.cc:150-167: task.request = false, encoded on the server's node
 * for the requester), and KVVector::SetValue on the requester
 * (kv_vector.h:129-212: the response's values matched into the stream's
 * zeroed key-ordered array).  Each request template has task.request = 1,
 * param.push = 0, UINT64 keys, no values, and its own key_channel.
 * psf_router_set_store: the KV map of this rank's servers (the router keeps
 * a reference).  psf_router_pull: `iters` whole pulls (native exchange, or a
 * world-1 router).  A caller-driven exchange instead runs
 * psf_router_pull_encode -> psf_router_fill -> all-to-all-v ->
 * psf_router_pull_serve -> psf_router_fill -> all-to-all-v ->
 * psf_router_pull_finish (sizes as psf_router_encode's).  Results: per
 * request stream, a message with its keys and one FLOAT value array in key
 * order (psf_router_pulled; a new handle), until the next pull.  With
 * psf_router_keep_encoded(1), psf_router_encoded lists the encoded requests
 * this rank sent and the encoded responses its servers sent
 * (task.request tells them apart). */
int psf_router_set_store(psf_router* r, psf_kvmap* store);
int psf_router_pull(psf_router* r, psf_message* const* requests, int n, int iters);
int psf_router_pull_encode(psf_router* r, psf_message* const* requests, int n, int64_t* sizes);
int psf_router_pull_serve(psf_router* r, const void* recvbuf, const int64_t* sizes_in, int64_t* sizes);
int psf_router_pull_finish(psf_router* r, const void* recvbuf, const int64_t* sizes_in);
int psf_router_num_pulled(psf_router* r);
int psf_router_pulled(psf_router* r, int i, int32_t* stream, psf_message** out);

/* ---- host-side accounting ----------------------------------------------
 * Host time blocked on the device, by cause: PSF_WAIT_SYNC stream
 * synchronisations, PSF_WAIT_PUBLISH waits on side-info a kernel publishes
 * (KEY_CACHING CRCs, FIXING_FLOAT ranges, snappy sizes), PSF_WAIT_SLICE waits
 * on the slicing pass.  wait_ns and waits hold PSF_WAIT_NUM entries. */
#define PSF_WAIT_SYNC 0
#define PSF_WAIT_PUBLISH 1
#define PSF_WAIT_SLICE 2
#define PSF_WAIT_NUM 3
int psf_context_host_stats(psf_context* ctx, int64_t* wait_ns, int64_t* waits);
int psf_context_host_stats_reset(psf_context* ctx);
/* The caching allocator: released codec buffers are kept for reuse on free
 * lists bounded per DEVICE -- one cap shared by every context on the device
 * (default 8 GiB of HBM, 1 GiB of pinned host memory); a release past the cap
 * frees the least recently released blocks of the whole device first, and an
 * allocation that fails drops every cached block of the device and retries.
 * psf_context_set_cache_limit sets the cap of the context's device (=
 * psf_set_device_cache_limit).  psf_context_memory_stats: out[8] = {HBM
 * cached, HBM cap, HBM allocated (live + cached), HBM evictions, pinned
 * cached, pinned cap, pinned allocated, pinned evictions} of the context's
 * stream (shared by the contexts on a shared stream); caps per device.
 * psf_device_memory_stats: out[10] = the same 8 for the whole device, then
 * the live streams with a cache share and the shared streams created. */
int psf_context_set_cache_limit(psf_context* ctx, uint64_t hbm_bytes, uint64_t pinned_bytes);
int psf_context_memory_stats(psf_context* ctx, uint64_t* out);
int psf_set_device_cache_limit(int device, uint64_t hbm_bytes, uint64_t pinned_bytes);
int psf_device_memory_stats(int device, uint64_t* out);
/* router phase timers: out[0] steps (encodes), out[1] host ns inside encode,
 * out[2] host ns inside the decodes (both include the waits above) */
int psf_router_host_stats(psf_router* r, int64_t* out);
int psf_router_host_stats_reset(psf_router* r);

/* ---- launch profiler (HIP events on the launch stream) ----------------- */
#define PSF_K_MINMAX 0
#define PSF_K_ENCODE 1
#define PSF_K_DECODE 2
#define PSF_K_CRC32C 3
#define PSF_K_NOISE 4
#define PSF_K_SNAPPY_COMPRESS 5
#define PSF_K_SNAPPY_DECOMPRESS 6
#define PSF_K_MATCH 7
#define PSF_K_KV_PUSH 8
#define PSF_K_KV_GET 9
#define PSF_K_NUM 10
/* kernel_mask: bit k times kernel PSF_K_k (-1 = all, 0 = off) */
int psf_profile_enable(psf_context* ctx, int kernel_mask);
/* time only every stride-th launch of each profiled kernel (1 = every launch;
 * resets the launch counts): keeps the event pairs from dominating a step of
 * many short kernels */
int psf_profile_stride(psf_context* ctx, int stride);
int psf_profile_reset(psf_context* ctx);
/* launches, summed kernel milliseconds and summed algorithmic HBM bytes */
int psf_profile_read(psf_context* ctx, int kernel, int64_t* launches, double* total_ms,
                     double* alg_bytes);
const char* psf_profile_kernel_name(int kernel);

#ifdef __cplusplus
}
#endif
#endif /* PSF_H_ */
