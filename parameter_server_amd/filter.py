"""Python face of the filter plugin surface (thin ctypes wrappers over
include/psf.h; all codec work runs in libpsf's HIP kernels).

Mirrors the reference's objects so tests read like its own:

* ``Context``     -- device + HIP stream (+ workspace) the kernels run on
* ``RemoteNode``  -- RemoteNode::EncodeMessage / DecodeMessage (remote_node.cc:17-29)
* ``Message``     -- Message/Task/FilterConfig fields (message.h:10-76,
                     task.proto:28-39, filter.proto:3-35)

Buffers are torch tensors on the context's device (or CPU tensors for the host
edge).  Messages keep the tensors they reference alive; nodes keep alive every
tensor a key cache may refer to.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from ._lib import (DT_DOUBLE, DT_FLOAT, DT_UINT64, LOC_DEVICE, LOC_HOST, FixedPoint, PsfError,  # noqa: F401
                   check, lib)

_TORCH_DT = {DT_FLOAT: torch.float32, DT_DOUBLE: torch.float64}


def dtype_code(t: torch.Tensor) -> int:
    return {torch.float32: DT_FLOAT, torch.float64: DT_DOUBLE, torch.int64: DT_UINT64,
            torch.uint8: 11}.get(t.dtype, 0)


def set_clock(t: Optional[int]) -> None:
    """Pin the FIXING_FLOAT seed source (time(NULL) in the reference)."""
    lib().psf_set_clock(0 if t is None else 1, 0 if t is None else int(t))


def device_memory_stats(device: int = 0) -> dict:
    """The device-wide caching allocator (every context on `device`): bytes
    cached / cap / allocated and evictions for HBM ("hbm_*") and pinned host
    memory ("pinned_*"), the live streams with a cache share and the shared
    streams created (psf_device_memory_stats)."""
    out = (C.c_uint64 * 10)()
    check(lib().psf_device_memory_stats(device, out))
    keys = ("cached", "cap", "allocated", "evictions")
    return {**{f"hbm_{k}": out[i] for i, k in enumerate(keys)},
            **{f"pinned_{k}": out[4 + i] for i, k in enumerate(keys)},
            "streams": out[8], "shared_streams": out[9]}


def set_device_cache_limit(device: int, hbm_bytes: int, pinned_bytes: int) -> None:
    check(lib().psf_set_device_cache_limit(device, hbm_bytes, pinned_bytes))


DEFAULT_CACHE_LIMIT = (8 << 30, 1 << 30)  # Context::kDefaultCache*Bytes


class Context:
    def __init__(self, device: int = 0, stream: Optional[torch.cuda.Stream] = None):
        self.device = device
        self.stream = stream if stream is not None else torch.cuda.current_stream(device)
        h = C.c_void_p()
        check(lib().psf_context_create(device, C.c_void_p(self.stream.cuda_stream), 0, C.byref(h)))
        self.h = h

    def sync(self):
        check(lib().psf_context_sync(self.h))

    # -- launch profiler -----------------------------------------------------
    def profile(self, on: bool = True, kernels=None, stride: int = 1):
        """Time kernel launches with HIP events: all kernels, or only `kernels`
        (names from _lib.KERNELS); every `stride`-th launch of each."""
        from ._lib import KERNELS
        mask = 0 if not on else (-1 if kernels is None else
                                 sum(1 << KERNELS.index(k) for k in kernels))
        check(lib().psf_profile_enable(self.h, mask))
        check(lib().psf_profile_stride(self.h, stride))

    def profile_reset(self):
        check(lib().psf_profile_reset(self.h))

    def profile_read(self) -> dict:
        """{kernel: (launches, total_ms, algorithmic_bytes)} for launched kernels."""
        from ._lib import KERNELS
        out = {}
        for k, name in enumerate(KERNELS):
            n, ms, b = C.c_int64(), C.c_double(), C.c_double()
            check(lib().psf_profile_read(self.h, k, C.byref(n), C.byref(ms), C.byref(b)))
            if n.value:
                out[name] = (n.value, ms.value, b.value)
        return out

    def host_waits(self, reset: bool = False) -> dict:
        """Host time blocked on the device since the last reset, by cause:
        {"sync" | "publish" | "slice": (seconds, count)}."""
        ns, cnt = (C.c_int64 * 3)(), (C.c_int64 * 3)()
        check(lib().psf_context_host_stats(self.h, ns, cnt))
        if reset:
            check(lib().psf_context_host_stats_reset(self.h))
        return {k: (ns[i] / 1e9, cnt[i]) for i, k in enumerate(("sync", "publish", "slice"))}

    def set_cache_limit(self, hbm_bytes: int, pinned_bytes: int) -> None:
        check(lib().psf_context_set_cache_limit(self.h, hbm_bytes, pinned_bytes))

    def memory_stats(self) -> dict:
        """This context's share of the device's caching allocator: bytes cached
        / allocated and evictions, for HBM ("hbm_*") and pinned host memory
        ("pinned_*"); the caps ("*_cap") are the device's."""
        out = (C.c_uint64 * 8)()
        check(lib().psf_context_memory_stats(self.h, out))
        keys = ("cached", "cap", "allocated", "evictions")
        return {**{f"hbm_{k}": out[i] for i, k in enumerate(keys)},
                **{f"pinned_{k}": out[4 + i] for i, k in enumerate(keys)}}

    def close(self):
        if self.h:
            lib().psf_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- layer 1 kernels -----------------------------------------------------
    def ff_encode(self, x: torch.Tensor, nb: int, seed: int, mn=None, mx=None, out=None):
        """FIXING_FLOAT encode; returns (codes uint8 tensor, min, max)."""
        fp = FixedPoint(mn is not None, mx is not None, 0.0 if mn is None else mn,
                        0.0 if mx is None else mx)
        if out is None:
            out = torch.empty(x.numel() * nb, dtype=torch.uint8, device=x.device)
        check(lib().psf_ff_encode(self.h, C.c_void_p(x.data_ptr()), x.numel(), dtype_code(x), nb,
                                  C.byref(fp), C.c_int32(seed), C.c_void_p(out.data_ptr())))
        return out, fp.min_value, fp.max_value

    def ff_encode_async(self, x, nb, seed, out, d_range, d_status=None, mn=None, mx=None):
        fp = FixedPoint(mn is not None, mx is not None, 0.0 if mn is None else mn,
                        0.0 if mx is None else mx)
        check(lib().psf_ff_encode_async(self.h, C.c_void_p(x.data_ptr()), x.numel(), dtype_code(x), nb,
                                        C.byref(fp), C.c_int32(seed), C.c_void_p(out.data_ptr()),
                                        C.c_void_p(d_range.data_ptr()),
                                        None if d_status is None else C.c_void_p(d_status.data_ptr())))

    def ff_decode(self, code: torch.Tensor, nb: int, mn: float, mx: float, dtype=torch.float32, out=None):
        n = code.numel() // nb
        if out is None:
            out = torch.empty(n, dtype=dtype, device=code.device)
        check(lib().psf_ff_decode(self.h, C.c_void_p(code.data_ptr()), n, dtype_code(out), nb, mn, mx,
                                  C.c_void_p(out.data_ptr())))
        return out

    def ff_decode_async(self, code, nb, d_range, out):
        n = code.numel() // nb
        check(lib().psf_ff_decode_async(self.h, C.c_void_p(code.data_ptr()), n, dtype_code(out), nb,
                                        C.c_void_p(d_range.data_ptr()), C.c_void_p(out.data_ptr())))
        return out

    def crc32c(self, t: torch.Tensor, nbytes: Optional[int] = None) -> int:
        v = C.c_uint32()
        nb = t.numel() * t.element_size() if nbytes is None else nbytes
        check(lib().psf_crc32c(self.h, C.c_void_p(t.data_ptr()), nb, C.byref(v)))
        return v.value

    def key_signature(self, t: torch.Tensor) -> int:
        v = C.c_uint32()
        check(lib().psf_key_signature(self.h, C.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                      C.byref(v)))
        return v.value

    # -- COMPRESSING codec (snappy 1.1.8 raw format) ------------------------
    def snappy_compress(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """snappy::RawCompress of t's bytes -> uint8 tensor (a view of `out`)."""
        n = t.numel() * t.element_size()
        cap = lib().psf_snappy_max_compressed_length(n)
        if out is None:
            out = torch.empty(cap, dtype=torch.uint8, device=t.device)
        assert out.numel() >= cap
        ln = C.c_size_t()
        check(lib().psf_snappy_compress(self.h, C.c_void_p(t.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                        C.byref(ln)))
        return out[:ln.value]

    def snappy_uncompress(self, s: torch.Tensor) -> torch.Tensor:
        """snappy::RawUncompress -> uint8 tensor; PsfError(PSF_ERR_CHECK) on a bad stream."""
        n = s.numel() * s.element_size()
        ln = C.c_size_t()
        check(lib().psf_snappy_uncompressed_length(self.h, C.c_void_p(s.data_ptr()), n, C.byref(ln)))
        out = torch.empty(max(ln.value, 1), dtype=torch.uint8, device=s.device)
        check(lib().psf_snappy_uncompress(self.h, C.c_void_p(s.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                          out.numel(), C.byref(ln)))
        return out[:ln.value]


    # -- server-side consumers ---------------------------
    def ordered_match(self, src_key, src_val, dst_key, dst_val, k=1, op=0) -> int:
        """ParallelOrderedMatch: dst_val op= src_val on equal keys; returns *n."""
        n = C.c_size_t()
        check(lib().psf_ordered_match(self.h, C.c_void_p(src_key.data_ptr()), src_key.numel(),
                                      C.c_void_p(src_val.data_ptr()), C.c_void_p(dst_key.data_ptr()),
                                      dst_key.numel(), C.c_void_p(dst_val.data_ptr()), k,
                                      dtype_code(dst_val), op, C.byref(n)))
        return n.value

    def ff_decode_match(self, src_key, codes, nb, mn, mx, dst_key, dst_val, k=1, op=0) -> int:
        """ordered_match with FIXING_FLOAT codes as the source (dequantised in-register)."""
        n = C.c_size_t()
        check(lib().psf_ff_decode_match(self.h, C.c_void_p(src_key.data_ptr()), src_key.numel(),
                                        C.c_void_p(codes.data_ptr()), nb, mn, mx,
                                        C.c_void_p(dst_key.data_ptr()), dst_key.numel(),
                                        C.c_void_p(dst_val.data_ptr()), k, op, C.byref(n)))
        return n.value


class KVMap:
    """KVMap<Key, float, FTRLEntry, SGDState> in HBM (kv_map.h:32-91,
    async_sgd.h:42-154)."""

    def __init__(self, ctx: Context, capacity=1 << 20, lr_type=2, alpha=0.01, beta=10.0, lambda1=0.0,
                 lambda2=0.0):
        self.ctx = ctx
        h = C.c_void_p()
        check(lib().psf_kvmap_create(ctx.h, capacity, lr_type, alpha, beta, lambda1, lambda2, C.byref(h)))
        self.h = h
        self._keepalive = []

    def __del__(self):
        try:
            if self.h:
                lib().psf_kvmap_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def set_value(self, msg: "Message"):
        self._keepalive.append(msg._refs)
        check(lib().psf_kvmap_set_value(self.h, msg.h))

    def get_value(self, msg: "Message"):
        check(lib().psf_kvmap_get_value(self.h, msg.h))

    def push(self, keys: torch.Tensor, grad: torch.Tensor):
        check(lib().psf_kvmap_push(self.h, C.c_void_p(keys.data_ptr()), keys.numel(),
                                   C.c_void_p(grad.data_ptr())))

    def pull(self, keys: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(keys.numel(), dtype=torch.float32, device=keys.device)
        check(lib().psf_kvmap_pull(self.h, C.c_void_p(keys.data_ptr()), keys.numel(),
                                   C.c_void_p(out.data_ptr())))
        return out

    def stats(self):
        """(nnz, weight_sum, delta_sum, size)"""
        a, b, c, d = C.c_int64(), C.c_double(), C.c_double(), C.c_uint64()
        check(lib().psf_kvmap_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return a.value, b.value, c.value, d.value


class HostContext(Context):
    """Host-only context (device -1): host-resident buffers, no HIP calls.
    KEY_CACHING on host keys runs here; codecs needing HBM report an error."""

    def __init__(self):
        self.device = -1
        self.stream = None
        h = C.c_void_p()
        check(lib().psf_context_create(-1, None, 0, C.byref(h)))
        self.h = h


class Message:
    def __init__(self, request=True, push=False, has_param=True, key_channel=0, key_range=None,
                 _handle=None, _refs=None):
        if _handle is not None:
            self.h = _handle
            self._refs = list(_refs or [])
            return
        h = C.c_void_p()
        kr = key_range
        check(lib().psf_msg_create(int(request), int(has_param), int(push), int(key_channel),
                                   int(kr is not None), 0 if kr is None else kr[0],
                                   0 if kr is None else kr[1], C.byref(h)))
        self.h = h
        self._refs = []

    def __del__(self):
        try:
            if self.h:
                lib().psf_msg_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def clone(self) -> "Message":
        """Receiver-side copy (Task + zero-copy buffers), as delivered by the wire."""
        h = C.c_void_p()
        check(lib().psf_msg_clone(self.h, C.byref(h)))
        return Message(_handle=h, _refs=self._refs)

    # -- wire (van.cc:122-269) ------------------------------------------------
    def task_bytes(self) -> bytes:
        """The Task frame: protobuf wire format, the reference's field numbers."""
        n = C.c_size_t()
        check(lib().psf_task_serialize(self.h, None, 0, C.byref(n)))
        buf = (C.c_uint8 * max(n.value, 1))()
        check(lib().psf_task_serialize(self.h, buf, n.value, C.byref(n)))
        return bytes(buf[:n.value])

    @classmethod
    def from_task_bytes(cls, b: bytes) -> "Message":
        """A received message: the parsed Task, no key/value frames yet."""
        h = C.c_void_p()
        raw = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b + b"\0")
        check(lib().psf_task_parse(raw, len(b), C.byref(h)))
        return cls(_handle=h)

    def frames(self, device=None):
        """[Task][key][value...] as Van::Send emits them (van.cc:122-191); the
        key frame only when the key is non-empty.  Buffers are copied to host."""
        out = [self.task_bytes()]
        p, n, loc = self.key_ptr()
        arrays = ([(p, n, loc)] if n else []) + [self.value_ptr(i) for i in range(self.num_values())]
        for p, n, loc in arrays:
            out.append(copy_out(p, n, loc, device).cpu().numpy().tobytes() if n else b"")
        return out

    def recv_frame(self, t: torch.Tensor):
        """Attach a received data frame as Van::Recv does (van.cc:240-255)."""
        t = t.contiguous()
        self._refs.append(t)
        check(lib().psf_msg_recv_frame(self.h, C.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                       self._loc(t)))

    @staticmethod
    def _loc(t: torch.Tensor) -> int:
        return LOC_DEVICE if t.is_cuda else LOC_HOST

    def set_key(self, keys: torch.Tensor, key_type: int = DT_UINT64):
        keys = keys.contiguous()
        self._refs.append(keys)
        check(lib().psf_msg_set_key(self.h, C.c_void_p(keys.data_ptr()), keys.numel() * keys.element_size(),
                                    key_type, self._loc(keys)))

    def add_value(self, v: torch.Tensor, value_type: Optional[int] = None):
        v = v.contiguous()
        self._refs.append(v)
        vt = dtype_code(v) if value_type is None else value_type
        check(lib().psf_msg_add_value(self.h, C.c_void_p(v.data_ptr()), v.numel() * v.element_size(),
                                      vt, self._loc(v)))

    def add_filter(self, type_: int, num_bytes=None, clear_cache_if_done=None, fixed_point=None,
                   noise=None) -> int:
        idx = check(lib().psf_msg_add_filter(self.h, type_))
        if num_bytes is not None:
            check(lib().psf_fc_set_num_bytes(self.h, idx, num_bytes))
        if clear_cache_if_done is not None:
            check(lib().psf_fc_set_clear_cache(self.h, idx, int(clear_cache_if_done)))
        if noise is not None:
            check(lib().psf_fc_set_noise(self.h, idx, noise[0], noise[1]))
        for fp in fixed_point or []:
            mn, mx = fp
            f = FixedPoint(mn is not None, mx is not None, 0.0 if mn is None else mn,
                           0.0 if mx is None else mx)
            check(lib().psf_fc_add_fixed_point(self.h, idx, C.byref(f)))
        return idx

    # -- inspection --------------------------------------------------------
    def key_ptr(self):
        p, n, loc = C.c_void_p(), C.c_size_t(), C.c_int()
        check(lib().psf_msg_key(self.h, C.byref(p), C.byref(n), C.byref(loc)))
        return p.value, n.value, loc.value

    def key_info(self):
        hk, kt = C.c_int(), C.c_int()
        check(lib().psf_msg_key_info(self.h, C.byref(hk), C.byref(kt)))
        return bool(hk.value), kt.value

    def num_values(self) -> int:
        return check(lib().psf_msg_num_values(self.h))

    def value_ptr(self, i: int):
        p, n, loc = C.c_void_p(), C.c_size_t(), C.c_int()
        check(lib().psf_msg_value(self.h, i, C.byref(p), C.byref(n), C.byref(loc)))
        return p.value, n.value, loc.value

    def fixed_points(self, idx: int):
        out = []
        for k in range(check(lib().psf_fc_num_fixed_point(self.h, idx))):
            f = FixedPoint()
            check(lib().psf_fc_fixed_point(self.h, idx, k, C.byref(f)))
            out.append((bool(f.has_min), f.min_value, bool(f.has_max), f.max_value))
        return out

    def signature(self, idx: int):
        h, s = C.c_int(), C.c_uint32()
        check(lib().psf_fc_signature(self.h, idx, C.byref(h), C.byref(s)))
        return bool(h.value), s.value

    def pending(self, i: int):
        """(num_bytes, min, max) of a value array left FIXING_FLOAT-encoded by a
        deferred decode, or None."""
        nb, mn, mx = C.c_int(), C.c_float(), C.c_float()
        check(lib().psf_msg_pending(self.h, i, C.byref(nb), C.byref(mn), C.byref(mx)))
        return (nb.value, mn.value, mx.value) if nb.value else None

    def materialize(self, ctx: Context):
        check(lib().psf_msg_materialize(ctx.h, self.h))

    def ordered_match(self, ctx: Context, i: int, dst_key, dst_val, k=1, op=0) -> int:
        """KVVector::SetValue's merge of value array i into (dst_key, dst_val)."""
        n = C.c_size_t()
        check(lib().psf_msg_ordered_match(ctx.h, self.h, i, C.c_void_p(dst_key.data_ptr()), dst_key.numel(),
                                          C.c_void_p(dst_val.data_ptr()), k, dtype_code(dst_val), op,
                                          C.byref(n)))
        return n.value

    def uncompressed_sizes(self, idx: int):
        out = []
        for i in range(check(lib().psf_fc_num_uncompressed(self.h, idx))):
            v = C.c_uint64()
            check(lib().psf_fc_uncompressed(self.h, idx, i, C.byref(v)))
            out.append(v.value)
        return out


def copy_out(ptr: int, nbytes: int, loc: int, device) -> torch.Tensor:
    """Copy a library-owned buffer into a fresh uint8 tensor (same device)."""
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8, device=device if loc == LOC_DEVICE else "cpu")
    if loc == LOC_HOST:
        buf = (C.c_uint8 * nbytes).from_address(ptr)
        return torch.frombuffer(bytearray(buf), dtype=torch.uint8)
    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    _memcpy_d2d(out.data_ptr(), ptr, nbytes)
    return out


_hip = None


def _memcpy_d2d(dst: int, src: int, n: int):
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemcpyAsync.restype = C.c_int
    stream = torch.cuda.current_stream()
    rc = _hip.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), n, 3, C.c_void_p(stream.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed: {rc}")


class RemoteNode:
    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        check(lib().psf_node_create(ctx.h, C.byref(h)))
        self.h = h
        self._keepalive = {}

    def __del__(self):
        try:
            if self.h:
                lib().psf_node_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def _hold(self, msg: Message):
        for t in msg._refs:
            self._keepalive[id(t)] = t

    def roundtrip(self, rcv: "RemoteNode", tmpls, iters: int, keep_last: bool = False):
        """Native loop: encode a copy of tmpls[i % len] here, deliver, decode on
        rcv.  keep_last: return the last (encoded, decoded) message pair."""
        tmpls = tmpls if isinstance(tmpls, (list, tuple)) else [tmpls]
        for t in tmpls:
            self._hold(t)
            rcv._hold(t)
        arr = (C.c_void_p * len(tmpls))(*[t.h.value for t in tmpls])
        enc, dec = C.c_void_p(), C.c_void_p()
        check(lib().psf_node_roundtrip_ex(self.h, rcv.h, arr, len(tmpls), iters,
                                          C.byref(enc) if keep_last else None,
                                          C.byref(dec) if keep_last else None))
        if not keep_last:
            return None
        refs = tmpls[(iters - 1) % len(tmpls)]._refs
        return Message(_handle=enc, _refs=refs), Message(_handle=dec, _refs=refs)

    def set_defer_dequant(self, on: bool = True) -> None:
        """Server side: FIXING_FLOAT decode leaves codes for the consumer."""
        check(lib().psf_node_set_defer_dequant(self.h, int(on)))

    @staticmethod
    def encode_many(nodes, msgs) -> None:
        """psf_nodes_encode: msgs[i] through nodes[i]'s chain, FIXING_FLOAT batched."""
        for nd, m in zip(nodes, msgs):
            nd._hold(m)
        n = len(msgs)
        check(lib().psf_nodes_encode((C.c_void_p * n)(*[nd.h.value for nd in nodes]),
                                     (C.c_void_p * n)(*[m.h.value for m in msgs]), n))

    @staticmethod
    def decode_many(nodes, msgs) -> None:
        for nd, m in zip(nodes, msgs):
            nd._hold(m)
        n = len(msgs)
        check(lib().psf_nodes_decode((C.c_void_p * n)(*[nd.h.value for nd in nodes]),
                                     (C.c_void_p * n)(*[m.h.value for m in msgs]), n))

    @staticmethod
    def roundtrip_many(snd, rcv, tmpls, iters: int, keep_last: bool = False, phase_end=None, wire: bool = False):
        """psf_nodes_roundtrip_opts: message i encoded on snd[i], decoded on
        rcv[i]; phase_end splits the messages into batches run in order.
        keep_last: return the last iteration's [(encoded, decoded)] per message.
        wire: the receiver decodes a message parsed from the serialised Task
        (side-info settled per phase, as Van::Send after EncodeMessage)."""
        n = len(tmpls)
        for a, b, t in zip(snd, rcv, tmpls):
            a._hold(t)
            b._hold(t)
        enc, dec = (C.c_void_p * n)(), (C.c_void_p * n)()
        pe = None if not phase_end else (C.c_int * len(phase_end))(*phase_end)
        check(lib().psf_nodes_roundtrip_opts((C.c_void_p * n)(*[nd.h.value for nd in snd]),
                                             (C.c_void_p * n)(*[nd.h.value for nd in rcv]),
                                             (C.c_void_p * n)(*[t.h.value for t in tmpls]), n, pe,
                                             len(phase_end or ()), iters, 1 if wire else 0,
                                             enc if keep_last else None, dec if keep_last else None))
        if not keep_last:
            return None
        return [(Message(_handle=C.c_void_p(enc[i]), _refs=tmpls[i]._refs),
                 Message(_handle=C.c_void_p(dec[i]), _refs=tmpls[i]._refs)) for i in range(n)]

    def encode(self, msg: Message) -> None:
        self._hold(msg)
        check(lib().psf_node_encode(self.h, msg.h))

    def decode(self, msg: Message) -> None:
        self._hold(msg)
        check(lib().psf_node_decode(self.h, msg.h))

    # convenience: copy results out
    def key(self, msg: Message) -> torch.Tensor:
        p, n, loc = msg.key_ptr()
        self.ctx.sync()
        return copy_out(p, n, loc, f"cuda:{self.ctx.device}")

    def value(self, msg: Message, i: int) -> torch.Tensor:
        p, n, loc = msg.value_ptr(i)
        self.ctx.sync()
        return copy_out(p, n, loc, f"cuda:{self.ctx.device}")
