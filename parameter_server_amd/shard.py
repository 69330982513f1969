"""The multi-GPU split of the filter path.

Server s owns Range<Key>(key_start, key_end).EvenDivide(S, s)
(src/system/assigner.h:17-28, src/util/range.h:100-107); servers live on ranks
in contiguous blocks (rank r hosts servers [r*S/W, (r+1)*S/W), one server per
GPU when S == W).  A push message is sliced at the server ranges
(SliceKOFVMessage, src/system/message.h:107-147), each slice is encoded by the
sender's per-(stream, server) RemoteNode (executor.cc:131-146) and delivered to
its server, whose per-(server, stream) RemoteNode decodes it -- all inside
libpsf (psf_router_*), one native call per phase of a step.

The only data-path collective is the cross-range spill: slices whose server
lives on another rank travel in one all-to-all-v per step (RCCL over xGMI with
the "nccl" backend; gloo for the CPU tests).  What travels is the ENCODED
slice -- the reference's wire frames [Task][key][value...] (van.cc:122-191),
laid out by libpsf in one gather launch and rebuilt on the receiver -- so
KEY_CACHING hits and FIXING_FLOAT's 4x shrink cut the xGMI bytes too.  Per
step the host does one small all-to-all of segment sizes (one device->host
read) and one all-to-all-v of bytes; no per-slice or per-frame host work.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import torch

from ._lib import check, lib

KEY_ALL = (0, (1 << 64) - 1)  # Range<Key>::All(), range.h:92-95


def even_divide(key_range, n: int, i: int):
    """Range<Key>(key_range).EvenDivide(n, i), exactly (long double)."""
    b, e = C.c_uint64(), C.c_uint64()
    check(lib().psf_range_even_divide(key_range[0], key_range[1], n, i, C.byref(b), C.byref(e)))
    return b.value, e.value


def server_ranges(nservers: int, key_range=KEY_ALL):
    """The key ranges of servers 0..nservers-1 (manager.cc:36-37 + assigner.h:21)."""
    return [even_divide(key_range, nservers, g) for g in range(nservers)]


def server_rank(server: int, nservers: int, world: int) -> int:
    """The rank hosting `server`: contiguous blocks of servers per rank."""
    return server * world // nservers


def _bounds(ranges: Sequence):
    n = len(ranges)
    for i in range(1, n):
        if ranges[i - 1][1] != ranges[i][0]:
            raise ValueError("ranges must be contiguous (message.h:120)")
    return (C.c_uint64 * (n + 1))(*([r[0] for r in ranges[:1]] + [r[1] for r in ranges]))


def slice_message(ctx, msg, ranges: Sequence, key_bytes: int = 8):
    """SliceKOFVMessage: returns one Message per range, or None where the range
    misses the message's key range (the reference marks those invalid and
    does not send them)."""
    return slice_messages(ctx, [msg], ranges, key_bytes)[0]


def slice_messages(ctx, msgs, ranges: Sequence, key_bytes: int = 8):
    """slice_message for many messages with one device synchronisation;
    returns one list per message."""
    from .filter import Message
    n, M = len(ranges), len(msgs)
    bounds = _bounds(ranges)
    outs = (C.c_void_p * (n * M))()
    valid = (C.c_int * (n * M))()
    hs = (C.c_void_p * M)(*[m.h.value for m in msgs])
    check(lib().psf_msgs_slice(ctx.h, hs, M, bounds, n, key_bytes, outs, valid))
    res = []
    for j, msg in enumerate(msgs):
        row = []
        for i in range(n):
            m = Message(_handle=C.c_void_p(outs[j * n + i]), _refs=msg._refs)
            row.append(m if valid[j * n + i] else None)
        res.append(row)
    return res


def w_channel(m) -> int:
    ch = C.c_int32()
    check(lib().psf_msg_key_channel(m.h, C.byref(ch)))
    return ch.value


class SpillExchange:
    """The collective side of the cross-range spill: one all-to-all of the
    2 x world segment sizes (meta, payload) and one all-to-all-v of the
    bytes, over `group`.

    `device` is where the buffers live ("cuda:k" with RCCL; with gloo, device
    buffers are staged through host memory, which is what the CPU tests and
    the single-GPU gloo rehearsals use)."""

    def __init__(self, ctx, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.ctx = ctx
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device if device is not None else (
            f"cuda:{ctx.device}" if ctx.device >= 0 else "cpu")
        self.staged = dist.get_backend(group) == "gloo" and str(self.device).startswith("cuda")
        self.wire = "cpu" if self.staged else self.device
        self.bytes_sent = 0
        self._send = torch.empty(0, dtype=torch.uint8, device=self.device)
        self._recv = torch.empty(0, dtype=torch.uint8, device=self.wire)

    def sizes(self, sizes) -> List[int]:
        """all-to-all of this rank's 2 x world segment sizes; returns what
        every source reports for this rank (the step's one device->host read)."""
        t = torch.tensor(list(sizes), dtype=torch.int64)
        out = torch.empty_like(t)
        if self.wire != "cpu":
            t, out = t.to(self.wire, non_blocking=True), out.to(self.wire)
        self.dist.all_to_all_single(out, t, group=self.group)
        return out.cpu().tolist()

    def send_buffer(self, nbytes: int) -> torch.Tensor:
        if self._send.numel() < nbytes:
            self._send = torch.empty(max(nbytes, 2 * self._send.numel()), dtype=torch.uint8, device=self.device)
        return self._send

    def move(self, sizes, sizes_in, after_send=None) -> torch.Tensor:
        """The all-to-all-v of the filled send buffer; `after_send` (device
        work that does not touch the buffers) is queued while it runs.
        Returns the receive buffer on the context's device."""
        W = self.world
        in_splits = [sizes[2 * r] + sizes[2 * r + 1] for r in range(W)]
        out_splits = [sizes_in[2 * s] + sizes_in[2 * s + 1] for s in range(W)]
        self.bytes_sent += sum(in_splits) - in_splits[self.rank]
        nout = sum(out_splits)
        if self._recv.numel() < nout:
            self._recv = torch.empty(max(nout, 2 * self._recv.numel()), dtype=torch.uint8, device=self.wire)
        send = self._send[:sum(in_splits)]
        recv = self._recv[:nout]
        if self.staged:
            self.ctx.sync()
            send = send.cpu()
        work = self.dist.all_to_all_single(recv, send, out_splits, in_splits, group=self.group, async_op=True)
        if after_send is not None:
            after_send()
        work.wait()
        return recv.to(self.device) if self.staged else recv

    def exchange(self, msgs, dest: List[int], server: List[int]):
        """Message-level spill (psf_spill_pack / fill / unpack): send msgs[i]
        to rank dest[i] addressed to server server[i]; returns (received
        messages, their servers)."""
        from .filter import Message
        L, W, n = lib(), self.world, len(msgs)
        sizes = (C.c_int64 * (2 * W))()
        plan = C.c_void_p()
        check(L.psf_spill_pack(self.ctx.h, (C.c_void_p * n)(*[m.h.value for m in msgs]),
                               (C.c_int * n)(*dest), (C.c_int * n)(*server), n, W, sizes, C.byref(plan)))
        try:
            sizes_in = self.sizes(sizes)
            buf = self.send_buffer(sum(sizes))
            check(L.psf_spill_fill(plan, C.c_void_p(buf.data_ptr())))
        finally:
            L.psf_spill_destroy(plan)
        recv = self.move(list(sizes), sizes_in)
        cap = max(1, sum(sizes_in[0::2]) // 24)  # a record is >= 24 bytes
        outs = (C.c_void_p * cap)()
        servers = (C.c_int * cap)()
        got = C.c_int()
        check(L.psf_spill_unpack(self.ctx.h, C.c_void_p(recv.data_ptr()), W, (C.c_int64 * (2 * W))(*sizes_in),
                                 outs, servers, cap, C.byref(got)))
        res = [Message(_handle=C.c_void_p(outs[i])) for i in range(got.value)]
        return res, [servers[i] for i in range(got.value)]


class NativeExchange:
    """libpsf's own exchange of the node's ranks (psf_exchange_*, exchange.h):
    per step the Task records of the slices for other ranks go through a host
    shared-memory mailbox and their data frames device to device -- RCCL
    point-to-point over xGMI (``transport="rccl"``, one communicator made
    here, once) or the mailbox itself (``"host"``: several ranks on one GPU,
    or host-only contexts).  A PushRouter with one runs whole steps in one
    native call at any world size (psf_router_step): no Python per step, no
    device->host read of sizes or records.  `group` is only used here, to
    hand rank 0's mailbox name and RCCL id to the other ranks."""

    def __init__(self, ctx, h, rank: int, world: int, transport: str):
        self.ctx, self.h, self.rank, self.world, self.transport = ctx, h, rank, world, transport
        self._base = 0

    @classmethod
    def create(cls, ctx, group=None, transport: str = "rccl", meta_cap: int = 0, host_cap: int = 0):
        import os
        import secrets

        import torch.distributed as dist

        from ._lib import PSF_EXCHANGE_HOST, PSF_EXCHANGE_RCCL
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        t = {"rccl": PSF_EXCHANGE_RCCL, "host": PSF_EXCHANGE_HOST}[transport]
        obj = [None]
        if rank == 0:
            uid = b""
            if t == PSF_EXCHANGE_RCCL:
                buf = (C.c_uint8 * 128)()
                check(lib().psf_exchange_unique_id(buf, 128))
                uid = bytes(buf)
            obj = [(f"psf_ex_{os.getpid()}_{secrets.token_hex(6)}", uid)]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        name, uid = obj[0]
        idbuf = (C.c_uint8 * 128).from_buffer_copy(uid) if uid else None
        h = C.c_void_p()
        check(lib().psf_exchange_create(ctx.h, rank, world, name.encode(), t, idbuf, meta_cap, host_cap, C.byref(h)))
        return cls(ctx, h, rank, world, transport)

    def __del__(self):
        try:
            if self.h:
                lib().psf_exchange_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def stats(self) -> dict:
        out = (C.c_int64 * 3)()
        check(lib().psf_exchange_stats(self.h, out))
        return {"bytes_sent": out[0], "steps": out[1], "wait_s": out[2] / 1e9}

    def data_stats(self) -> dict:
        """the data path: bytes handed to ncclSend and the send calls made
        (rccl), bytes the runtime copied instead (the self slice, or the
        host mailbox), and whether a step failed on this rank"""
        out = (C.c_int64 * 4)()
        check(lib().psf_exchange_data_stats(self.h, out))
        return {"rccl_bytes": out[0], "rccl_sends": out[1], "copied_bytes": out[2], "failed": bool(out[3])}

    @property
    def bytes_sent(self) -> int:
        """records + data posted for other ranks since the last reset (set to 0)"""
        return self.stats()["bytes_sent"] - self._base

    @bytes_sent.setter
    def bytes_sent(self, v: int) -> None:
        self._base = self.stats()["bytes_sent"] - v


class PushRouter:
    """The multi-server push path of one rank (libpsf
    psf_router_*): every local stream's message is sliced at the `ranges` of S
    servers, each slice encoded by the sender's per-(stream, server) node;
    slices whose server lives on this rank are decoded here, the others travel
    in ONE all-to-all-v per step (the cross-range spill) and are decoded by
    their server's per-stream node.  The stream id travels as the Task's
    key_channel.  `loopback` sends the local slices through the exchange too
    (a world-1 run of the RCCL path)."""

    def __init__(self, ctx, ranges, rank: int, world: int, exchange: SpillExchange = None,
                 loopback: bool = False):
        self.ctx, self.ranges, self.rank, self.world = ctx, ranges, rank, world
        self.nservers = len(ranges)
        if self.nservers < world:
            raise ValueError("need at least one server per rank")
        if (world > 1 or loopback) and exchange is None:
            raise ValueError("a spill exchange is needed")
        self.exchange, self.loopback = exchange, loopback
        h = C.c_void_p()
        check(lib().psf_router_create(ctx.h, _bounds(ranges), self.nservers, rank, world, int(loopback),
                                      C.byref(h)))
        self.h = h
        self._held = {}
        self.native = isinstance(exchange, NativeExchange)
        if self.native:
            check(lib().psf_router_set_exchange(h, exchange.h))

    def __del__(self):
        try:
            if self.h:
                lib().psf_router_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def owner(self, server: int) -> int:
        return server_rank(server, self.nservers, self.world)

    def _handles(self, streams):
        for sid, m in streams.items():
            if self._held.get(sid) is not m:  # nodes and caches refer to template buffers
                self._held[sid] = m
        msgs = list(streams.values())
        return (C.c_void_p * len(msgs))(*[m.h.value for m in msgs]), len(msgs)

    def run(self, streams, steps: int, keep_encoded=None) -> None:
        """`steps` whole steps; one native call with a NativeExchange, or at
        world 1 without loopback.  keep_encoded: None leaves the router's
        setting (psf_router_keep_encoded) as it is."""
        if self.native or (self.world == 1 and not self.loopback):
            if keep_encoded is not None:
                check(lib().psf_router_keep_encoded(self.h, int(keep_encoded)))
            hs, n = self._handles(streams)
            check(lib().psf_router_step(self.h, hs, n, steps))
            return
        for _ in range(steps):
            self.step(streams, bool(keep_encoded))

    def step(self, streams, keep_encoded: bool = False) -> None:
        """streams: {stream id: template Message (key_channel = stream id)} of
        this rank.  The decoded messages this rank's servers received are in
        results(); with keep_encoded, the encoded slices in encoded()."""
        L = lib()
        check(L.psf_router_keep_encoded(self.h, int(keep_encoded)))
        hs, n = self._handles(streams)
        if self.native or (self.world == 1 and not self.loopback):
            check(L.psf_router_step(self.h, hs, n, 1))
            return
        W = self.world
        sizes = (C.c_int64 * (2 * W))()
        check(L.psf_router_encode(self.h, hs, n, sizes))
        ex = self.exchange
        sizes_in = ex.sizes(sizes)
        buf = ex.send_buffer(sum(sizes))
        check(L.psf_router_fill(self.h, C.c_void_p(buf.data_ptr())))
        recv = ex.move(list(sizes), sizes_in, after_send=lambda: check(L.psf_router_decode_local(self.h)))
        check(L.psf_router_decode_received(self.h, C.c_void_p(recv.data_ptr()),
                                           (C.c_int64 * (2 * W))(*sizes_in)))

    def set_store(self, kvmap) -> None:
        """The KV map (filter.KVMap) answering the pulls addressed to this
        rank's servers (KVMap::GetValue, kv_map.h:69-77)."""
        self._store = kvmap
        check(lib().psf_router_set_store(self.h, kvmap.h if kvmap is not None else None))

    def pull(self, requests, steps: int = 1, keep_encoded=None) -> None:
        """`steps` pulls of every request stream's keys ({stream id: template
        Message with request=True, push=False, keys only}) from the server
        group: sliced per server, answered from each server's store, merged
        back in key order (pulled()).  One native call with a NativeExchange
        or at world 1; else the three phases around the SpillExchange's
        all-to-all-v."""
        L = lib()
        if keep_encoded is not None:
            check(L.psf_router_keep_encoded(self.h, int(keep_encoded)))
        hs, n = self._handles(requests)
        if self.native or (self.world == 1 and not self.loopback):
            check(L.psf_router_pull(self.h, hs, n, steps))
            return
        W, ex = self.world, self.exchange
        for _ in range(steps):
            sizes = (C.c_int64 * (2 * W))()
            check(L.psf_router_pull_encode(self.h, hs, n, sizes))
            sizes_in = ex.sizes(sizes)
            buf = ex.send_buffer(sum(sizes))
            check(L.psf_router_fill(self.h, C.c_void_p(buf.data_ptr())))
            recv = ex.move(list(sizes), sizes_in)
            out = (C.c_int64 * (2 * W))()
            check(L.psf_router_pull_serve(self.h, C.c_void_p(recv.data_ptr()), (C.c_int64 * (2 * W))(*sizes_in),
                                          out))
            back_in = ex.sizes(out)
            buf = ex.send_buffer(sum(out))
            check(L.psf_router_fill(self.h, C.c_void_p(buf.data_ptr())))
            recv = ex.move(list(out), back_in)
            check(L.psf_router_pull_finish(self.h, C.c_void_p(recv.data_ptr()), (C.c_int64 * (2 * W))(*back_in)))

    def pulled(self):
        """[(stream, Message)] of the last pull: the stream's keys and one
        float array of the pulled values in key order."""
        from .filter import Message
        L = lib()
        out = []
        for i in range(check(L.psf_router_num_pulled(self.h))):
            st, h = C.c_int32(), C.c_void_p()
            check(L.psf_router_pulled(self.h, i, C.byref(st), C.byref(h)))
            out.append((st.value, Message(_handle=h)))
        return out

    def host_stats(self, reset: bool = False) -> dict:
        """Host phase timers since the last reset: encodes, and seconds spent
        inside the encodes and the decodes (blocked time included)."""
        out = (C.c_int64 * 3)()
        check(lib().psf_router_host_stats(self.h, out))
        if reset:
            check(lib().psf_router_host_stats_reset(self.h))
        return {"steps": out[0], "encode_s": out[1] / 1e9, "decode_s": out[2] / 1e9}

    def results(self):
        """[(server, decoded Message)] of the last step."""
        from .filter import Message
        L = lib()
        out = []
        for i in range(check(L.psf_router_num_results(self.h))):
            s, h = C.c_int(), C.c_void_p()
            check(L.psf_router_result(self.h, i, C.byref(s), C.byref(h)))
            out.append((s.value, Message(_handle=h)))
        return out

    def encoded(self):
        """[((stream, server), encoded Message)] of the last step (keep_encoded)."""
        from .filter import Message
        L = lib()
        out = []
        for i in range(check(L.psf_router_num_encoded(self.h))):
            st, s, h = C.c_int32(), C.c_int(), C.c_void_p()
            check(L.psf_router_encoded(self.h, i, C.byref(st), C.byref(s), C.byref(h)))
            out.append(((st.value, s.value), Message(_handle=h)))
        return out
